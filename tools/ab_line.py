"""Print one A/B line from two bench.py logs (their last JSON line):
python tools/ab_line.py <label> <old.log> <new.log>"""
import json
import sys


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def main():
    label, a, b = sys.argv[1:4]
    ja, jb = last_json(a), last_json(b)
    if ja is None or jb is None:
        print(f"{label}: no JSON line ({a if ja is None else b})")
        return
    va, vb = ja["value"], jb["value"]
    print(f"{label}: old {va:.2f} ({ja['ms_per_step']:.3f} ms)  new {vb:.2f} ({jb['ms_per_step']:.3f} ms)  "
          f"{100.0 * (vb / va - 1):+.2f} %")


if __name__ == "__main__":
    main()
