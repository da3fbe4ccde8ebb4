"""Per-kernel time difference of two rocprofv3 kernel_stats.csv files (us per
step, given the step count of each run).  usage: prof_diff.py A.csv B.csv [steps]"""
import csv
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"].replace("(anonymous namespace)::", "")
        n = n.split("(")[0] if not n.startswith("void ") else n[5:].split("(")[0]
        d = out.setdefault(n, [0, 0.0])
        d[0] += int(r["Calls"])
        d[1] += float(r["TotalDurationNs"])
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 13.0
keys = sorted(set(a) | set(b), key=lambda k: -abs(a.get(k, [0, 0])[1] - b.get(k, [0, 0])[1]))
ta = sum(v[1] for v in a.values()) / steps / 1e3
tb = sum(v[1] for v in b.values()) / steps / 1e3
print(f"total us/step: A {ta:9.1f}  B {tb:9.1f}  diff {ta - tb:+8.1f}")
for k in keys[:30]:
    ca, sa = a.get(k, [0, 0.0])
    cb, sb = b.get(k, [0, 0.0])
    print(f"{(sa - sb) / steps / 1e3:+9.1f}  A {sa / steps / 1e3:8.1f} ({ca / steps:5.1f}x)  B {sb / steps / 1e3:8.1f} ({cb / steps:5.1f}x)  {k[:90]}")
