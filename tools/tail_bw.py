"""Achieved HBM bandwidth per kernel: PMC bytes per launch (tools/pmc_traffic.py
json, FETCH_SIZE x2 + WRITE_SIZE) / rocprofv3 --stats average duration of the
same kernel, sorted by time per step.  VERDICT r3 item 6 asks >= 4.8 TB/s
(0.6 of 8) for the memory-bound tail of config 2.

usage: python tools/tail_bw.py pmc_traffic.json kernel_stats.csv [steps] [top]
"""
import csv
import json
import re
import sys


def short(name):
    return re.sub(r"\(anonymous namespace\)::|void |at::native::", "", name).split("(")[0][:64]


def main():
    pmc = json.load(open(sys.argv[1]))["per_kernel"]
    stats = {r["Name"]: r for r in csv.DictReader(open(sys.argv[2]))}
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 13
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    rows = []
    for name, v in pmc.items():
        st = stats.get(name)
        if st is None:
            continue
        avg_ns = float(st["AverageNs"])
        per_step_us = float(st["TotalDurationNs"]) / steps / 1e3
        rows.append((per_step_us, v["hbm_bytes_per_launch"] / avg_ns / 1e3, v["read_bytes_per_launch"] / 1e6,
                     v["write_bytes_per_launch"] / 1e6, avg_ns / 1e3, int(st["Calls"]), short(name)))
    rows.sort(reverse=True)
    print(f"{'us/step':>8s} {'TB/s':>6s} {'frac8':>6s} {'readMB':>8s} {'writeMB':>8s} {'avg_us':>8s} {'calls':>6s}  kernel")
    for t, bw, r, w, a, n, k in rows[:top]:
        print(f"{t:8.1f} {bw:6.2f} {bw / 8:6.3f} {r:8.1f} {w:8.1f} {a:8.1f} {n:6d}  {k}")


if __name__ == "__main__":
    main()
