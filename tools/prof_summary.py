"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_stats.csv) into a
per-kernel stats table (calls, total/avg ns, % of GPU time).

usage: python tools/prof_summary.py <run_results.db | *_kernel_stats.csv> [steps]
"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    return [(n, int(k), float(t)) for n, k, t in
            c.execute("select name, count(*), sum(duration) from kernels group by name")]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])))
    return out


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    print("Name,Calls,TotalDurationNs,AverageNs,Percentage" + (",MsPerStep" if steps else ""))
    for n, k, t in rows:
        line = f'"{n}",{k},{t:.0f},{t / k:.1f},{100 * t / tot:.2f}'
        if steps:
            line += f",{t / steps / 1e6:.4f}"
        print(line)
    if steps:
        print(f"# total GPU kernel time {tot / 1e6:.2f} ms over {steps} steps = {tot / steps / 1e6:.3f} ms/step")


if __name__ == "__main__":
    main()
