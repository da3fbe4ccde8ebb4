"""Per-kernel L2 hit rate and TCC request counts from one rocprofv3 PMC pass
(`--pmc TCC_HIT_sum TCC_MISS_sum`), for the streaming GEMMs whose LDS fill
rate is below the L2 rate (MI355X_MICROARCH.md "Indexed rows": 66-73 GB/s per
CU from L2, 23-33 from the Infinity Cache / HBM).

usage: python tools/pmc_l2.py <pmc_dir> [top]
"""
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    kern = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = re.sub(r"\(anonymous namespace\)::|void ", "", row["Kernel_Name"]).split("(")[0][:60]
                k = kern.setdefault(name, {"hit": 0.0, "miss": 0.0, "ids": set()})
                k["ids"].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
                if row["Counter_Name"].startswith("TCC_HIT"):
                    k["hit"] += float(row["Counter_Value"])
                elif row["Counter_Name"].startswith("TCC_MISS"):
                    k["miss"] += float(row["Counter_Value"])
    rows = sorted(kern.items(), key=lambda kv: -(kv[1]["hit"] + kv[1]["miss"]))
    print(f"{'launches':>8s} {'req/launch(M)':>14s} {'hit%':>6s}  kernel")
    for name, k in rows[:top]:
        n = max(len(k["ids"]), 1)
        req = k["hit"] + k["miss"]
        print(f"{n:8d} {req / n / 1e6:14.3f} {100 * k['hit'] / max(req, 1):6.1f}  {name}")


if __name__ == "__main__":
    main()
