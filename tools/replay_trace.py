"""Per-step kernel census of a rocprofv3 kernel trace (csv), split at the
AdamW launch that ends every training step: launch counts per step for the
library's own kernels, ATen kernels and runtime copies/fills, and the full
launch list of the last step (a graph replay when the bench ran with
--graph: its warm-up and capture steps come first and show up as the
irregular leading rows).

usage: python tools/replay_trace.py p_kernel_trace.csv [--list-last]
"""
import csv
import re
import sys
from collections import Counter


def short(name):
    n = re.sub(r"\(anonymous namespace\)::|void |at::native::", "", name)
    return n.split("(")[0][:90]


def kind(name):
    if name.startswith("__amd_rocclr"):
        return "runtime"
    if "at::native" in name or name.startswith("void at::") or "at::" in name.split("(")[0]:
        return "aten"
    return "library"


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "mt_adamw" in r["Kernel_Name"]]
    if not ends:
        sys.exit("no AdamW launch in the trace")
    steps, s0 = [], 0
    for e in ends:
        steps.append(rows[s0:e + 1])
        s0 = e + 1
    print(f"{len(steps)} steps (each ends at the AdamW launch); trailing {len(rows) - s0} launches after the last")
    print("step  launches  library  aten  runtime   gpu_ms(sum of kernel durations)")
    for i, st in enumerate(steps):
        c = Counter(kind(r["Kernel_Name"]) for r in st)
        ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st) / 1e6
        print(f"{i:4d} {len(st):9d} {c['library']:8d} {c['aten']:5d} {c['runtime']:8d}   {ms:8.3f}")
    last = steps[-1]
    print("\nnon-library launches of the last step:")
    for r in last:
        if kind(r["Kernel_Name"]) != "library":
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"  {kind(r['Kernel_Name']):8s} {d:8.1f} us  grid={r['Grid_Size_X']:>8s}  {short(r['Kernel_Name'])}")
    if "--list-last" in sys.argv:
        print("\nall launches of the last step:")
        for r in last:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"  {d:8.1f} us  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
