"""Per-kernel SQ timing summary from the rocprofv3 --pmc passes of
tools/gpu_sq_timing.sh (counter_collection.csv under each pass directory).

Columns, per kernel name (all launches of one bench step summed):
  us/launch   GRBM_GUI_ACTIVE / 8 XCDs / launches at 2.4 GHz (upper clock; a
              relative measure of the kernel's share, not its wall time)
  wait%       SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked on s_waitcnt / barrier)
  stall%      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (ready, issue-stalled)
  lds%        SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES   (sub-bucket of stall%)
  issue%      SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  mfma%       SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs):
              the matrix pipes' busy share of the kernel's lifetime
  and, from the second pass when present: VALU / LDS / VMEM / SALU instructions
  per wave, LDS bank-conflict cycles per LDS instruction, MFMA-VALU co-issue share.
(MI355X_MICROARCH.md: SQ_WAVE_CYCLES / WAIT_* / ACTIVE_INST_* count quad-cycles
and are compared only with each other here.)

usage: python tools/sq_timing.py <pass1_dir> [pass2_dir]
"""
import csv
import glob
import os
import sys

FAMILY = ("conv3x3_pp_kernel", "conv3x3_halo_kernel", "wgrad3x3_halo_kernel", "conv3x3_pers_kernel", "conv3x3_c64_kernel",
          "conv3x3_sg_kernel")


def load(d):
    per = {}
    if not d or not os.path.isdir(d):
        return per
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                k = per.setdefault(name, {"_ids": set()})
                k["_ids"].add(did)
                c = row["Counter_Name"]
                k[c] = k.get(c, 0.0) + float(row["Counter_Value"])
    return per


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:64]


def pct(a, b):
    return 100.0 * a / b if b else float("nan")


def main():
    p1 = load(sys.argv[1])
    p2 = load(sys.argv[2] if len(sys.argv) > 2 else None)
    rows = sorted(p1.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0.0))
    tot = sum(k.get("GRBM_GUI_ACTIVE", 0.0) for _, k in rows)
    hdr = f"{'kernel':64s} {'n':>4s} {'time%':>6s} {'us/l':>7s} {'wait%':>6s} {'stall%':>6s} {'lds%':>5s} {'issue%':>6s} {'mfma%':>6s}"
    if p2:
        hdr += f" {'valu/w':>7s} {'lds/w':>6s} {'vmem/w':>6s} {'salu/w':>6s} {'bc/lds':>6s} {'coex%':>6s}"
    print(hdr)
    fam = {}
    for name, k in rows[:45]:
        n = len(k["_ids"])
        gui = k.get("GRBM_GUI_ACTIVE", 0.0)
        xcd_cyc = gui / 8.0
        wc = k.get("SQ_WAVE_CYCLES", 0.0)
        line = (f"{short(name):64s} {n:4d} {pct(gui, tot):6.2f} {xcd_cyc / n / 2400.0:7.1f} "
                f"{pct(k.get('SQ_WAIT_ANY', 0.0), wc):6.1f} {pct(k.get('SQ_WAIT_INST_ANY', 0.0), wc):6.1f} "
                f"{pct(k.get('SQ_WAIT_INST_LDS', 0.0), wc):5.1f} {pct(k.get('SQ_ACTIVE_INST_ANY', 0.0), wc):6.1f} "
                f"{pct(k.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0), xcd_cyc * 1024):6.1f}")
        q = p2.get(name)
        if q:
            w = max(q.get("SQ_WAVES", 0.0), 1.0)
            lds = max(q.get("SQ_INSTS_LDS", 0.0), 1.0)
            g2 = q.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
            line += (f" {q.get('SQ_INSTS_VALU', 0.0) / w:7.0f} {q.get('SQ_INSTS_LDS', 0.0) / w:6.0f} "
                     f"{q.get('SQ_INSTS_VMEM', 0.0) / w:6.0f} {q.get('SQ_INSTS_SALU', 0.0) / w:6.0f} "
                     f"{q.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds:6.2f} "
                     f"{pct(q.get('SQ_VALU_MFMA_COEXEC_CYCLES', 0.0), g2 * 1024):6.1f}")
        print(line)
    for name, k in rows:
        if any(f in name for f in FAMILY):
            for c, v in k.items():
                if c != "_ids":
                    fam[c] = fam.get(c, 0.0) + v
    if fam:
        wc = fam.get("SQ_WAVE_CYCLES", 0.0)
        xc = fam.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        print(f"\n3x3 family: time% {pct(fam.get('GRBM_GUI_ACTIVE', 0.0), tot):.1f}  wait% "
              f"{pct(fam.get('SQ_WAIT_ANY', 0.0), wc):.1f}  stall% {pct(fam.get('SQ_WAIT_INST_ANY', 0.0), wc):.1f}  "
              f"lds% {pct(fam.get('SQ_WAIT_INST_LDS', 0.0), wc):.1f}  issue% "
              f"{pct(fam.get('SQ_ACTIVE_INST_ANY', 0.0), wc):.1f}  mfma% "
              f"{pct(fam.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0), xc * 1024):.1f}")


if __name__ == "__main__":
    main()
