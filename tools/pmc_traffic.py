"""HBM traffic per launch of the 3x3 conv kernels from rocprofv3 PMC passes
(MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced stream -> x2; WRITE_SIZE
is exact for 16-byte stores).  Reads the counter_collection CSVs of two
separate passes (`--pmc FETCH_SIZE`, `--pmc WRITE_SIZE`, tools/gpu_evidence.sh) and
writes profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import sys

FAMILY = ("conv3x3_pp_kernel", "conv3x3_halo_kernel", "wgrad3x3_halo_kernel", "conv3x3_pers_kernel", "conv3x3_c64_kernel",
          "conv3x3_sg_kernel")


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Kernel_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    return per


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")

    def fam(name):
        return any(k in name for k in FAMILY)
    kern = {}
    for (did, name), v in fetch.items():
        k = kern.setdefault(name, {"launches": 0, "fetch_kb": 0.0, "write_kb": 0.0, "wlaunches": 0})
        k["launches"] += 1
        k["fetch_kb"] += v
    for (did, name), v in write.items():
        k = kern.setdefault(name, {"launches": 0, "fetch_kb": 0.0, "write_kb": 0.0, "wlaunches": 0})
        k["wlaunches"] += 1
        k["write_kb"] += v
    per_kernel = {}
    tot_b, tot_n = 0.0, 0
    for name, k in sorted(kern.items(), key=lambda kv: -(kv[1]["fetch_kb"] + kv[1]["write_kb"])):
        n = max(k["launches"], 1)
        rd = 2.0 * k["fetch_kb"] * 1024 / n
        wr = k["write_kb"] * 1024 / max(k["wlaunches"], 1)
        per_kernel[name] = {"launches": k["launches"], "read_bytes_per_launch": rd,
                            "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr}
        if fam(name):
            tot_b += (rd + wr) * n
            tot_n += n
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes over "
                     "`bench.py --steps 1 --warmup 1`; bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024",
           "family": list(FAMILY),
           "conv3x3_hbm_bytes_per_launch": tot_b / tot_n if tot_n else None,
           "conv3x3_launches": tot_n,
           "per_kernel": dict(list(per_kernel.items())[:40])}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}))


if __name__ == "__main__":
    main()
