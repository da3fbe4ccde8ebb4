#!/bin/bash
# round 4: L2 hit rate + SQ wait of the 1x1 / ConvT kernels (tools/gemm1x1_bench.py, 3 reps)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4v
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_l2 -o l -- python -u $R/tools/gemm1x1_bench.py --reps 3 > $O/pmc_l2.log 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_l2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/pmc_sq -o s -- python -u $R/tools/gemm1x1_bench.py --reps 3 > $O/pmc_sq.log 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_sq.log; exit 1; }
cd $R
python tools/pmc_l2.py $O/pmc_l2 40 > $O/l2.txt && cat $O/l2.txt
python - <<'PY'
import csv, glob, collections, re
R = "gpurun_out/r4v/pmc_sq"
k = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for fn in glob.glob(R + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        name = re.sub(r"\(anonymous namespace\)::|void ", "", row["Kernel_Name"]).split("(")[0][:60]
        k[name][row["Counter_Name"]] += float(row["Counter_Value"])
        n[name].add(row.get("Dispatch_Id"))
for name, c in sorted(k.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0))[:12]:
    w = max(c.get("SQ_WAVES", 1), 1)
    print(f"{name:60s} waves/launch {w/len(n[name]):8.0f} wait_any/busy {c.get('SQ_WAIT_ANY',0)/max(c.get('SQ_BUSY_CYCLES',1),1):6.2f} "
          f"VALU/wave {c.get('SQ_INSTS_VALU',0)/w:8.0f} SALU/wave {c.get('SQ_INSTS_SALU',0)/w:8.0f} LDS/wave {c.get('SQ_INSTS_LDS',0)/w:8.0f}")
PY
rm -rf $O/pmc_l2 $O/pmc_sq
