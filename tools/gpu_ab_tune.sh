#!/bin/bash
# Same-box A/B of one library tuning key: bench.py with KEY=A vs KEY=B, interleaved,
# 2 reps.  usage: bash tools/gpu_ab_tune.sh KEY A B MODELS [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$1; A=$2; B=$3; MODELS=$4; shift 4
O=$R/gpurun_out/abt_$K
mkdir -p $O
cd $R
for rep in 1 2; do
  for m in $MODELS; do
    for v in $A $B; do
      timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline --no-roofline \
        --tune $K=$v "$@" > $O/${m}_${v}_$rep.log 2>&1 || { echo FAIL $m $v; tail -30 $O/${m}_${v}_$rep.log; exit 1; }
      echo "$m $K=$v rep$rep: $(tail -1 $O/${m}_${v}_$rep.log | cut -c1-100)"
    done
  done
done
