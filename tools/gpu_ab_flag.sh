#!/bin/bash
# Same-box A/B of one engine switch: bench.py with NAME=1 vs NAME=0, both models,
# interleaved, 2 reps.  usage: bash tools/gpu_ab_flag.sh NAME [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
F=$1; shift
O=$R/gpurun_out/ab_$F
mkdir -p $O
cd $R
for rep in 1 2; do
  for m in unet vae; do
    for v in 1 0; do
      timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline --no-roofline \
        --engine-flag $F=$v "$@" > $O/${m}_${v}_$rep.log 2>&1 || { echo FAIL $m $v; tail -30 $O/${m}_${v}_$rep.log; exit 1; }
      echo "$m $F=$v rep$rep: $(tail -1 $O/${m}_${v}_$rep.log | cut -c1-120)"
    done
  done
done
