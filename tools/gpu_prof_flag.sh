#!/bin/bash
# rocprofv3 kernel stats of the UNet bench with an engine switch on and off
# usage: bash tools/gpu_prof_flag.sh NAME [model]  -> gpurun_out/prof_NAME/{on,off}_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
F=$1; M=${2:-unet}
O=$R/gpurun_out/prof_$F
mkdir -p $O
cd /tmp
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o p -- python3 -u $R/bench.py --model $M --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --engine-flag $F=$v > $O/run_$v.log 2>&1 || { echo PROF_FAIL $v; tail -20 $O/run_$v.log; exit 1; }
  find $O/p$v -name "*kernel_stats.csv" -exec cp {} $O/${v}_kernel_stats.csv \;
  rm -rf $O/p$v
done
ls $O
