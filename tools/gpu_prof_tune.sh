#!/bin/bash
# rocprofv3 kernel stats of a bench model with one library tuning key at two values
# usage: bash tools/gpu_prof_tune.sh KEY A B [model]  -> gpurun_out/proft_KEY/{A,B}_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$1; A=$2; B=$3; M=${4:-unet}
O=$R/gpurun_out/proft_$K
mkdir -p $O
cd /tmp
for v in $A $B; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o p -- python3 -u $R/bench.py --model $M --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --tune $K=$v > $O/run_$v.log 2>&1 || { echo PROF_FAIL $v; tail -20 $O/run_$v.log; exit 1; }
  find $O/p$v -name "*kernel_stats.csv" -exec cp {} $O/${v}_kernel_stats.csv \;
  rm -rf $O/p$v
done
ls $O
