#!/bin/bash
# rocprofv3 kernel stats of the UNet bench with two library builds (A/B of a
# compile-time change): ab/lib_<A>.so vs ab/lib_<B>.so -> gpurun_out/prof_so/<v>_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_so
mkdir -p $O
cd /tmp
for v in "$@"; do
  cp $R/ab/lib_$v.so $R/vaeunet_amd/libvaeunet_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o p -- python3 -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/run_$v.log 2>&1 || { echo PROF_FAIL $v; exit 1; }
  find $O/p$v -name "*kernel_stats.csv" -exec cp {} $O/${v}_kernel_stats.csv \;
  rm -rf $O/p$v
done
ls $O
