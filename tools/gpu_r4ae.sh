#!/bin/bash
# round 4: c64 statistics computed during the next group's taps: tests + bench A/B + c64 kernel durations
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4ae
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_production_parity.py -k "c64 or production or every" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_lib.sh old new "unet" || exit 1
cd /tmp
for v in old new; do
  VU_LIB_PATH=$R/ab/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o p -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$v.log 2>&1 || { echo PROF_FAIL; exit 1; }
  echo "== $v"; find $O/prof_$v -name "*kernel_stats.csv" -exec grep -h c64 {} \; | cut -d, -f1-4
  rm -rf $O/prof_$v
done
