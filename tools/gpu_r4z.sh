#!/bin/bash
# round 4: packed-fp32 BN statistics in the ping-pong epilogue: tests, per-layer fwd A/B (graph-timed), bench A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4z
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "pingpong or splitk or halo or c64" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for v in old new; do
  VU_LIB_PATH=$R/ab/lib_$v.so timeout -k 10 200 python -u tools/conv_bench.py --only fwd,fwdnostats > $O/cb_${v}_$rep.log 2>&1 || { echo CB_FAIL; tail -20 $O/cb_${v}_$rep.log; exit 1; }
  echo "== $v rep$rep"; grep TOTAL $O/cb_${v}_$rep.log
done; done
bash tools/gpu_ab_lib.sh old new "unet"
