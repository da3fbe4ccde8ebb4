#!/bin/bash
# round 4: linear-gather DMA pointers in the v2 weight gradient (+ optional 256x256 tiles)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4x
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "big_tiles or conv_transpose or conv1x1 or wgrad" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in old new; do
  VU_LIB_PATH=$R/ab/lib_$v.so timeout -k 10 200 python -u tools/gemm1x1_bench.py > $O/g1_$v.log 2>&1 || { echo G1_FAIL; tail -20 $O/g1_$v.log; exit 1; }
  echo "== $v"; grep -E "wgrad|TOTAL" $O/g1_$v.log
done
VU_LIB_PATH=$R/ab/lib_new.so timeout -k 10 200 python -u tools/gemm1x1_bench.py --tune 28=1 > $O/g1_new_big.log 2>&1 || { echo G1_FAIL; exit 1; }
echo "== new + W2_BIG"; grep -E "wgrad|TOTAL" $O/g1_new_big.log
bash tools/gpu_ab_lib.sh old new "unet vae"
