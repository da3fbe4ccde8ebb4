#!/bin/bash
# round 4: 256x256 v2 weight-gradient tiles (VU_TUNE_W2_BIG): tests + 1x1/ConvT table A/B + bench A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4w
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "big_tiles or conv_transpose or conv1x1" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for t in 0 1; do
  timeout -k 10 200 python -u tools/gemm1x1_bench.py --tune 28=$t > $O/g1_${t}_$rep.log 2>&1 || { echo G1_FAIL; tail -20 $O/g1_${t}_$rep.log; exit 1; }
done; done
echo "== W2_BIG=0"; grep -E "wgrad|TOTAL" $O/g1_0_1.log; echo "== W2_BIG=1"; grep -E "wgrad|TOTAL" $O/g1_1_1.log
grep TOTAL $O/g1_*_2.log
