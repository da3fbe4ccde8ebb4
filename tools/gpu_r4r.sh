#!/bin/bash
# round 4: c64 butterfly statistics: tests, per-layer A/B (fwd of the two 64->64 layers), UNet bench A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4r
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "c64 or bn or stats" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for v in old new; do
  VU_LIB_PATH=$R/ab/lib_$v.so timeout -k 10 200 python -u tools/conv_bench.py --only fwd,dgrad --layers inc.2,up4.2 > $O/cb_${v}_$rep.log 2>&1 || { echo CB_FAIL; tail -20 $O/cb_${v}_$rep.log; exit 1; }
  echo "== $v rep$rep"; grep -v amdgpu.ids $O/cb_${v}_$rep.log | tail -6
done; done
bash tools/gpu_ab_lib.sh old new "unet"
