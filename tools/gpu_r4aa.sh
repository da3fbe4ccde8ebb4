#!/bin/bash
# round 4: 64-input-channel wide no-stats convs as v6 column slices: tests + per-layer dgrad A/B + bench A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4aa
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "c64" tests/test_gpu_production_parity.py > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in old new; do
  VU_LIB_PATH=$R/ab/lib_$v.so timeout -k 10 200 python -u tools/conv_bench.py --only dgrad --layers up4.1,up4.2,inc.2 > $O/cb_$v.log 2>&1 || { echo CB_FAIL; tail -20 $O/cb_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu $O/cb_$v.log
done
bash tools/gpu_ab_lib.sh old new "unet vae"
