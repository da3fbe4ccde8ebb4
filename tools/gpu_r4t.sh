#!/bin/bash
# round 4: v7 for the 832-column decoder gradient; v6 grid cap for the 128^2 64->64 encoder layers
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4t
mkdir -p $O
cd $R
for v in old new; do
  VU_LIB_PATH=$R/ab/lib_$v.so timeout -k 10 200 python -u tools/enc_bench.py > $O/enc_$v.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/enc_$v.log
done
for t in 256 128; do
  VU_LIB_PATH=$R/ab/lib_new.so timeout -k 10 200 python -u tools/enc_bench.py --tune 11=$t > $O/enc_v6_$t.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc_v6_$t.log; exit 1; }
  echo "== v6 cap $t"; grep -E "layer1|TOTAL" $O/enc_v6_$t.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "v7 or sg or small" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_lib.sh old new "vae"
