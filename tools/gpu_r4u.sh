#!/bin/bash
# round 4: v4 split-K on 64-column tiles (832-column decoder gradient) vs v7; v6 at one tile per CU
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4u
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "splitk or c64 or v7 or small" tests/test_gpu_production_parity.py > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/enc_bench.py > $O/enc_new.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc_new.log; exit 1; }
timeout -k 10 200 python -u tools/enc_bench.py --tune 16=2 > $O/enc_v7m2.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc_v7m2.log; exit 1; }
echo "== new (v4 split 64)"; grep -E "layer1|dec1|TOTAL" $O/enc_new.log
echo "== v7 mode 2"; grep -E "dec1|TOTAL" $O/enc_v7m2.log
bash tools/gpu_ab_lib.sh old new "vae"
