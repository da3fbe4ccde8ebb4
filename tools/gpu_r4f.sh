#!/bin/bash
# round 4: column-major halo wgrad walk + FastDiv / image-conv prefetch (tests + A/B vs HEAD build),
# encoder weight-gradient split-K cap sweep
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad or fwd_dgrad or image or stream or v5" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for ws in 0 8 4 2; do
  timeout -k 10 200 python -u tools/enc_bench.py --wsplit $ws > $O/enc_ws$ws.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc_ws$ws.log; exit 1; }
  echo "wsplit=$ws"; grep -v amdgpu.ids $O/enc_ws$ws.log | cut -c1-150
done
bash tools/gpu_ab_lib.sh old new "unet"
