# v5 persistent + fp8 kernels: parity tests, per-layer timing (v5 on / off), fp8 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fp8.py -q -x --timeout 100 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pt.log | head -20; tail -30 $O/pt.log; exit 1; }
tail -2 $O/pt.log
timeout -k 10 200 python -u tools/conv_bench.py --check --only fwd,dgrad > $O/conv_v5.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_v5.log; exit 1; }
grep -v amdgpu.ids $O/conv_v5.log
timeout -k 10 200 python -u tools/conv_bench.py --only fwd,dgrad --tune 1=0 > $O/conv_v5off.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_v5off.log; exit 1; }
grep -v amdgpu.ids $O/conv_v5off.log
timeout -k 10 300 python -u tools/fp8_bench.py --batch 2 --json $O/fp8_bench.json > $O/fp8_bench.log 2>&1 || { echo FP8_FAIL; tail -30 $O/fp8_bench.log; exit 1; }
grep -v amdgpu.ids $O/fp8_bench.log
