# v5 (persistent short-K GEMM): parity tests, then the per-call bench with v5 off / on
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "v5 or conv1x1 or conv_transpose or stream" > gpurun_out/v5_tests.log 2>&1
timeout -k 10 120 python tools/gemm1x1_bench.py --check --tune 10=0 > gpurun_out/v5_off.log 2>&1
timeout -k 10 120 python tools/gemm1x1_bench.py --check > gpurun_out/v5_on.log 2>&1
