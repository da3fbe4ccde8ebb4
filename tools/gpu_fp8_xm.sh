set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/t_fp8.log 2>&1
timeout -k 10 300 python -u tools/fp8_bench.py --json gpurun_out/fp8_pp.json > gpurun_out/fp8_pp.log 2>&1
timeout -k 10 300 python -u tools/fp8_bench.py --no-bf16 --tune 21=0 > gpurun_out/fp8_pers.log 2>&1
