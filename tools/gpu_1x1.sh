set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python -u tools/gemm1x1_bench.py --check > $O/g1_stream.log 2>&1 || { echo FAIL; tail -30 $O/g1_stream.log; exit 1; }
grep -v amdgpu.ids $O/g1_stream.log
VU_GEMM_STREAM=0 timeout -k 10 200 python -u tools/gemm1x1_bench.py > $O/g1_v2.log 2>&1 || { echo FAIL; tail -30 $O/g1_v2.log; exit 1; }
grep -v amdgpu.ids $O/g1_v2.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/pytest_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" $O/pytest_kernels.log | head -30; exit 1; }
tail -2 $O/pytest_kernels.log
