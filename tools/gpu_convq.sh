# 3x3 fwd/dgrad layer timings + kernel/parity tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 150 python -u tools/conv_bench.py --only ${ONLY:-fwd,dgrad} > $O/convq.log 2>&1 || { echo FAIL; tail -20 $O/convq.log; exit 1; }
grep -v amdgpu.ids $O/convq.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pt_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" $O/pt_kernels.log | head -30; exit 1; }
tail -1 $O/pt_kernels.log
