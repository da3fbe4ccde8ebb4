set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread ${PYT_ARGS:-} > $O/pytest_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" $O/pytest_kernels.log | head -30; tail -30 $O/pytest_kernels.log; exit 1; }
tail -3 $O/pytest_kernels.log
