set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest tests/test_gpu_production_parity.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r4a/prod.log 2>&1 || { echo PROD_FAIL; tail -30 gpurun_out/r4a/prod.log; exit 1; }
tail -3 gpurun_out/r4a/prod.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a/kern.log 2>&1 || { echo KERN_FAIL; tail -30 gpurun_out/r4a/kern.log; exit 1; }
tail -2 gpurun_out/r4a/kern.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_config_parity.py -x -v -s -k backward --timeout 600 --timeout-method thread > gpurun_out/r4a/bw.log 2>&1 || { echo BW_FAIL; tail -30 gpurun_out/r4a/bw.log; exit 1; }
tail -3 gpurun_out/r4a/bw.log
