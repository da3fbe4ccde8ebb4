# wgrad halo kernel experiment modes (VU_W3_XM, gemm_wgrad3.hip) + kernel parity
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for m in ${XMS:-0 3}; do
  echo "== W3 XM=$m"
  VU_W3_XM=$m timeout -k 10 150 python -u tools/conv_bench.py --only wgrad > $O/w3xm$m.log 2>&1 || { echo FAIL; tail -20 $O/w3xm$m.log; exit 1; }
  grep -v amdgpu.ids $O/w3xm$m.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pt_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" $O/pt_kernels.log | head -30; exit 1; }
tail -1 $O/pt_kernels.log
