# 1x1 / 3x3 weight-gradient split sweep (VU_WGRAD_SPLIT_PIX), then kernel tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 150 python -u tools/wgrad1x1_bench.py --splits 256,512 > $O/w1.log 2>&1 || { echo FAIL; tail -20 $O/w1.log; exit 1; }
grep -v amdgpu.ids $O/w1.log
for sp in ${SPS:-1000000000 4096 2048}; do
  echo "== SPLIT_PIX=$sp"
  VU_WGRAD_SPLIT_PIX=$sp timeout -k 10 150 python -u tools/conv_bench.py --only wgrad > $O/w3_$sp.log 2>&1 || { echo FAIL; tail -20 $O/w3_$sp.log; exit 1; }
  grep -v amdgpu.ids $O/w3_$sp.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pt_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" $O/pt_kernels.log | head -30; exit 1; }
tail -1 $O/pt_kernels.log
