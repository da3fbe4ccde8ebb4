# v4 weight-ring depth / column-tile sweep on the 3x3 layer shapes, then kernel parity
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for cfg in ${CFGS:-"3 256" "4 256" "6 256" "3 128" "6 128"}; do
  set -- $cfg
  echo "== NBW=$1 PREF_BN=$2"
  VU_V4_NBW=$1 VU_V4_PREF_BN=$2 timeout -k 10 150 python -u tools/conv_bench.py --only fwd,dgrad > $O/nbw_$1_$2.log 2>&1 || { echo FAIL; tail -20 $O/nbw_$1_$2.log; exit 1; }
  grep -v amdgpu.ids $O/nbw_$1_$2.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pt_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" $O/pt_kernels.log | head -30; exit 1; }
tail -1 $O/pt_kernels.log
