# persistent v5 3x3 kernel for the narrow-input layers (VU_TUNE_V5_MAX_C = 1) vs default
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for mc in ${MAXCS:-0 64 128}; do
  echo "== V5_MAX_C=$mc"
  timeout -k 10 150 python -u tools/conv_bench.py --only fwd,dgrad --tune 1=$mc > $O/v5_$mc.log 2>&1 || { echo FAIL; tail -20 $O/v5_$mc.log; exit 1; }
  grep -v amdgpu.ids $O/v5_$mc.log
done
