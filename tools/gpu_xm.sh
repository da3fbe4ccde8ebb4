# v4 experiment modes (VU_V4_XM, gemm_fwd4.hip) on the large 3x3 layers
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
L=${LAYERS:-inc.2,down1.2,down2.2,down3.2,up1.1,up2.1,up3.1,up4.1}
for m in ${XMS:-0 1 2 3}; do
  echo "== XM=$m"
  VU_V4_XM=$m timeout -k 10 120 python -u tools/conv_bench.py --only fwd --layers $L > $O/xm$m.log 2>&1 || { echo FAIL; tail -20 $O/xm$m.log; exit 1; }
  grep -v amdgpu.ids $O/xm$m.log
done
