set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python -u tools/conv_bench.py --check --only fwd,dgrad > $O/conv_v4b.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_v4b.log; exit 1; }
grep -v amdgpu.ids $O/conv_v4b.log
VU_V4_XM=4 timeout -k 10 200 python -u tools/conv_bench.py --only fwd > $O/conv_v4b_xm4.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_v4b_xm4.log; exit 1; }
grep -v amdgpu.ids $O/conv_v4b_xm4.log
