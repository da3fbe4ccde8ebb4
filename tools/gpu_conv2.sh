set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python -u tools/conv_bench.py --check --only fwd,dgrad > $O/conv_v4.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_v4.log; exit 1; }
cat $O/conv_v4.log
VU_GEMM_V4=0 timeout -k 10 200 python -u tools/conv_bench.py --only fwd,dgrad > $O/conv_v3.log 2>&1 || { echo CONV3_FAIL; tail -30 $O/conv_v3.log; exit 1; }
tail -3 $O/conv_v3.log
echo DONE
