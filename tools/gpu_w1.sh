# ConvTranspose weight-gradient split sweep (tools/wgrad1x1_bench.py --convt)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 150 python -u tools/wgrad1x1_bench.py --convt --splits ${SPLITS:-1,2,4,8,16,32} > $O/wT.log 2>&1 || { echo FAIL; tail -20 $O/wT.log; exit 1; }
grep -v amdgpu.ids $O/wT.log
