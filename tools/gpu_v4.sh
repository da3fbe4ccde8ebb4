set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 100 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pt.log | head -20; tail -20 $O/pt.log; exit 1; }
tail -2 $O/pt.log
timeout -k 10 200 python -u tools/conv_bench.py --check --only fwd,dgrad > $O/conv_v4p.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_v4p.log; exit 1; }
grep -v amdgpu.ids $O/conv_v4p.log
