# kernel parity + per-layer timing + bench (no profiler)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pt.log | head -20; tail -20 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 200 python -u tools/conv_bench.py --only fwd,dgrad > $O/conv.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv.log; exit 1; }
grep TOTAL $O/conv.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
