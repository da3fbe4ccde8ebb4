# full GPU check: parity tests, bench (with cpu baseline), rocprof kernel trace (csv)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
if [ -z "${NOPROF:-}" ]; then
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -30 $O/prof.log; exit 1; }
tail -1 $O/prof.log
fi
echo DONE
