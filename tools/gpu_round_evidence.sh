# full GPU test suite, then the round evidence (benches, rocprof stats, PMC traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-r3b}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/$tag/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$tag/gpu_tests.log
bash tools/gpu_evidence.sh $tag
