#!/bin/bash
# GPU test run: the whole -m gpu suite, one process, bounded
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 150 --timeout-method thread -s \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
