#!/bin/bash
# run a selection of GPU tests: tools/gpu_r2_sel.sh <log name> <pytest args...>
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 150 --timeout-method thread -s "$@" \
  > gpurun_out/$name.log 2>&1
rc=$?
tail -30 gpurun_out/$name.log
exit $rc
