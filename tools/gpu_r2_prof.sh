#!/bin/bash
# per-layer 3x3 timings (+MIOpen fwd reference) and a rocprof kernel-stats pass of the bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-r2}
[ -n "$CONV" ] && { timeout -k 10 300 python tools/conv_bench.py --miopen > gpurun_out/${tag}_conv_bench.log 2>&1 || exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o ${tag} -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/${tag}_prof_bench.log 2>&1 || exit 1
find gpurun_out/${tag}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${tag}_kernel_stats.csv \;
tail -3 gpurun_out/${tag}_conv_bench.log
