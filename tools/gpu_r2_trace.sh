#!/bin/bash
# kernel trace (per-dispatch durations) of a tool run: tools/gpu_r2_trace.sh <tag> <python args...>
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$(pwd)
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_$tag -o t -- python -u "$@" > $R/gpurun_out/tr_$tag.log 2>&1 || { echo TRACE_FAIL; tail -20 $R/gpurun_out/tr_$tag.log; exit 1; }
find $R/gpurun_out/tr_$tag -name "*kernel_trace.csv" -exec cp {} $R/gpurun_out/tr_${tag}_kernels.csv \;
echo TRACE_OK
