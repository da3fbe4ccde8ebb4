#!/bin/bash
# round 4 close: the default bench line, then rocprof / PMC / replay / tail evidence (tools/gpu_r4an.sh)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4ar
mkdir -p $O
cd $R
timeout -k 10 560 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
bash tools/gpu_r4an.sh r4ar
