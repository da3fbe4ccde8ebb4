#!/bin/bash
# SQ counters of the 1x1 / ConvT weight-gradient kernels (tools/wgrad1x1_bench.py --convt)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmcw -o w -- python -u $R/tools/wgrad1x1_bench.py --convt --splits 4 > $R/gpurun_out/pmcw.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/pmcw.log; exit 1; }
echo PMC_OK
