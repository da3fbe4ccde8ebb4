#!/bin/bash
# SQ instruction-timing counters per kernel over one UNet (or VAE) bench step:
# where the 3x3 MFMA kernels' wave cycles go (parked on s_waitcnt/barrier,
# issue-stalled, issuing) and how busy the matrix pipes are
# (MI355X_MICROARCH.md, rocprofv3 PMC slots: WAIT_ANY + WAIT_INST_ANY +
# ACTIVE_INST_ANY ~= WAVE_CYCLES).  Two separate --pmc passes, each within
# the per-block slot limits (SQ <= 8, GRBM <= 2), no trace domains.
# usage: bash tools/gpu_sq_timing.sh <tag> [unet|vae]   -> gpurun_out/<tag>/
set -o pipefail
export TMPDIR=/tmp
tag=${1:-sq}
m=${2:-unet}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $O/sq1_$m -o s -- python -u $R/bench.py --model $m --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/sq1_$m.log 2>&1 || { echo SQ1_FAIL; tail -20 $O/sq1_$m.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $O/sq2_$m -o s -- python -u $R/bench.py --model $m --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/sq2_$m.log 2>&1 || { echo SQ2_FAIL; tail -20 $O/sq2_$m.log; }
cd $R
python tools/sq_timing.py $O/sq1_$m $O/sq2_$m > $O/sq_timing_$m.txt && cat $O/sq_timing_$m.txt | cut -c1-220
