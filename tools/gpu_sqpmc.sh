# SQ counters of the 3x3 conv kernels on a few layers (one pass, <= 8 SQ counters)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $O/sqpmc -o s -- python -u $R/tools/conv_bench.py --only fwd,dgrad,wgrad --layers down2.2,up3.1,inc.2 --reps 3 > $O/sqpmc.log 2>&1 || { echo PMC_FAIL; tail -20 $O/sqpmc.log; exit 1; }
echo DONE
