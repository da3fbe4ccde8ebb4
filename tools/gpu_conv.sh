# conv microbench + SQ counter pass on the conv bench (run via gpurun)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/conv_bench.py --check --miopen ${CONV_ARGS:-} > $O/conv_bench.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv_bench.log; exit 1; }
cat $O/conv_bench.log
if [ -n "${PMC:-}" ]; then
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_sq -o conv -- python -u $R/tools/conv_bench.py --only fwd --reps 3 --layers inc.2,up3.2,up1.1,up4.1 > $O/pmc_sq.log 2>&1 || { echo PMC_FAIL; tail -20 $O/pmc_sq.log; exit 1; }
fi
echo DONE
