# two separate PMC passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: never together)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_write.log 2>&1 || { echo WRITE_FAIL; tail -20 $O/pmc_write.log; exit 1; }
cd $R && python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json
