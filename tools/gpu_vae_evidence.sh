# config-3 (VAE-U-Net) evidence: full bench line (cpu_baseline + parity +
# roofline), then the HBM traffic PMC passes of its 3x3 kernels
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/vae
mkdir -p $O
cd $R
timeout -k 10 900 python -u bench.py --model vae > $O/bench_vae.log 2>&1 || { echo VAE_FAIL; tail -20 $O/bench_vae.log; exit 1; }
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python -u $R/bench.py --model vae --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python -u $R/bench.py --model vae --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
cd $R && python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic_vae.json && rm -rf $O/pmc_fetch $O/pmc_write && tail -1 $O/bench_vae.log | cut -c1-1500
