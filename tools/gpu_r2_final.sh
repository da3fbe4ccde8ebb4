#!/bin/bash
# Round-2 evidence: full bench (cpu_baseline + parity + roofline), rocprof
# kernel stats of the UNet and VAE benches, HBM traffic PMC passes.
# usage: bash tools/gpu_r2_final.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python -u bench.py --model vae --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo VAE_FAIL; tail -20 $O/bench_vae.log; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_unet -o u -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_unet.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o v -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROFV_FAIL; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
cd $R && python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json && find $O/prof_unet -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats.csv \; && find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \; && rm -rf $O/pmc_fetch $O/pmc_write && tail -1 $O/bench.log | cut -c1-600 && tail -1 $O/bench_vae.log | cut -c1-300
