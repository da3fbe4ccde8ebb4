#!/bin/bash
# Round evidence on one GPU box: both bench lines (UNet = the metric, with
# cpu_baseline + parity + roofline; VAE-U-Net = config 3), rocprofv3 kernel
# stats of each bench, and the HBM-traffic PMC passes of each (FETCH_SIZE and
# WRITE_SIZE in separate runs: MI355X_MICROARCH.md HBM section).
# usage: bash tools/gpu_evidence.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
export TMPDIR=/tmp
tag=${1:-evidence}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
cd /tmp
for m in unet vae; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o p -- python -u $R/bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$m.log 2>&1 || { echo PROF_FAIL $m; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$m -o f -- python -u $R/bench.py --model $m --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_fetch_$m.log 2>&1 || { echo FETCH_FAIL $m; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$m -o w -- python -u $R/bench.py --model $m --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_write_$m.log 2>&1 || { echo WRITE_FAIL $m; exit 1; }
done
cd $R
python tools/pmc_traffic.py $O/pmc_fetch_unet $O/pmc_write_unet $O/pmc_traffic.json &&
python tools/pmc_traffic.py $O/pmc_fetch_vae $O/pmc_write_vae $O/pmc_traffic_vae.json &&
for m in unet vae; do find $O/prof_$m -name "*kernel_stats.csv" -exec cp {} $O/${m}_kernel_stats.csv \; ; done &&
rm -rf $O/pmc_fetch_* $O/pmc_write_*
for m in unet vae; do python tools/replay_trace.py $O/prof_$m/p_kernel_trace.csv --list-last > $O/replay_trace_$m.txt || exit 1; done
python tools/tail_bw.py $O/pmc_traffic.json $O/unet_kernel_stats.csv 13 45 > $O/tail_bw_unet.txt &&
python tools/tail_bw.py $O/pmc_traffic_vae.json $O/vae_kernel_stats.csv 13 45 > $O/tail_bw_vae.txt &&
rm -f $O/prof_unet/p_kernel_trace.csv.gz && echo evidence-done
