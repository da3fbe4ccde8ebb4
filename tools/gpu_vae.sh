# BASELINE configs[2]: VAE-U-Net bench + kernel stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u bench.py --model vae --steps 20 --warmup 5 > $O/bench_vae.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o run -- python -u $R/bench.py --model vae --steps 5 --warmup 2 --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; tail -30 $O/prof_vae.log; exit 1; }
echo DONE
