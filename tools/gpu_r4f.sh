#!/bin/bash
# round 4: latent bottleneck kernels rewrite, column-major halo wgrad walk, FastDiv / image prefetch
# (tests + A/B vs HEAD~ build), encoder weight-gradient split-K cap sweep, L2 hit rates
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py tests/test_gpu_kernels.py tests/test_gpu_ops.py -k "latent or wgrad or fwd_dgrad or image or stream or v5 or full_phase or vae" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --model vae --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log | cut -c1-300
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_vae.log; exit 1; }
find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \;
cd $R
for ws in 0 8 4; do
  timeout -k 10 200 python -u tools/enc_bench.py --wsplit $ws > $O/enc_ws$ws.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc_ws$ws.log; exit 1; }
  echo "wsplit=$ws"; grep -v amdgpu.ids $O/enc_ws$ws.log | cut -c1-150
done
bash tools/gpu_ab_lib.sh old new "unet"
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_l2_unet -o l -- python -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/pmc_l2_unet.log 2>&1 || { echo L2_FAIL; tail -5 $O/pmc_l2_unet.log; exit 1; }
cd $R
python tools/pmc_l2.py $O/pmc_l2_unet 30 > $O/l2_unet.txt && cat $O/l2_unet.txt
rm -rf $O/pmc_l2_unet
