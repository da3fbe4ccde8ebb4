#!/bin/bash
# round 4: v7 prologue wait + two-group epilogue: tests, encoder layer bench, VAE bench/profile
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4l
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "small_grid or v7 or splitk_auto or stride2 or permute" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_production_parity.py -k config3 -x -q -s --timeout 500 --timeout-method thread > $O/prod.log 2>&1 || { echo PROD_FAIL; tail -30 $O/prod.log; exit 1; }
tail -1 $O/prod.log
timeout -k 10 200 python -u tools/enc_bench.py > $O/enc.log 2>&1 || { echo ENC_FAIL; tail -20 $O/enc.log; exit 1; }
grep -v amdgpu.ids $O/enc.log | cut -c1-150
timeout -k 10 300 python -u bench.py --model vae --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo VBENCH_FAIL; tail -20 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_vae.log; exit 1; }
find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \;
grep -E "conv3x3_sg|latent_bwd" $O/vae_kernel_stats.csv | cut -c1-160
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_unet -o p -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_unet.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_unet.log; exit 1; }
find $O/prof_unet -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats.csv \;
grep -E "permute4" $O/unet_kernel_stats.csv | cut -c1-160
