#!/bin/bash
# round 4: latent backward over the concatenated consumer space (LDS job table)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py tests/test_gpu_ops.py -k "latent or vae" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_vae.log; exit 1; }
find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \;
grep -E "latent|heads_fwd" $O/vae_kernel_stats.csv | cut -c1-160
