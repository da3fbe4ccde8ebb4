#!/bin/bash
# round 4: latent bwd batched loads; fp8 chained blocks; A/B of the FastDiv / image prefetch / column-major wgrad kernels
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py tests/test_gpu_fp8.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --model vae --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_vae.log; exit 1; }
find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \;
cd $R
timeout -k 10 300 python -u tools/fp8_bench.py --double --json $O/fp8_double.json > $O/fp8_double.log 2>&1 || { echo FP8D_FAIL; tail -20 $O/fp8_double.log; exit 1; }
grep -v amdgpu.ids $O/fp8_double.log | cut -c1-330
bash tools/gpu_ab_lib.sh old new "unet vae"
