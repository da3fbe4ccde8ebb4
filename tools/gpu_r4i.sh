#!/bin/bash
# round 4: remaining GPU test files after the ops fix, tap-merged weight-image transpose, benches
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4i
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_optim.py tests/test_gpu_parallel.py tests/test_gpu_parity.py tests/test_gpu_production_parity.py tests/test_gpu_graph.py "tests/test_gpu_kernels.py::test_permute_batch_matches_single_launches" -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --model vae --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo VBENCH_FAIL; tail -20 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_unet.log 2>&1 || { echo UBENCH_FAIL; tail -20 $O/bench_unet.log; exit 1; }
tail -1 $O/bench_unet.log | cut -c1-1200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_unet -o p -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_unet.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_unet.log; exit 1; }
find $O/prof_unet -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats.csv \;
