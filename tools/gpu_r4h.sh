#!/bin/bash
# round 4: full GPU suite + both benches (latent bwd uniform job loops, split-K FULL)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4h
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --model vae --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo VBENCH_FAIL; tail -20 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_unet.log 2>&1 || { echo UBENCH_FAIL; tail -20 $O/bench_unet.log; exit 1; }
tail -1 $O/bench_unet.log | cut -c1-900
