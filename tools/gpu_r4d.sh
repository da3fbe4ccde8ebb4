#!/bin/bash
# round 4: new dispatcher ops + inference tests; kernel profiles of both benches
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4d
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_inference.py tests/test_gpu_fold.py -x -q --timeout 200 --timeout-method thread > $O/ops.log 2>&1 || { echo OPS_FAIL; tail -40 $O/ops.log; exit 1; }
tail -1 $O/ops.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_unet.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_unet.log; exit 1; }
tail -1 $O/bench_unet.log | cut -c1-600
cd /tmp
for m in unet vae; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o p -- python -u $R/bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$m.log 2>&1 || { echo PROF_FAIL $m; tail -5 $O/prof_$m.log; exit 1; }
  find $O/prof_$m -name "*kernel_stats.csv" -exec cp {} $O/${m}_kernel_stats.csv \;
done
ls $O
cd $R
timeout -k 10 300 python -u tools/gemm1x1_bench.py > $O/gemm1x1.log 2>&1 || { echo G1_FAIL; tail -5 $O/gemm1x1.log; exit 1; }
cat $O/gemm1x1.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/census.py --model unet --steps 2 --top 70 > $O/census_unet.log 2>&1 || { echo CENSUS_FAIL; tail -5 $O/census_unet.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 120 --timeout-method thread > $O/fp8_tests.log 2>&1 || { echo FP8T_FAIL; tail -30 $O/fp8_tests.log; exit 1; }
tail -1 $O/fp8_tests.log
timeout -k 10 300 python -u tools/fp8_bench.py --double --json $O/fp8_double.json > $O/fp8_double.log 2>&1 || { echo FP8D_FAIL; tail -20 $O/fp8_double.log; exit 1; }
grep -v amdgpu.ids $O/fp8_double.log
