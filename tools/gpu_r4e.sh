#!/bin/bash
# round 4: v2 tail kernel / small-M wgrad (config 3 generic rows), fused fp8 BN-apply quantise
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4e
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_kernels.py -k "fp8 or image or stream or v5 or full_phase" -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --model vae --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_vae.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_vae.log; exit 1; }
tail -1 $O/bench_vae.log | cut -c1-400
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_vae.log; exit 1; }
find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \;
cd $R
timeout -k 10 300 python -u tools/fp8_bench.py --double --json $O/fp8_double.json > $O/fp8_double.log 2>&1 || { echo FP8D_FAIL; tail -20 $O/fp8_double.log; exit 1; }
grep -v amdgpu.ids $O/fp8_double.log
for rep in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python -u tools/conv_bench.py --only fwd --tune 27=$v > $O/cbpp_${v}_$rep.log 2>&1 || { echo CB_FAIL; tail -20 $O/cbpp_${v}_$rep.log; exit 1; }
    echo "ppfull=$v rep$rep: $(grep TOTAL $O/cbpp_${v}_$rep.log | tr '\n' ' ')"
  done
done
bash tools/gpu_ab_tune.sh 27 0 1 "unet"
