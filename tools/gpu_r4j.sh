#!/bin/bash
# round 4: two-chunk resident-weight fp8 conv (128 -> 64), fp8 benches
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4j
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/fp8_bench.py --json $O/fp8_layers.json > $O/fp8_layers.log 2>&1 || { echo FP8L_FAIL; tail -20 $O/fp8_layers.log; exit 1; }
grep SUMMARY $O/fp8_layers.log | cut -c1-400
grep '"up4' $O/fp8_layers.log | cut -c1-300
timeout -k 10 300 python -u tools/fp8_bench.py --double --json $O/fp8_double.json > $O/fp8_double.log 2>&1 || { echo FP8D_FAIL; tail -20 $O/fp8_double.log; exit 1; }
grep -v amdgpu.ids $O/fp8_double.log | cut -c1-330
timeout -k 10 300 python -u -m pytest "tests/test_gpu_kernels.py::test_permute_batch_matches_single_launches" tests/test_gpu_graph.py -k "permute or graph" -x -q --timeout 200 --timeout-method thread > $O/tests2.log 2>&1 || { echo TESTS2_FAIL; tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_unet -o p -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_unet.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_unet.log; exit 1; }
find $O/prof_unet -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats.csv \;
grep -E "permute4_batch|conv3x3_image" $O/unet_kernel_stats.csv | cut -c1-200
tail -1 $O/prof_unet.log | cut -c1-150
