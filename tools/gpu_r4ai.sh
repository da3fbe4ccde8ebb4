#!/bin/bash
# round 4: 8-channel input pack (pixel per thread) + 64x64 weight-image transposes + batched clip-norm loads + unguarded pointwise-conv / scalar-BN-partial loads: tests + A/B + kernel times
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4ai
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py::test_permute_batch_matches_single_launches tests/test_gpu_kernels.py::test_input_pack_8_channels tests/test_gpu_kernels.py::test_outconv_pointwise_fwd tests/test_gpu_inference.py tests/test_gpu_attention_kernels.py tests/test_gpu_bn_fused.py tests/test_gpu_optim.py tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_production_parity.py > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_lib.sh old new "unet vae" || exit 1
cd /tmp
for v in old new; do
  cp $R/ab/lib_$v.so $R/vaeunet_amd/libvaeunet_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o p -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$v.log 2>&1 || { echo PROF_FAIL; cp $R/ab/lib_new.so $R/vaeunet_amd/libvaeunet_hip.so; exit 1; }
  find $O/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats_$v.csv \;
  rm -rf $O/prof_$v
done
cp $R/ab/lib_new.so $R/vaeunet_amd/libvaeunet_hip.so
