#!/bin/bash
# round 4: BatchNorm backward through the max-pool (engine.POOL_BN_BWD): tests + A/B + kernel table
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4af
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bn_fused.py tests/test_gpu_model.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_production_parity.py tests/test_gpu_config_parity.py > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_flag.sh engine.POOL_BN_BWD || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python -u $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats.csv \;
rm -rf $O/prof
grep -E "pool_bn|maxpool_bwd|chan_partial|bn_bwd_apply" $O/unet_kernel_stats.csv | cut -d, -f1-4
