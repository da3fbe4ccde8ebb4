#!/bin/bash
# round 4: whole-tree A/B (ab/tree = HEAD before): upsample backward gather loads issued together
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4av
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_config_parity.py tests/test_gpu_latent.py tests/test_gpu_graph.py tests/test_gpu_production_parity.py > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in vae; do
  for i in 1 2; do
    (cd ab/tree && timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --steps 40) > $O/${m}_old_$i.log 2>&1 || { echo FAIL old $m; tail -5 $O/${m}_old_$i.log; exit 1; }
    timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --steps 40 > $O/${m}_new_$i.log 2>&1 || { echo FAIL new $m; tail -5 $O/${m}_new_$i.log; exit 1; }
    echo "$m rep$i old $(tail -1 $O/${m}_old_$i.log | cut -c90-130) new $(tail -1 $O/${m}_new_$i.log | cut -c90-130)"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_old -o p -- python -u $R/ab/tree/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_old.log 2>&1 || { echo PROF_FAIL old; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_new.log 2>&1 || { echo PROF_FAIL new; exit 1; }
for v in old new; do find $O/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/unet_kernel_stats_$v.csv \; ; rm -rf $O/prof_$v; done
echo done
