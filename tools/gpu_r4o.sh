#!/bin/bash
# round 4: global-address-space latent backward / permutes / AdamW: parity
# tests, latent phase timing, bench + kernel stats of both models
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4o
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_latent.py tests/test_gpu_optim.py tests/test_gpu_graph.py "tests/test_gpu_kernels.py" -k "latent or adamw or optim or graph or clip or permute or eager or unused" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp
for m in unet vae; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o p -- python -u $R/bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$m.log 2>&1 || { echo PROF_FAIL $m; exit 1; }
  tail -1 $O/prof_$m.log | cut -c1-200
  find $O/prof_$m -name "*kernel_stats.csv" -exec cp {} $O/${m}_kernel_stats.csv \;
  rm -rf $O/prof_$m
done
echo done
