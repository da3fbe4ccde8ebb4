#!/bin/bash
# round 4: weight-image refresh in two launches; latent bwd (uniform job loops) profile
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest "tests/test_gpu_kernels.py::test_permute_batch_matches_single_launches" tests/test_gpu_graph.py tests/test_gpu_latent.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for m in unet vae; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o p -- python -u $R/bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$m.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_$m.log; exit 1; }
  find $O/prof_$m -name "*kernel_stats.csv" -exec cp {} $O/${m}_kernel_stats.csv \;
  grep -E "permute4|latent_bwd|heads_fwd|latent_sums|latent_fwd" $O/${m}_kernel_stats.csv | cut -c1-160
  tail -1 $O/prof_$m.log | cut -c1-120
done
