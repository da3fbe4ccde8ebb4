#!/bin/bash
# round 4: two-launch latent backward: parity tests + VAE bench kernel stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_latent.py tests/test_gpu_graph.py $(ls tests/test_gpu_vae*.py tests/test_gpu_infer*.py 2>/dev/null) > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vae -o p -- python -u $R/bench.py --model vae --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_vae.log 2>&1 || { echo PROF_FAIL; exit 1; }
grep '"metric"' $O/prof_vae.log | cut -c1-200
find $O/prof_vae -name "*kernel_stats.csv" -exec cp {} $O/vae_kernel_stats.csv \;
rm -rf $O/prof_vae
grep -E "latent|heads" $O/vae_kernel_stats.csv | cut -c1-160
echo done
