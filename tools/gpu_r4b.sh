#!/bin/bash
# round 4: halo weight-gradient main loop (VU_TUNE_W3_FAST = 26) correctness + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wgrad or fwd_dgrad" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo KERN_FAIL; tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_production_parity.py -x -q -s --timeout 500 --timeout-method thread > $O/prod.log 2>&1 || { echo PROD_FAIL; tail -30 $O/prod.log; exit 1; }
tail -1 $O/prod.log
for rep in 1 2; do
  for v in 0 1 2; do
    timeout -k 10 200 python -u tools/conv_bench.py --only wgrad --tune 26=$v > $O/cb_${v}_$rep.log 2>&1 || { echo CB_FAIL; tail -20 $O/cb_${v}_$rep.log; exit 1; }
    echo "w3fast=$v rep$rep: $(grep TOTAL $O/cb_${v}_$rep.log)"
  done
done
bash tools/gpu_ab_tune.sh 26 0 1 "unet vae"
timeout -k 10 900 python -u -m pytest tests/test_gpu_config_parity.py -x -v -s -k backward --timeout 600 --timeout-method thread > $O/bw.log 2>&1 || { echo BW_FAIL; tail -30 $O/bw.log; exit 1; }
grep "adjudicated" $O/bw.log; tail -1 $O/bw.log
