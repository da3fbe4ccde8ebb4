#!/bin/bash
# round 4: latent vector path (csrc/latent.hip) correctness + A/B; backward parity; DP unused params
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py -x -v -s --timeout 200 --timeout-method thread > $O/latent.log 2>&1 || { echo LAT_FAIL; tail -40 $O/latent.log; exit 1; }
grep -E "worst|passed|failed" $O/latent.log | tail -14
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_inference.py -x -q -k "vae or resnet or decoder or latent or graph or infer" --timeout 300 --timeout-method thread > $O/vae_tests.log 2>&1 || { echo VAE_FAIL; tail -40 $O/vae_tests.log; exit 1; }
tail -1 $O/vae_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1 || { echo PAR_FAIL; tail -40 $O/par.log; exit 1; }
tail -1 $O/par.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_config_parity.py -x -v -s --timeout 800 --timeout-method thread > $O/cfg.log 2>&1 || { echo CFG_FAIL; tail -40 $O/cfg.log; exit 1; }
grep -E "adjudicated|flips|passed|failed" $O/cfg.log | tail -10
timeout -k 10 600 python -u -m pytest tests/test_gpu_production_parity.py -x -q -s -k config3 --timeout 500 --timeout-method thread > $O/prod3.log 2>&1 || { echo PROD_FAIL; tail -30 $O/prod3.log; exit 1; }
tail -1 $O/prod3.log
for rep in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python -u bench.py --model vae --steps 30 --warmup 5 --no-cpu-baseline --no-roofline \
      --engine-flag vae_engine.LATENT_VECTORS=$v > $O/vae_${v}_$rep.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/vae_${v}_$rep.log; exit 1; }
    echo "vae LATENT_VECTORS=$v rep$rep: $(tail -1 $O/vae_${v}_$rep.log | cut -c100-190)"
  done
done
