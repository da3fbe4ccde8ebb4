# v8 (ping-pong tiles on 32x32x16 MFMAs): kernel tests, per-layer A/B vs v4, bench A/B
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "pingpong or splitk or fwd_dgrad_wgrad or small_grid" > gpurun_out/t_v8.log 2>&1
for v in 0 1; do timeout -k 10 200 python -u tools/conv_bench.py --only fwd,dgrad --check --tune 22=$v > gpurun_out/conv_v8_$v.log 2>&1; done
bash tools/gpu_ab_tune.sh 22 0 1 "unet vae"
