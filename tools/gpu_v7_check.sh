# v7 small-grid conv: kernel tests, then per-layer timings (graph replay)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "small_grid or pingpong_splitk or splitk_auto" > gpurun_out/t_v7.log 2>&1
timeout -k 10 120 python -u tools/enc_bench.py --tune 16=1 > gpurun_out/enc_v7_1.log 2>&1
timeout -k 10 120 python -u tools/enc_bench.py --tune 16=1,17=3 > gpurun_out/enc_v7_1n3.log 2>&1
for m in 2 4; do timeout -k 10 120 python -u tools/enc_bench.py --tune 16=1,18=$m > gpurun_out/enc_g_xm_$m.log 2>&1; done
timeout -k 10 120 python -u tools/enc_bench.py --tune 16=2 > gpurun_out/enc_v7_2.log 2>&1
