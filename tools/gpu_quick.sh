# quick check: all GPU tests, UNet + VAE bench (no cpu baseline), census
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/q_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q_unet.log 2>&1
timeout -k 10 300 python -u bench.py --model vae --no-cpu-baseline > gpurun_out/q_vae.log 2>&1
timeout -k 10 300 python tools/census.py --top 150 > gpurun_out/census9.log 2>&1
