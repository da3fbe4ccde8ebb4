set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/v2a_tests.log 2>&1
VU_LIB_PATH=ab/lib_957.so timeout -k 10 120 python tools/enc_bench.py > gpurun_out/v2a_enc_old.log 2>&1
timeout -k 10 120 python tools/enc_bench.py > gpurun_out/v2a_enc_new.log 2>&1
VU_LIB_PATH=ab/lib_957.so timeout -k 10 300 python -u bench.py --model vae --no-cpu-baseline --no-roofline > gpurun_out/v2a_vae_old.log 2>&1
timeout -k 10 300 python -u bench.py --model vae --no-cpu-baseline --no-roofline > gpurun_out/v2a_vae_new.log 2>&1
