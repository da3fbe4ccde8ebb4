# v6 (64->64 resident-weight 3x3): kernel tests, experiment modes, A/B vs ab/base.so in one process set
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "c64 or conv3x3_fwd_dgrad" > $O/v6_tests.log 2>&1 || { tail -30 $O/v6_tests.log; exit 1; }
tail -1 $O/v6_tests.log
for m in 0 1 2 3; do echo "== xm $m"; timeout -k 10 120 python -u tools/conv_bench.py --layers inc.2,up4.2 --only fwd,dgrad --tune 12=$m || exit 1; done > $O/v6_xm.log 2>&1
echo "== base" >> $O/v6_xm.log; VU_LIB_PATH=ab/base.so timeout -k 10 120 python -u tools/conv_bench.py --layers inc.2,up4.2 --only fwd,dgrad >> $O/v6_xm.log 2>&1
grep -v amdgpu $O/v6_xm.log | grep -v "^inc\|^up4"
