set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv" --timeout 100 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pt.log | head -20; tail -20 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for tj in 1 2; do
VU_W3_TJ=$tj timeout -k 10 200 python -u tools/conv_bench.py --check --only wgrad,fwd > $O/w3_$tj.log 2>&1 || { echo FAIL; tail -20 $O/w3_$tj.log; exit 1; }
echo "TJ=$tj"; grep -v amdgpu.ids $O/w3_$tj.log
done
