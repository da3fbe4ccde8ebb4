set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_optim.py -q -x --timeout 100 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -2 $O/pt.log
for m in 1 2; do
echo "== W3 XM=$m"
VU_W3_XM=$m timeout -k 10 200 python -u tools/conv_bench.py --only wgrad > $O/w3xm$m.log 2>&1 || { echo FAIL; tail -30 $O/w3xm$m.log; exit 1; }
grep -v amdgpu.ids $O/w3xm$m.log
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python -u $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof2.log 2>&1 || { echo PROF_FAIL; exit 1; }
grep permute $O/prof2/run_kernel_stats.csv | cut -c1-150
