set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for c in 0 1 2; do
echo "== VU_V2_CFG=$c"
VU_V2_CFG=$c timeout -k 10 200 python -u tools/gemm1x1_bench.py --check > $O/g1_cfg$c.log 2>&1 || { echo FAIL; tail -30 $O/g1_cfg$c.log; exit 1; }
grep -v amdgpu.ids $O/g1_cfg$c.log
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -k permute --timeout 100 --timeout-method thread 2>&1 | tail -2
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python -u $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof2.log 2>&1 || { echo PROF_FAIL; exit 1; }
grep permute $O/prof2/run_kernel_stats.csv | cut -c1-150
