set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for t in "" "0=255"; do
timeout -k 10 200 python -u tools/conv_bench.py --only fwd,dgrad --layers down1.1,inc.2,up4.2,down2.2 --reps 30 ${t:+--tune $t} > $O/tune.log 2>&1 || { echo FAIL; tail -20 $O/tune.log; exit 1; }
echo "tune=$t"; grep -v amdgpu.ids $O/tune.log
done
