set -e
cd $GRAFT_REPO_ROOT
L=inc.2,down3.2,down4.2,up1.1,up2.1,up4.1
for m in 0 1 2; do timeout -k 10 200 python -u tools/fp8_bench.py --layers $L --no-bf16 --tune 20=$m > gpurun_out/fp8pp_xm$m.log 2>&1; done
