# v7 fragment-read placement x (loop DMA on / off), graph-replay timing
set -e
cd $GRAFT_REPO_ROOT
for rp in 0 1 2; do for xm in 0 2; do timeout -k 10 120 python -u tools/enc_bench.py --tune 16=1,18=$xm,19=$rp > gpurun_out/enc_rp${rp}_xm$xm.log 2>&1; done; done
