#!/bin/bash
# Same-box A/B of two library builds (a compile-time change): ab/lib_relu.so vs ab/lib_norelu.so
# usage: MODEL=unet|vae bash tools/gpu_ab_so.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_so
for rep in 1 2; do
  for v in relu norelu; do
    cp ab/lib_$v.so vaeunet_amd/libvaeunet_hip.so
    timeout -k 10 200 python -u bench.py --model ${MODEL:-unet} --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/ab_so/${MODEL:-unet}_${v}_$rep.log 2>&1 || { echo FAIL; exit 1; }
    echo "$v rep$rep: $(tail -1 gpurun_out/ab_so/${MODEL:-unet}_${v}_$rep.log | cut -c80-140)"
  done
done
cp ab/lib_relu.so vaeunet_amd/libvaeunet_hip.so
