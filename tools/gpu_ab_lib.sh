#!/bin/bash
# Same-box A/B of two library builds ab/lib_$A.so vs ab/lib_$B.so (compile-time
# changes): the 1x1/ConvT kernel table (tools/gemm1x1_bench.py) and bench.py,
# interleaved, 2 reps.  usage: bash tools/gpu_ab_lib.sh A B "unet vae"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$1; B=$2; MODELS=$3
O=$R/gpurun_out/ab_lib_${A}_$B
mkdir -p $O
cd $R
cp vaeunet_amd/libvaeunet_hip.so $O/lib_orig.so
for rep in 1 2; do
  for v in $A $B; do
    cp ab/lib_$v.so vaeunet_amd/libvaeunet_hip.so
    timeout -k 10 200 python -u tools/gemm1x1_bench.py > $O/g1_${v}_$rep.log 2>&1 || { echo G1FAIL $v; tail -20 $O/g1_${v}_$rep.log; cp $O/lib_orig.so vaeunet_amd/libvaeunet_hip.so; exit 1; }
    echo "g1 $v rep$rep: $(grep -i total $O/g1_${v}_$rep.log | tr '\n' ' ')"
    for m in $MODELS; do
      timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/${m}_${v}_$rep.log 2>&1 || { echo FAIL $m $v; tail -20 $O/${m}_${v}_$rep.log; cp $O/lib_orig.so vaeunet_amd/libvaeunet_hip.so; exit 1; }
      echo "$m $v rep$rep: $(tail -1 $O/${m}_${v}_$rep.log | cut -c1-100)"
    done
  done
done
cp $O/lib_orig.so vaeunet_amd/libvaeunet_hip.so
