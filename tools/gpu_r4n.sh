#!/bin/bash
# round 4: latent backward phase timing; wgrad side-stream overlap A/B (graph replay)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4n
mkdir -p $O
cd $R
bash tools/gpu_ab_flag.sh engine.OVERLAP_WGRAD
