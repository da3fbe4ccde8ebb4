#!/bin/bash
# round 4: latent backward phase timing; wgrad side-stream overlap A/B (graph replay)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4n
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/latent_phases.py > $O/latent_phases.log 2>&1 || { echo LP_FAIL; tail -20 $O/latent_phases.log; exit 1; }
grep -v amdgpu.ids $O/latent_phases.log
bash tools/gpu_ab_flag.sh engine.OVERLAP_WGRAD
