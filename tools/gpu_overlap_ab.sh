#!/bin/bash
# A/B of the side-stream weight-gradient overlap (engine.OVERLAP_WGRAD) on one
# box, both models, plus the host-CPU probe.  -> gpurun_out/ovl/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ovl
mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/cpu_probe.py > $O/cpu_probe.log 2>&1 || echo CPU_PROBE_FAIL
for rep in 1 2; do
  for m in unet vae; do
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --overlap > $O/${m}_on_$rep.log 2>&1 || { echo FAIL $m on; tail -30 $O/${m}_on_$rep.log; exit 1; }
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/${m}_off_$rep.log 2>&1 || { echo FAIL $m off; exit 1; }
  done
done
for f in $O/*_o*.log; do echo "$(basename $f): $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
cat $O/cpu_probe.log
