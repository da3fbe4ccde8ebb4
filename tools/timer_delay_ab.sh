#!/bin/bash
# Same-box check of the roofline leg's per-launch timing with and without a
# GPU delay queued in front of each timed launch (bench.py --timer-delay):
# if host enqueue time leaks into the event brackets, the delayed runs report
# shorter kernel times.  usage: bash tools/timer_delay_ab.sh <tag> [delay]
set -o pipefail
tag=${1:-timer_delay}; d=${2:-20}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$tag
mkdir -p $O
for i in 1 2; do
  for dl in 0 $d; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 40 --timer-delay $dl \
      > $O/b_${dl}_$i.json 2> $O/b_${dl}_$i.err || { echo "BENCH_FAIL delay $dl"; tail -5 $O/b_${dl}_$i.err; exit 1; }
    python - "$O/b_${dl}_$i.json" "$dl" <<'PY' | tee -a $O/summary.txt
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
kinds = {k: v["ms_per_step"] for k, v in r["per_kind"].items() if k.startswith("conv3x3_") and "image" not in k}
print(f"delay {sys.argv[2]:>3}: value {l['value']} frac {r['frac']} 3x3 ms/step {kinds}")
PY
  done
done
