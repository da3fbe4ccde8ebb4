#!/bin/bash
# A/B of an environment knob on one box: bench.py per value, alternating
# usage: bash tools/gpu_env_ab.sh <VAR> <model> <rounds> <value>...
set -o pipefail
var=$1; model=$2; rounds=$3; shift 3
for i in $(seq $rounds); do
  for v in "$@"; do
    env $var=$v timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --no-roofline --steps 40 2>/dev/null | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$var=$v', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
