# A/B of the whole product path: an older tree (Python + library) copied to
# ab/tree vs the current one, bench.py alternating on the same box
# usage: bash tools/gpu_ab_tree.sh [model]
set -e
model=${1:-unet}
R=$(pwd)
for i in 1 2; do
  (cd ab/tree && timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --no-roofline --steps 40) | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('old', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --no-roofline --steps 40 | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('new', d['value'], d['ms_per_step'])"
done
