# A/B of two library builds on the same box: bench.py alternating
# usage: bash tools/gpu_ab.sh <old.so> [model]
set -e
old=$1; model=${2:-unet}
for i in 1 2; do
  VU_LIB_PATH=$old timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --no-roofline --steps 40 | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('old', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --no-roofline --steps 40 | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('new', d['value'], d['ms_per_step'])"
done
