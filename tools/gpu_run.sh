#!/bin/bash
# One parameterised GPU-box run: a chain of steps, each under its own time
# limit, stopping at the first failure.  Replaces the per-call gpu_r4*.sh
# scripts of round 4.
#
# usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]      -> gpurun_out/<tag>/
# steps:
#   tests[:<pytest -k or file list, comma separated>]  GPU tests (default: whole -m gpu suite)
#   bench[:<model>]        the default bench line (model unet: CPU leg + config-3 secondary)
#   ab[:<model>[:<reps>]]  whole-tree A/B vs the tree copied to ab/tree (alternating, same box)
#   flag:<module.NAME>[:<model>]  A/B of an engine flag (0 vs 1) on the current tree
#   tune:<KEY>:<A>:<B>[:<model>]   A/B of a library tuning key (vu_gemm_set_tuning) A vs B
#   prof[:<model>[:<module.NAME=v>]]  rocprofv3 --kernel-trace --stats of a short bench
#                          (optionally with an engine flag set) -> <model>[_<flag>]_kernel_stats.csv
#   evidence               tools/gpu_evidence.sh (both benches profiled + PMC traffic + tables)
#   sq[:<model>]           tools/gpu_sq_timing.sh (SQ wave-cycle / MFMA-busy counters per kernel)
#   conv[:<args>]          tools/conv_bench.py with the given args (spaces as '+')
#   enc[:<args>]           tools/enc_bench.py with the given args (spaces as '+')
#   py:<script>[:<args>]   any python tool under tools/ (args: spaces as '+')
#   rprof:<script>[:<args>]  the same under rocprofv3 --kernel-trace --stats -> rprof_<script>_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""; [[ "$step" == *:* ]] && arg=${step#*:}
  case $kind in
    tests)
      # comma list: items under tests/ are files, the others -k name fragments (OR-ed)
      files=""; keys=""
      IFS=',' read -ra items <<< "$arg"
      for it in "${items[@]}"; do
        if [[ "$it" == tests/* ]]; then files="$files $it"; else keys="${keys:+$keys or }$it"; fi
      done
      sel="${files:-tests}"
      if [ -n "$keys" ]; then
        if [ -n "$files" ]; then sel="tests"; keys="$keys or $(for f in $files; do basename $f .py; done | paste -sd' ' | sed 's/ / or /g')"; fi
      fi
      timeout -k 10 1000 python -u -m pytest $sel ${keys:+-k "$keys"} -m gpu --maxfail=10 -q -rP --timeout 300 --timeout-method thread \
        > $O/tests_$n.log 2>&1 || { echo "TESTS_FAIL ($step)"; tail -40 $O/tests_$n.log; exit 1; }
      tail -1 $O/tests_$n.log ;;
    bench)
      m=${arg:-unet}
      extra=""; [ "$m" != unet ] && extra="--model $m"
      timeout -k 10 600 python -u bench.py $extra > $O/bench_$m.json 2> $O/bench_$m.err \
        || { echo "BENCH_FAIL $m"; tail -20 $O/bench_$m.err; exit 1; }
      tail -1 $O/bench_$m.json | cut -c1-240 ;;
    ab)
      m=${arg%%:*}; m=${m:-unet}
      reps=2; [[ "$arg" == *:* ]] && reps=${arg#*:}
      for i in $(seq 1 $reps); do
        (cd ab/tree && timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --steps 40) \
          > $O/ab_${m}_old_$i.log 2>&1 || { echo "AB_FAIL old $m"; tail -5 $O/ab_${m}_old_$i.log; exit 1; }
        timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --steps 40 \
          > $O/ab_${m}_new_$i.log 2>&1 || { echo "AB_FAIL new $m"; tail -5 $O/ab_${m}_new_$i.log; exit 1; }
        python tools/ab_line.py "$m rep$i" $O/ab_${m}_old_$i.log $O/ab_${m}_new_$i.log | tee -a $O/ab_summary.txt
      done ;;
    flag)
      f=${arg%%:*}; m=unet; [[ "$arg" == *:* ]] && m=${arg#*:}
      for i in 1 2; do
        for v in 0 1; do
          timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --steps 40 \
            --engine-flag $f=$v > $O/flag_${f}_${m}_${v}_$i.log 2>&1 || { echo "FLAG_FAIL $f=$v"; tail -5 $O/flag_${f}_${m}_${v}_$i.log; exit 1; }
        done
        python tools/ab_line.py "$f $m rep$i (0 vs 1)" $O/flag_${f}_${m}_0_$i.log $O/flag_${f}_${m}_1_$i.log | tee -a $O/ab_summary.txt
      done ;;
    tune)
      IFS=':' read -r key va vb tm <<< "$arg"; tm=${tm:-unet}
      for i in 1 2; do
        for v in $va $vb; do
          timeout -k 10 300 python -u bench.py --model $tm --no-cpu-baseline --no-roofline --steps 40 \
            --tune $key=$v > $O/tune_${key}_${tm}_${v}_$i.log 2>&1 || { echo "TUNE_FAIL $key=$v"; tail -5 $O/tune_${key}_${tm}_${v}_$i.log; exit 1; }
        done
        python tools/ab_line.py "tune $key $tm rep$i ($va vs $vb)" $O/tune_${key}_${tm}_${va}_$i.log $O/tune_${key}_${tm}_${vb}_$i.log | tee -a $O/ab_summary.txt
      done ;;
    prof)
      m=${arg%%:*}; m=${m:-unet}
      fl=""; [[ "$arg" == *:* ]] && fl=${arg#*:}
      t=$m${fl:+_$fl}
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o p -- \
        python -u $R/bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline \
        ${fl:+--engine-flag $fl} > $O/prof_$t.log 2>&1) \
        || { echo "PROF_FAIL $t"; tail -5 $O/prof_$t.log; exit 1; }
      find $O/prof_$t -name "*kernel_stats.csv" -exec cp {} $O/${t}_kernel_stats.csv \;
      rm -rf $O/prof_$t
      echo "prof $t done" ;;
    evidence)
      bash tools/gpu_evidence.sh $tag || exit 1 ;;
    sq)
      bash tools/gpu_sq_timing.sh $tag ${arg:-unet} > $O/sq_${arg:-unet}.out 2>&1 || { echo "SQ_FAIL"; tail -5 $O/sq_${arg:-unet}.out; exit 1; }
      echo "sq ${arg:-unet} done" ;;
    conv)
      timeout -k 10 400 python -u tools/conv_bench.py ${arg//+/ } > $O/conv_$n.log 2>&1 \
        || { echo "CONV_FAIL"; tail -10 $O/conv_$n.log; exit 1; }
      tail -3 $O/conv_$n.log ;;
    enc)
      timeout -k 10 300 python -u tools/enc_bench.py ${arg//+/ } > $O/enc_$n.log 2>&1 \
        || { echo "ENC_FAIL"; tail -10 $O/enc_$n.log; exit 1; }
      tail -3 $O/enc_$n.log ;;
    py)
      s=${arg%%:*}; a=""; [[ "$arg" == *:* ]] && a=${arg#*:}
      timeout -k 10 500 python -u tools/$s ${a//+/ } > $O/py_${n}_${s%.py}.log 2>&1 \
        || { echo "PY_FAIL $s"; tail -15 $O/py_${n}_${s%.py}.log; exit 1; }
      tail -3 $O/py_${n}_${s%.py}.log ;;
    rprof)
      s=${arg%%:*}; a=""; [[ "$arg" == *:* ]] && a=${arg#*:}
      t=${s%.py}
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rprof_$t -o p -- \
        python -u $R/tools/$s ${a//+/ } > $O/rprof_$t.log 2>&1) \
        || { echo "RPROF_FAIL $s"; tail -10 $O/rprof_$t.log; exit 1; }
      find $O/rprof_$t -name "*kernel_stats.csv" -exec cp {} $O/rprof_${t}_kernel_stats.csv \;
      rm -rf $O/rprof_$t
      echo "rprof $t done" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu_run $tag done"
