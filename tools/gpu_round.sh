#!/bin/bash
# The one GPU-box script of a round (replaces round 4's per-lease step scripts):
#
#   bash tools/gpu_round.sh STEP [STEP ...]
#
#   tests[:PYTEST_ARGS]   pytest -m gpu (args, comma-separated: e.g. tests:tests/test_gpu_multi.py)
#   smoke                 __graft_entry__.smoke()
#   bench                 the default bench line (python bench.py), JSON under gpurun_out/
#   configs[:LIST]        bench lines for LIST (cfg:method,...; default: every configuration)
#   profile:CFG:METHOD    tools/profile_round.sh (autotuned bench, rocprofv3 kernel stats, PMC passes)
#   physics:CFG           tools/profile_physics.sh (c3p / c4p)
#   rank:CFG[:RANKS]      tools/rank_timing.py (one rank's slab, emulated transfers 0 / 40 / 80 us)
#   prof_default          rocprofv3 --kernel-trace --stats of the default bench command itself
#   pin:CFG:PINS          tools/pin_timing.py (ms/step of pinned variants, one process)
#   lpeslabs[:LIST]       c4p bench lines at N slabs of the ring decomposition on this GPU (default 1,2,8)
#   bvslabs[:LIST]        the same for c3p (the vorticity model's decomposition)
#
# Every step runs under its own time limit; the first failing step ends the script (a GPU
# fault, abort or time limit must not be followed by more GPU work in the same call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-200}
WARM=${WARM:-300}

fail() { echo "step '$1' failed (rc=$2)"; exit "$2"; }

for step in "$@"; do
  IFS=':' read -r name a1 a2 <<< "$step"
  rest=""; [[ "$step" == *:* ]] && rest=${step#*:}   # everything after the step name
  echo "== $step"
  case "$name" in
    tests)
      args=${rest//,/ }
      timeout -k 10 ${PYTEST_T:-900} python -u -m pytest ${args:-tests} -m gpu -x -q --timeout 150 --timeout-method thread \
          > "$OUT/gpu_tests.log" 2>&1
      rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    bench)
      timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
      rc=$?; cut -c1-400 "$OUT/bench_default.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_default.err"; fail "$step" $rc; } ;;
    configs)
      list=${rest:-c1:rk4,c2:rk4,c2:rk2,c2:euler,c3:rk4,c4:rk4,c5:rk4,c2_slab2:rk4,c2_slab4:rk4,c2_slab8:rk4,c3p:rk4,c4p:rk4}
      mkdir -p "$OUT/all"
      for spec in ${list//,/ }; do
        c=${spec%%:*}; m=${spec#*:}
        timeout -k 10 300 python bench.py --config $c --method $m --steps $STEPS --warmup $WARM --no-cpu-baseline \
            > "$OUT/all/${c}_${m}.json" 2> "$OUT/all/${c}_${m}.err"
        rc=$?; [ $rc -eq 0 ] || { tail -3 "$OUT/all/${c}_${m}.err"; fail "$step ($c $m)" $rc; }
        python3 -c "
import json; d=json.load(open('$OUT/all/${c}_${m}.json')); r=d['roofline']
print('%-9s %-5s %8.2f Gcell/s %8.4f ms/step %s tb %s seg %s launch %.4f ms frac %.3f' % ('$c','$m',d['value']/1e9,
      d['ms_per_step'],r['kernel'],r.get('steps_per_launch'),r.get('seg_rows'),r['mean_launch_ms'],r['frac']))"
      done ;;
    profile)
      CFG=$a1 METHOD=${a2:-rk4} timeout -k 10 1000 bash tools/profile_round.sh > "$OUT/profile_${a1}_${a2:-rk4}.log" 2>&1
      rc=$?; tail -3 "$OUT/profile_${a1}_${a2:-rk4}.log"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    physics)
      CFG=$a1 timeout -k 10 600 bash tools/profile_physics.sh > "$OUT/profile_$a1.log" 2>&1
      rc=$?; tail -2 "$OUT/profile_$a1.log"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    rank)
      timeout -k 10 500 python tools/rank_timing.py --config ${a1:-c2} --ranks ${a2:-2,4,8} --xfer-us 0,40,80 \
          --variants off,on,auto > "$OUT/rank_timing_${a1:-c2}.txt" 2>&1
      rc=$?; cat "$OUT/rank_timing_${a1:-c2}.txt"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    pin)
      timeout -k 10 500 python tools/pin_timing.py --config $a1 --pins "$a2" > "$OUT/pin_${a1}.txt" 2>&1
      rc=$?; cat "$OUT/pin_${a1}.txt"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    prof_default)
      mkdir -p "$OUT/prof_default"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_default" -o run \
          --output-format csv -- python3 "$R/bench.py" > "$OUT/prof_default/bench.json" 2> "$OUT/prof_default/bench.err")
      rc=$?; cut -c1-200 "$OUT/prof_default/bench.json"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    lpeslabs|bvslabs)
      c=$([ "$name" = lpeslabs ] && echo c4p || echo c3p)
      mkdir -p "$OUT/$c"
      for n in $(echo "${rest:-1,2,8}" | tr ',' ' '); do
        timeout -k 10 300 python bench.py --config $c --slabs $n --steps 100 --warmup 20 --no-cpu-baseline \
            > "$OUT/$c/slabs$n.json" 2> "$OUT/$c/slabs$n.err"
        rc=$?; [ $rc -eq 0 ] || { tail -3 "$OUT/$c/slabs$n.err"; fail "$step (slabs $n)" $rc; }
        python3 -c "import json; d=json.load(open('$OUT/$c/slabs$n.json')); print('$c', '$n', d['value']/1e9, d['ms_per_step'], d['config']['parallelism'])"
      done ;;
    *)
      echo "unknown step '$step'"; exit 2 ;;
  esac
done
