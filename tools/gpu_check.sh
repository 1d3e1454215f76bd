#!/bin/bash
# GPU-box validation round: parity tests, smoke, short bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/timeout (rc not in {0,1}) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-20}
WARM=${WARM:-5}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

timeout -k 10 ${PYTEST_T:-400} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
ok $rc || exit $rc

timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
ok $rc || exit $rc

timeout -k 10 400 python bench.py --steps $STEPS --warmup $WARM ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
[ "$rc" -eq 0 ] || exit $rc

if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python "$R/bench.py" --steps $STEPS --warmup $WARM --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc"
  find "$OUT/prof" -name "*stats*" | head
fi
