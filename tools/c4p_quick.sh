#!/bin/bash
# c4p (physics-mode layered PE) check: GPU tests, bench, rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/c4pq; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_layered_pe.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config c4p --steps 100 --warmup 50 --no-cpu-baseline > $OUT/bench.json 2>$OUT/bench.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('c4p', d['value']/1e9, d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c4p --steps 50 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')): print(r['Name'][:40], r['Calls'], r['AverageNs'])"
