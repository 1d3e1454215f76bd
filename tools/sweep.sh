#!/bin/bash
# Quick A/B sweep of bench.py variants on the GPU box (compact one-line results).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
STEPS=${STEPS:-50}
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  env $line timeout -k 10 180 python bench.py --steps $STEPS --warmup ${WARM:-300} --no-cpu-baseline ${ARGS:-} > $OUT/r$i.json 2> $OUT/r$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$line] rc=$rc"; tail -3 $OUT/r$i.err; exit $rc; fi
  python -c "
import json; d=json.load(open('$OUT/r$i.json'))
print('%-60s %8.2f Gcell/s %7.4f ms/step  kernel %6.0f GB/s (%.3f)' % ('$line', d['value']/1e9, d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac']))"
done < "${1:-/dev/stdin}"
