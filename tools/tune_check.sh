#!/bin/bash
# Autotuner check: the choice and its table for the bench configs (WS_AUTOTUNE=2), then c3p.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tune; mkdir -p $OUT
for c in ${CFGS:-c2 c2_slab8}; do
  for rep in 1 2; do
    WS_AUTOTUNE=2 timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${c}_$rep.json 2> $OUT/${c}_$rep.err || { tail -5 $OUT/${c}_$rep.err; exit 1; }
    grep chosen $OUT/${c}_$rep.err
    python3 -c "import json; d=json.load(open('$OUT/${c}_$rep.json')); r=d['roofline']; print('$c', '%.2f Gcell/s %.4f ms/step launch %.4f' % (d['value']/1e9, d['ms_per_step'], r['mean_launch_ms']))"
  done
done
