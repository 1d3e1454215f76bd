#!/bin/bash
# Every bench configuration on one GPU (autotuned), long warm-up, JSON per line into
# gpurun_out/all/. Usage: bash tools/measure_all.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/all
mkdir -p $OUT
for spec in ${SPECS:-"c2 rk4" "c2 rk2" "c2 euler" "c3 rk4" "c4 rk4" "c5 rk4" "c2_slab2 rk4" "c2_slab4 rk4" "c2_slab8 rk4" "c3p rk4" "c4p rk4"}; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --method $2 --steps ${STEPS:-200} --warmup ${WARM:-300} \
      ${CPU:---no-cpu-baseline} > $OUT/$1_$2.json 2> $OUT/$1_$2.err
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -3 $OUT/$1_$2.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$OUT/$1_$2.json')); r=d['roofline']
print('%-10s %-6s %7.2f Gcell/s %8.4f ms/step  kernel %s seg %s %.4f ms %6.0f GB/s frac %.3f' % ('$1','$2',d['value']/1e9,d['ms_per_step'],r['kernel'][:24],r.get('seg_rows'),r['mean_launch_ms'],r['achieved'],r['frac']))"
done
