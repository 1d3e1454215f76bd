#!/bin/bash
# Short bench lines for a list of configs (no CPU baseline): CFGS="c2:rk4 c2_slab8:rk4" bash tools/quick_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
for spec in ${CFGS:-c2:rk4 c2_slab8:rk4}; do
  c=${spec%%:*}; m=${spec##*:}
  timeout -k 10 200 python bench.py --config $c --method $m --steps ${STEPS:-200} --warmup ${WARM:-300} --no-cpu-baseline > gpurun_out/q/${c}_$m.json 2> gpurun_out/q/${c}_$m.err || { echo "$spec failed"; tail -5 gpurun_out/q/${c}_$m.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/q/${c}_$m.json')); r=d['roofline']
print('%-10s %-6s %7.2f Gcell/s %8.4f ms/step  kernel %s seg %s cols %s %.4f ms %6.0f GB/s frac %.3f' % ('$c','$m',d['value']/1e9,d['ms_per_step'],r['kernel'],r.get('seg_rows'),r.get('strip_out_cols'),r['mean_launch_ms'],r['achieved'],r['frac']))"
done
