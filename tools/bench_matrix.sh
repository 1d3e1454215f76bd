#!/bin/bash
# Bench lines for a matrix of configs x environment settings (no CPU baseline), one JSON line
# each under gpurun_out/m/, plus a one-line summary per run on stdout:
#   RUNS="c2:rk4:WS_NUMERICS=exact c2:rk4:WS_NUMERICS=fast,WS_KERNEL=dppy" bash tools/bench_matrix.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/m
i=0
for spec in ${RUNS:-c2:rk4:}; do
  i=$((i+1))
  IFS=: read -r c m envs <<< "$spec"
  tag="${i}_${c}_${m}"
  ( [ -n "$envs" ] && export ${envs//,/ }
    timeout -k 10 ${BENCH_T:-240} python bench.py --config $c --method $m --steps ${STEPS:-200} --warmup ${WARM:-300} \
        --no-cpu-baseline > gpurun_out/m/$tag.json 2> gpurun_out/m/$tag.err ) || { echo "$spec failed"; tail -5 gpurun_out/m/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/m/$tag.json')); r=d['roofline']
print('%-10s %-5s %-40s %7.2f Gcell/s %8.4f ms/step  %s seg %s cols %s %.4f ms frac %.3f' % ('$c','$m','$envs',d['value']/1e9,d['ms_per_step'],r['kernel'],r.get('seg_rows'),r.get('strip_out_cols'),r['mean_launch_ms'],r['frac']))"
done
