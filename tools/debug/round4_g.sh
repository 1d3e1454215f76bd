#!/bin/bash
# round 4 GPU step g: every bench configuration (autotuned) and the slab-share rank timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/all
SPECS="c1 rk4|c2 rk4|c2 rk2|c2 euler|c3 rk4|c4 rk4|c5 rk4|c2_slab2 rk4|c2_slab4 rk4|c2_slab8 rk4|c3p rk4|c4p rk4"
IFS='|'
for spec in $SPECS; do
  IFS=' ' read -r c m <<< "$spec"
  timeout -k 10 300 python bench.py --config $c --method $m --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/all/${c}_${m}.json 2> gpurun_out/all/${c}_${m}.err || { echo "$c $m failed"; tail -3 gpurun_out/all/${c}_${m}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/all/${c}_${m}.json')); r=d['roofline']
print('%-9s %-5s %8.2f Gcell/s %8.4f ms/step %s seg %s launch %.4f ms achieved %6.0f GB/s frac %.3f' % ('$c','$m',d['value']/1e9,d['ms_per_step'],r['kernel'],r.get('seg_rows'),r['mean_launch_ms'],r['achieved'],r['frac']))"
done
unset IFS
timeout -k 10 400 python tools/rank_timing.py --config c2 --ranks 2,4,8 --xfer-us 0,40,80 --variants off,on,auto > gpurun_out/rank_timing_c2.txt 2>&1
echo "rank c2 rc=$?"; cat gpurun_out/rank_timing_c2.txt
