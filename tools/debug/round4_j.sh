#!/bin/bash
# round 4 GPU step j: the DMA prefetch stops at the cone (no HBM reads past y1 + kNS): the whole
# GPU suite, then the fused configs (autotuned)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/all_j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_j.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests_j.log; [ $rc -eq 0 ] || exit $rc
SPECS="c2 rk4|c2 rk2|c2 euler|c3 rk4|c4 rk4|c5 rk4|c2_slab8 rk4"
IFS='|'
for spec in $SPECS; do
  IFS=' ' read -r c m <<< "$spec"
  timeout -k 10 300 python bench.py --config $c --method $m --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/all_j/${c}_${m}.json 2> gpurun_out/all_j/${c}_${m}.err || { echo "$c $m failed"; tail -3 gpurun_out/all_j/${c}_${m}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/all_j/${c}_${m}.json')); r=d['roofline']
print('%-9s %-5s %8.2f Gcell/s %8.4f ms/step %s seg %s launch %.4f ms achieved %6.0f GB/s frac %.3f' % ('$c','$m',d['value']/1e9,d['ms_per_step'],r['kernel'],r.get('seg_rows'),r['mean_launch_ms'],r['achieved'],r['frac']))"
done
