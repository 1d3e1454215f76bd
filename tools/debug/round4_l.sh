#!/bin/bash
# round 4 GPU step l: four-step launches (Euler / RK2 on dppy, x2y in fp32): parity tests, then
# pinned timings and the autotuned benches of the configs they apply to
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/all_l
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_strips.py tests/test_gpu_numerics.py -k "tb4 or four_step or x2y4 or 4" > gpurun_out/t_tb4.log 2>&1
rc=$?; echo "tb4 tests rc=$rc"; tail -4 gpurun_out/t_tb4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/pin_timing.py --config c3 --pins x2y:2:-2:0,x2y:2:24:0,x2y:4:-2:0,x2y:4:24:0,x2y:4:40:0,x2y:4:-3:0,dppy:4:-2:0 > gpurun_out/pins_l_c3.log 2>&1
echo "pins c3 rc=$?"; cat gpurun_out/pins_l_c3.log
timeout -k 10 400 python tools/pin_timing.py --config c4 --pins x2y:2:40:0,x2y:4:40:0,x2y:4:64:0,x2y:4:-2:0,x2y:4:24:0 > gpurun_out/pins_l_c4.log 2>&1
echo "pins c4 rc=$?"; cat gpurun_out/pins_l_c4.log
SPECS="c3 rk4|c4 rk4|c2 rk2|c2 euler|c1 rk4"
IFS='|'
for spec in $SPECS; do
  IFS=' ' read -r c m <<< "$spec"
  timeout -k 10 300 python bench.py --config $c --method $m --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/all_l/${c}_${m}.json 2> gpurun_out/all_l/${c}_${m}.err || { echo "$c $m failed"; tail -3 gpurun_out/all_l/${c}_${m}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/all_l/${c}_${m}.json')); r=d['roofline']
print('%-9s %-5s %8.2f Gcell/s %8.4f ms/step %s tb %s seg %s launch %.4f ms achieved %6.0f GB/s frac %.3f' % ('$c','$m',d['value']/1e9,d['ms_per_step'],r['kernel'],r['steps_per_launch'],r.get('seg_rows'),r['mean_launch_ms'],r['achieved'],r['frac']))"
done
