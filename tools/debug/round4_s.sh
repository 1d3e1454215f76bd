#!/bin/bash
# round 4 GPU step s: chain counts in waves per SIMD (1, 2, 3, 4, 6) instead of rounds of the
# kernel's occupancy: chain parity tests, pinned C3 / C2 / C4 timings, autotuned benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/all_s
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_slab_overlap.py -k "chain or tiling or full_size or slab" > gpurun_out/t_chainsimd.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_chainsimd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pin_timing.py --config c3 --pins x2y:2:24:0,x2y:2:-2:0,x2y:2:-3:0,x2y:2:-4:0,x2y:4:-2:0,x2y:4:-3:0 > gpurun_out/pins_s_c3.log 2>&1
echo "c3 rc=$?"; cat gpurun_out/pins_s_c3.log
timeout -k 10 300 python tools/pin_timing.py --config c2 --pins dppy:2:-2:0,dppy:2:-3:0,dppy:2:-5:0,pc:2:-3:0,pc:2:-5:0 > gpurun_out/pins_s_c2.log 2>&1
echo "c2 rc=$?"; cat gpurun_out/pins_s_c2.log
timeout -k 10 300 python tools/pin_timing.py --config c4 --pins x2y:4:56:0,x2y:4:-2:0,x2y:4:-3:0,x2y:4:-4:0 > gpurun_out/pins_s_c4.log 2>&1
echo "c4 rc=$?"; cat gpurun_out/pins_s_c4.log
for c in c3 c2 c4 c2_slab8; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/all_s/${c}_rk4.json 2> gpurun_out/all_s/${c}_rk4.err || { echo "$c failed"; tail -3 gpurun_out/all_s/${c}_rk4.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/all_s/${c}_rk4.json')); r=d['roofline']
print('%-9s %8.2f Gcell/s %8.4f ms/step %s tb %s seg %s launch %.4f ms' % ('$c',d['value']/1e9,d['ms_per_step'],r['kernel'],r['steps_per_launch'],r.get('seg_rows'),r['mean_launch_ms']))"
done
