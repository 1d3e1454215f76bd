#!/bin/bash
# round 4 GPU step aa: eight-step Euler launches: parity (stepping fixtures, strips, the launch
# counts, full-size digests incl. C1 Euler), then C2 / C1 Euler timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/all_aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_strips.py -k "tb8 or four_step or full_size or slab_group" > gpurun_out/t_tb8.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_tb8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pin_timing.py --config c2 --method euler --pins dppy:4:72:0,dppy:8:-3:0,dppy:8:40:0,dppy:8:-2:0 > gpurun_out/pins_aa.log 2>&1
echo "pins rc=$?"; cat gpurun_out/pins_aa.log
for spec in "c2 euler" "c1 euler"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --method $2 --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/all_aa/$1_$2.json 2> gpurun_out/all_aa/$1_$2.err || { echo "$spec failed"; tail -3 gpurun_out/all_aa/$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/all_aa/$1_$2.json')); r=d['roofline']
print('$1 $2: %.2f Gcell/s %.4f ms/step %s tb %s seg %s' % (d['value']/1e9,d['ms_per_step'],r['kernel'],r['steps_per_launch'],r.get('seg_rows')))"
done
