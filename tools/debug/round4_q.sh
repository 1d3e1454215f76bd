#!/bin/bash
# round 4 GPU step q: the PE T / P drift applied once per run (tp_flush): the parity suites that
# cover PE (fixtures, alternation, stale handle, C4 per-level digests, slab groups, overlap),
# then the C4 bench against the previous tree's 0.0947 ms/step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/all_q
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_slab_overlap.py tests/test_gpu_output.py tests/test_gpu_doc_examples.py > gpurun_out/t_tp.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_tp.log; [ $rc -eq 0 ] || exit $rc
for c in c4; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/all_q/${c}_rk4.json 2> gpurun_out/all_q/${c}_rk4.err || { echo "$c failed"; tail -3 gpurun_out/all_q/${c}_rk4.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/all_q/${c}_rk4.json')); r=d['roofline']
print('%-9s %8.2f Gcell/s %8.4f ms/step %s tb %s seg %s launch %.4f ms' % ('$c',d['value']/1e9,d['ms_per_step'],r['kernel'],r['steps_per_launch'],r.get('seg_rows'),r['mean_launch_ms']))"
done
timeout -k 10 300 python tools/pin_timing.py --config c4 --pins x2y:4:40:0,x2y:4:56:0 > gpurun_out/pins_q_c4.log 2>&1
echo "pins rc=$?"; cat gpurun_out/pins_q_c4.log
