#!/bin/bash
# round 4 GPU step d: chain / steal parity, then C2 timings of the schedules
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "long_horizon or (tiling and (-2 or -4 or -12)) or (full_size and (chain or steal))" > gpurun_out/t_steal.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_steal.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pin_timing.py --config c2 --pins auto,dppy:2:56:0,dppy:2:-2:0,dppy:2:-12:0,dppy:2:-13:0,x2y:2:-12:0,pc:2:-2:0 > gpurun_out/pins_c2d.log 2>&1
echo "pins rc=$?"; cat gpurun_out/pins_c2d.log
