#!/bin/bash
# round 4 GPU step x: C3 variant / schedule sweep (chains per SIMD, four-step launches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python tools/pin_timing.py --config c3 --pins x2y:4:-2:0,x2y:4:-3:0,x2y:2:-3:0,dppy:4:-2:0,dppy:4:-3:0,dppy:2:-3:0,pc2:2:-2:0,pc2:2:-3:0,pc:2:-3:0,pc:2:-5:0,x2y:4:8:0,x2y:4:16:0,x2y:4:-2:0 > gpurun_out/pins_x_c3.log 2>&1
echo "c3 rc=$?"; cat gpurun_out/pins_x_c3.log
