#!/bin/bash
# round 4 GPU step e: schedule / variant timings on C2, C3, C4 and the C2 8-slab share
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
P="timeout -k 10 300 python tools/pin_timing.py"
$P --config c2 --pins auto,dppy:2:56:0,dppy:2:-2:0,dppy:2:-3:0,pc:2:-2:0,pc2:2:-2:0 > gpurun_out/pins_e_c2.log 2>&1; echo "c2 rc=$?"; cat gpurun_out/pins_e_c2.log
$P --config c3 --pins auto,x2y:2:24:0,x2y:2:-2:0,x2y:2:-3:0,x2y:2:-4:0,dppy:2:-2:0,dppy:2:-3:0,pc2:2:-2:0,pc:2:-3:0 > gpurun_out/pins_e_c3.log 2>&1; echo "c3 rc=$?"; cat gpurun_out/pins_e_c3.log
$P --config c4 --steps 100 --warmup 200 --pins auto,x2y:2:24:0,x2y:2:-2:0,x2y:2:-3:0,dppy:2:-3:0,pc2:2:-2:0,pc:2:-3:0 > gpurun_out/pins_e_c4.log 2>&1; echo "c4 rc=$?"; cat gpurun_out/pins_e_c4.log
$P --config c2_slab8 --pins auto,dppy:2:24:0,pc:2:24:0,dppy:2:-2:0,dppy:2:-3:0,pc:2:-2:0,pc:2:-3:0,dppy:1:-2:0,dppy:1:-3:0,x2y:1:-2:0 > gpurun_out/pins_e_s8.log 2>&1; echo "s8 rc=$?"; cat gpurun_out/pins_e_s8.log
