#!/bin/bash
# round 4 GPU step y: chains priced dearer on XCDs 6 / 7 (measurement builds of ws_schedule.cpp:
# xw12 = 1.12 / 1.12, xw20 = 1.2 / 1.1) against the product, C2 and C3, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in base xw12 xw20 base xw12 xw20; do
  if [ $v = base ]; then L=$PWD/nvidia-jetson-workload_amd/lib/libws_hip.so; else L=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_$v.so; fi
  WS_HIP_LIB=$L timeout -k 10 300 python tools/pin_timing.py --config c2 --pins dppy:2:-3:0 > gpurun_out/pins_y_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; cat gpurun_out/pins_y_$v.log; [ $rc -eq 0 ] || exit $rc
  WS_HIP_LIB=$L timeout -k 10 300 python tools/pin_timing.py --config c3 --pins x2y:4:-2:0 > gpurun_out/pins_y3_$v.log 2>&1
  cat gpurun_out/pins_y3_$v.log
done
