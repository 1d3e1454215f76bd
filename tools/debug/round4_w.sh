#!/bin/bash
# round 4 GPU step w: LDS-DMA prefetch distance of the fp64 two-step march under the chain
# schedule (WS_DPPY_PF = 1 / 3 groups vs the product's 2), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in base pf3 pf1 base pf3 pf1; do
  if [ $v = base ]; then L=$PWD/nvidia-jetson-workload_amd/lib/libws_hip.so; else L=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_$v.so; fi
  WS_HIP_LIB=$L timeout -k 10 300 python tools/pin_timing.py --config c2 --pins dppy:2:-3:0,dppy:2:-4:0 > gpurun_out/pins_w_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; cat gpurun_out/pins_w_$v.log; [ $rc -eq 0 ] || exit $rc
done
