#!/bin/bash
# round 4 GPU step p: cached output stores for the fp32 pair kernel (WS_F32_STORE_POL=0 variant
# of the x2y fp32 two- and four-step TUs): parity, then C3 / C4 pinned timings vs the product
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
V=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_f32c.so
B=$PWD/nvidia-jetson-workload_amd/lib/libws_hip.so
WS_HIP_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "x2y_tb2 or x2y_tb4 or x2y4" > gpurun_out/t_f32c.log 2>&1
rc=$?; echo "f32c tests rc=$rc"; tail -2 gpurun_out/t_f32c.log; [ $rc -eq 0 ] || exit $rc
for v in base f32c base f32c; do
  if [ $v = base ]; then L=$B; else L=$V; fi
  WS_HIP_LIB=$L timeout -k 10 300 python tools/pin_timing.py --config c3 --pins x2y:2:-2:0,x2y:2:24:0,x2y:4:24:0 > gpurun_out/pins_p_c3_$v.log 2>&1
  rc=$?; echo "c3 $v rc=$rc"; cat gpurun_out/pins_p_c3_$v.log; [ $rc -eq 0 ] || exit $rc
  WS_HIP_LIB=$L timeout -k 10 300 python tools/pin_timing.py --config c4 --pins x2y:4:40:0,x2y:4:56:0 > gpurun_out/pins_p_c4_$v.log 2>&1
  rc=$?; echo "c4 $v rc=$rc"; cat gpurun_out/pins_p_c4_$v.log; [ $rc -eq 0 ] || exit $rc
done
