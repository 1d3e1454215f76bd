#!/bin/bash
# round 4 GPU step o: deferred row stores (WS_DPPY_DEFER=1, variant library built from the fp64
# two-step TU): bitwise parity of the fp64 dppy two-step paths, then pinned C2 timings against
# the product library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
V=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_defer.so
B=$PWD/nvidia-jetson-workload_amd/lib/libws_hip.so
WS_HIP_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_strips.py -k "dppy_tb2 or (full_size and (2 or chain)) or long_horizon or tiling" > gpurun_out/t_defer.log 2>&1
rc=$?; echo "defer tests rc=$rc"; tail -3 gpurun_out/t_defer.log; [ $rc -eq 0 ] || exit $rc
for v in base defer base defer; do
  if [ $v = base ]; then L=$B; else L=$V; fi
  WS_HIP_LIB=$L timeout -k 10 300 python tools/pin_timing.py --config c2 --pins dppy:2:-2:0,dppy:2:56:0,dppy:2:-3:0 > gpurun_out/pins_o_$v.log 2>&1
  rc=$?; echo "pins $v rc=$rc"; cat gpurun_out/pins_o_$v.log; [ $rc -eq 0 ] || exit $rc
done
WS_HIP_LIB=$V timeout -k 10 300 python tools/pin_timing.py --config c2 --method rk2 --pins dppy:2:-2:0,dppy:2:88:0 > gpurun_out/pins_o_rk2.log 2>&1
echo "rk2 defer rc=$?"; cat gpurun_out/pins_o_rk2.log
WS_HIP_LIB=$B timeout -k 10 300 python tools/pin_timing.py --config c2 --method rk2 --pins dppy:2:-2:0,dppy:2:88:0 > gpurun_out/pins_o_rk2b.log 2>&1
echo "rk2 base rc=$?"; cat gpurun_out/pins_o_rk2b.log
