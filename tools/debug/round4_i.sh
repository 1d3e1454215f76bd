#!/bin/bash
# round 4 GPU step i: slab schedule tests + auto choice on emulated ranks; scheduler-strategy
# variants of the fp64 two-step kernel (tools/variant.sh maxilp / itilp)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_slab_overlap.py tests/test_gpu_slab_rccl.py tests/test_gpu_selfcheck.py > gpurun_out/t_slab.log 2>&1
rc=$?; echo "slab tests rc=$rc"; tail -3 gpurun_out/t_slab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/rank_timing.py --config c2 --ranks 2,4,8 --xfer-us 0,40,80 --variants off,on,auto > gpurun_out/rank_timing_c2.txt 2>&1
echo "rank c2 rc=$?"; cat gpurun_out/rank_timing_c2.txt
for v in base maxilp itilp base; do
  if [ $v = base ]; then L="$PWD/nvidia-jetson-workload_amd/lib/libws_hip.so"; else L="$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_$v.so"; fi
  WS_HIP_LIB=$L timeout -k 10 200 python tools/pin_timing.py --config c2 --pins dppy:2:-2:0,dppy:2:56:0 > gpurun_out/pins_i_$v.log 2>&1
  rc=$?; echo "pins $v rc=$rc"; cat gpurun_out/pins_i_$v.log; [ $rc -eq 0 ] || exit $rc
done
