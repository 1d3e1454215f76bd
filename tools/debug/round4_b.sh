#!/bin/bash
# round 4 GPU step b: the bvort stage-kernel fix (prefetched z0 / accumulator, no store switch)
# against its oracle, then the per-wave timeline of the chain schedule vs segments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bvort.py > gpurun_out/t_bvort.log 2>&1
rc=$?; echo "bvort tests rc=$rc"; tail -3 gpurun_out/t_bvort.log; [ $rc -eq 0 ] || exit $rc
WS_HIP_LIB=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_stamps.so timeout -k 10 300 python tools/wave_timeline.py \
    --pins dppy:2:48:0,dppy:2:-2:0,dppy:2:-3:0,x2y:2:-2:0 --json gpurun_out/timeline_c2b.json > gpurun_out/timeline_c2b.log 2>&1
echo "timeline rc=$?"
timeout -k 10 60 tools/issue_probe > gpurun_out/issue_probe.log 2>&1
echo "probe rc=$?"; cat gpurun_out/issue_probe.log
