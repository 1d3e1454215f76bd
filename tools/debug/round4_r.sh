#!/bin/bash
# round 4 GPU step r: per-wave timeline of the C3 fp32 pair launch (x2y, two steps; chains and
# 24-row segments) from a -DWS_WAVE_STAMPS build of the fp32 pair TU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
WS_HIP_LIB=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_stamps32.so timeout -k 10 300 python tools/wave_timeline.py --config c3 --pins x2y:2:-2:0,x2y:2:24:0,x2y:2:-2:0 --json gpurun_out/timeline_c3.json > gpurun_out/timeline_c3.log 2>&1
echo "timeline rc=$?"; cut -c1-900 gpurun_out/timeline_c3.log
