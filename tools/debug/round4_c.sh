#!/bin/bash
# round 4 GPU step c: per-wave timeline of the chain schedule (rows, XCD, edge strips), table
# in order and reversed (does the slow tail follow the rows or the XCDs?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
V=$PWD/nvidia-jetson-workload_amd/lib/variants
WS_HIP_LIB=$V/libws_hip_stamps.so timeout -k 10 300 python tools/wave_timeline.py \
    --pins dppy:2:48:0,dppy:2:-2:0,dppy:2:-3:0 --json gpurun_out/timeline_c2c.json > gpurun_out/timeline_c2c.log 2>&1
echo "timeline rc=$?"
WS_HIP_LIB=$V/libws_hip_stampsrev.so timeout -k 10 300 python tools/wave_timeline.py \
    --pins dppy:2:-2:0 --json gpurun_out/timeline_c2rev.json > gpurun_out/timeline_c2rev.log 2>&1
echo "timeline rev rc=$?"
