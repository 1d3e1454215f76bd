#!/bin/bash
# round 4 GPU step v: C2 box check (pinned chains / segments, then the default bench line)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/pin_timing.py --config c2 --pins dppy:2:-3:0,dppy:2:56:0,dppy:2:-3:0 > gpurun_out/pins_v.log 2>&1
echo "pins rc=$?"; cat gpurun_out/pins_v.log
timeout -k 10 300 python bench.py > gpurun_out/bench_v.json 2> gpurun_out/bench_v.err
echo "bench rc=$?"; cut -c1-260 gpurun_out/bench_v.json
