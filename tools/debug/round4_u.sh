#!/bin/bash
# round 4 GPU step u: which chain candidate fails at C5 (16384^2): one pin per process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for p in dppy:2:-2:0 dppy:2:-7:0 pc2:2:-2:0 pc2:2:-7:0 x2y:2:-2:0 x2y:2:-7:0 pc:2:-2:0 dppy:1:-2:0 x2y:1:-2:0 x2y:1:-7:0; do
  timeout -k 10 120 python tools/pin_timing.py --config c5 --steps 4 --pins $p > gpurun_out/u_$p.log 2>&1
  echo "$p rc=$?"; grep -E "ms/step|Error" gpurun_out/u_$p.log | tail -1 | cut -c1-200
done
