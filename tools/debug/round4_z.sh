#!/bin/bash
# round 4 GPU step z: physics-mode profile rounds (c3p with the round-4 stage kernel, c4p)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for c in c3p c4p; do
  CFG=$c timeout -k 10 600 bash tools/profile_physics.sh > gpurun_out/profile_$c.log 2>&1
  rc=$?; echo "profile $c rc=$rc"; tail -2 gpurun_out/profile_$c.log; [ $rc -eq 0 ] || exit $rc
done
