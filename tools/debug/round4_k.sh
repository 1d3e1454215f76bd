#!/bin/bash
# round 4 GPU step k: profile rounds (bench, rocprofv3 kernel stats, PMC traffic / VALU passes)
# of C2, C3, C4 and C5 with the cone-bounded prefetch, then every bench configuration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for c in c2 c3 c4 c5; do
  CFG=$c METHOD=rk4 timeout -k 10 420 bash tools/profile_round.sh > gpurun_out/profile_$c.log 2>&1
  rc=$?; echo "profile $c rc=$rc"; tail -1 gpurun_out/profile_$c.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
bash tools/debug/round4_g.sh
