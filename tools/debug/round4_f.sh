#!/bin/bash
# round 4 GPU step f: the whole GPU suite, smoke, then the C2 profile round (bench, rocprofv3
# kernel stats, PMC passes incl. the VALU type split)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
CFG=c2 METHOD=rk4 timeout -k 10 900 bash tools/profile_round.sh > gpurun_out/profile_c2.log 2>&1
echo "profile rc=$?"; tail -5 gpurun_out/profile_c2.log
