#!/bin/bash
# round 4 GPU step m (final tree): the whole GPU suite, smoke, the C4 profile round (four-step
# launches), every bench configuration + slab rank timing, then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
CFG=c4 METHOD=rk4 timeout -k 10 420 bash tools/profile_round.sh > gpurun_out/profile_c4.log 2>&1
rc=$?; echo "profile c4 rc=$rc"; tail -1 gpurun_out/profile_c4.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/debug/round4_g.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo "bench rc=$?"; cut -c1-400 gpurun_out/bench_default.json
