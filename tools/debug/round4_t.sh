#!/bin/bash
# round 4 GPU step t (final tree): the whole GPU suite, smoke, profile rounds of C2 / C3 / C4,
# every bench configuration + slab rank timing, then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c4; do
  CFG=$c METHOD=rk4 timeout -k 10 420 bash tools/profile_round.sh > gpurun_out/profile_$c.log 2>&1
  rc=$?; echo "profile $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/debug/round4_g.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo "bench rc=$?"; cut -c1-300 gpurun_out/bench_default.json
