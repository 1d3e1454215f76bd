#!/bin/bash
# GPU: overlap-schedule parity tests, then the one-GPU slab-schedule emulation with and
# without the overlap schedule (tools/group_timing.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_slab_overlap.py tests/test_gpu_slab_rccl.py -x -q --timeout 120 --timeout-method thread > $OUT/ovl_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/ovl_tests.log
[ $rc -eq 0 ] || exit $rc
for o in 0 1; do
  WS_SLAB_OVERLAP=$o timeout -k 10 200 python tools/group_timing.py --slabs ${SLABS:-2,4,8} --steps 120 > $OUT/ovl_timing_$o.txt 2>&1
  rc=$?; echo "overlap=$o rc=$rc"; cat $OUT/ovl_timing_$o.txt
  [ $rc -eq 0 ] || exit $rc
done
