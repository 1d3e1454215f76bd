#!/bin/bash
# GPU: parity suite, then the C2 autotune table (WS_AUTOTUNE=2) and a bench line per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tb; mkdir -p $OUT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for spec in ${CFGS:-c2:rk4}; do
  c=${spec%%:*}; m=${spec##*:}
  WS_AUTOTUNE=2 timeout -k 10 300 python bench.py --config $c --method $m --steps ${STEPS:-200} --warmup ${WARM:-300} --no-cpu-baseline > $OUT/${c}_$m.json 2> $OUT/${c}_$m.err
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -5 $OUT/${c}_$m.err; exit $rc; }
  grep "autotune" $OUT/${c}_$m.err | sort -t' ' -k11 -n | head -8
  python3 -c "
import json; d=json.load(open('$OUT/${c}_$m.json')); r=d['roofline']
print('%-10s %-6s %7.2f Gcell/s %8.4f ms/step  kernel %s seg %s cols %s %.4f ms/launch %6.0f GB/s frac %.3f' % ('$c','$m',d['value']/1e9,d['ms_per_step'],r['kernel'],r.get('seg_rows'),r.get('strip_out_cols'),r['mean_launch_ms'],r['achieved'],r['frac']))"
done
