#!/bin/bash
# c4p A/B on one box: total-thickness carry between stages on / off (WS_LPE_TOTALS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c4pab; mkdir -p $OUT
for rep in 1 2; do for t in 1 0; do
  WS_LPE_TOTALS=$t timeout -k 10 200 python bench.py --config c4p --steps 100 --warmup 50 --no-cpu-baseline > $OUT/t$t.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/t$t.json')); print('totals $t', '%.2f Gcell/s %.4f ms' % (d['value']/1e9, d['ms_per_step']))"
done; done
