#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no tracing domains) over a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/pmc${TAG:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/bench.py" --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" | tee "$OUT/summary.txt"
