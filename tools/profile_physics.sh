#!/bin/bash
# Physics-mode configs (c3p, c4p): bench -> rocprofv3 kernel stats -> FETCH / WRITE passes ->
# traffic per step (tools/traffic_step.py). Outputs under gpurun_out/phys_<cfg>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
CFG=${CFG:-c3p}; METHOD=${METHOD:-rk4}; STEPS=${STEPS:-50}; WARM=${WARM:-20}
OUT=$R/gpurun_out/phys_$CFG; mkdir -p "$OUT/pmc"
SUBS=${SUBS:-"bv_ lpe_"}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $CFG --method $METHOD --steps $STEPS --warmup $WARM --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc/p$i" -o run -- \
      python3 "$R/bench.py" --config $CFG --method $METHOD --steps 10 --warmup 0 --no-cpu-baseline > "$OUT/pmc/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc/p$i.log"; exit $rc; }
done
python3 "$R/tools/traffic_step.py" "$OUT/pmc" 10 "$OUT/traffic_${CFG}_${METHOD}.json" $SUBS
python3 "$R/tools/pmc_summary.py" "$OUT/pmc" > "$OUT/pmc_summary.txt"
