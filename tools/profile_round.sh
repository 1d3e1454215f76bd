#!/bin/bash
# Round profile of the bench workload: bench (autotuned) -> rocprofv3 kernel-trace stats and
# PMC passes with the variant the autotuner chose pinned (so every profiled dispatch of the
# kernel is the measured one) -> traffic JSON. Outputs under gpurun_out/round_<cfg>_<method>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
CFG=${CFG:-c2}; METHOD=${METHOD:-rk4}; STEPS=${STEPS:-200}; WARM=${WARM:-300}
OUT=$R/gpurun_out/round_${CFG}_${METHOD}
mkdir -p "$OUT/pmc"
timeout -k 10 400 python bench.py --config $CFG --method $METHOD --steps $STEPS --warmup $WARM > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; }
read KERN KNAME SEG ALIGN TB < <(python3 -c "
import json; d=json.load(open('$OUT/bench.json'))['roofline']
k={'fused_dppy':'dppy','fused_x2y':'x2y','fused_pc':'pc','fused_pc2':'pc2','fused_lds':'lds'}.get(d['kernel'],'dppy')
n={'dppy':'fused_dppy_kernel','x2y':'fused_dppy_kernel','pc':'fused_dppy_kernel','pc2':'fused_dppy_kernel','lds':'fused_step_kernel'}[k]
tb=d.get('steps_per_launch') or 1
nst={'euler':1,'rk2':2,'rk4':4}['$METHOD']
nst=2 if nst==4 and '$CFG' in ('c3','c4') else nst
cone=nst*tb
g=16//(8 if '$CFG' in ('c2','c5') or '$CFG'.startswith('c2_') else 4)
margin=(cone+g-1)//g*g if k in ('dppy','x2y','pc','pc2') else cone
full={'dppy':64,'x2y':128,'pc':64,'pc2':128,'lds':256}[k]-2*margin
print(k, n, d.get('seg_rows') or 0, 1 if (d.get('strip_out_cols') or full) != full else 0, tb)")
PIN="$KERN:$TB:$SEG:$ALIGN"
echo "pinned: --pin $PIN (kernel:steps per launch:seg rows:align)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $CFG --method $METHOD --steps $STEPS --warmup $WARM --no-cpu-baseline --no-check --pin $PIN > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
# the kernels' VGPR / LDS / scratch as dispatched (tools/kernel_resources.py: the trace's VGPR
# units corrected for gfx950)
python3 "$R/tools/kernel_resources.py" "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" > "$OUT/kernel_resources.txt"
head -3 "$OUT/kernel_resources.txt" | cut -c1-160
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc/p$i" -o run -- \
      python3 "$R/bench.py" --config $CFG --method $METHOD --steps 20 --warmup 2 --no-cpu-baseline --no-check --pin $PIN > "$OUT/pmc/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc/p$i.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$OUT/pmc" > "$OUT/pmc_summary.txt"
python3 "$R/tools/traffic.py" "$OUT/pmc" "$KNAME" "$OUT/traffic_${CFG}_${METHOD}.json"
# the profiled variant: bench.py uses these counters only for runs of the same kernel and steps per launch
python3 -c "
import json; p='$OUT/traffic_${CFG}_${METHOD}.json'; d=json.load(open(p))
d['variant'] = {'kernel': '$KERN', 'tb': $TB}; d['pin'] = '$PIN'
import sys; sys.path.insert(0, '$R/tools'); import glob, kernel_resources as kr
top = kr.summarize(glob.glob('$OUT/prof/**/*kernel_trace.csv', recursive=True)[0], '$KNAME')
d['resources'] = top[0] if top else None
json.dump(d, open(p, 'w'))"
