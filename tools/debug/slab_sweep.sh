# Per-rank share of C2 at 8 GPUs: every fused variant x segment length, pinned.
set -u
mkdir -p gpurun_out/sweep
for k in dpp dppy x2y lds; do
  for seg in 8 12 16 24 32 48 64; do
    WS_KERNEL=$k WS_SEG_ROWS=$seg timeout -k 10 60 python bench.py --config ${CFG:-c2_slab8} --method rk4 --steps 200 --warmup 200 --no-cpu-baseline > gpurun_out/sweep/${k}_$seg.json 2>/dev/null || { echo "$k $seg failed"; continue; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sweep/${k}_$seg.json')); r=d['roofline']
print('%-5s seg %3d  %6.2f Gcell/s  kernel %.4f ms' % ('$k', $seg, d['value']/1e9, r['mean_launch_ms']))"
  done
done
