# layered PE (c4p): GPU tests on the default build, then the bench per variant library
set -e
timeout -k 10 200 python -u -m pytest tests/test_gpu_layered_pe.py -q --timeout 120 --timeout-method thread > gpurun_out/lpe_tests.log 2>&1 || { tail -30 gpurun_out/lpe_tests.log; exit 1; }
tail -1 gpurun_out/lpe_tests.log
for v in ${VARIANTS:-default lpe64x8}; do
  lib=nvidia-jetson-workload_amd/lib/libws_hip.so
  [ $v = default ] || lib=nvidia-jetson-workload_amd/lib/variants/libws_hip_$v.so
  WS_HIP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c4p --method rk4 --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/lpe_$v.json 2>/dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/lpe_$v.json')); r=d['roofline']
print('%-9s %.2f Gcell/s %.4f ms/step frac %.3f' % ('$v', d['value']/1e9, d['ms_per_step'], r['frac']))"
done
