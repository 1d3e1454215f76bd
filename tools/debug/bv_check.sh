# barotropic physics model: GPU tests (both Poisson paths), then c3p bench with each path
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bv_tests.log 2>&1 || { tail -30 gpurun_out/bv_tests.log; exit 1; }
tail -2 gpurun_out/bv_tests.log
for fft in lds hipfft; do
  WS_BV_FFT=$fft timeout -k 10 120 python bench.py --config c3p --method rk4 --steps 200 --warmup 100 --no-cpu-baseline > gpurun_out/bv_$fft.json 2>/dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/bv_$fft.json')); r=d['roofline']
print('$fft', '%.2f Gcell/s %.4f ms/step frac %.3f' % (d['value']/1e9, d['ms_per_step'], r['frac']))"
done
