set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cw
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cw/bvort_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cw/bvort_tests.log; [ $rc -eq 0 ] || exit $rc
for cw in 1 2 4 8; do
  WS_BV_CW=$cw timeout -k 10 200 python bench.py --config c3p --steps 100 --warmup 50 --no-cpu-baseline > gpurun_out/cw/c3p_$cw.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/cw/c3p_$cw.json')); print('cw $cw', d['value']/1e9, d['ms_per_step'])"
done
CFG=c3p bash tools/profile_physics.sh
