mkdir -p gpurun_out
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1; true)
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "long_horizon or kernel_adapter or (tiling and (-2 or -4)) or (full_size and chain)" > gpurun_out/t_chain.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/t_chain.log
timeout -k 10 300 python tools/pin_timing.py --config c2 --pins auto,dppy:2:56:0,dppy:2:-2:0,dppy:2:-3:0,dppy:2:-4:0,pc:2:48:0,pc:2:-2:0,pc:2:-3:0,pc2:2:88:0,pc2:2:-2:0,pc2:2:-3:0,x2y:2:-2:0 > gpurun_out/pins_c2.log 2>&1
echo "pins rc=$?"; cat gpurun_out/pins_c2.log
WS_HIP_LIB=$PWD/nvidia-jetson-workload_amd/lib/variants/libws_hip_stamps.so timeout -k 10 300 python tools/wave_timeline.py --pins dppy:2:48:0,dppy:2:56:0,dppy:2:184:0,dppy:2:-2:0,dppy:2:-3:0 --json gpurun_out/timeline_c2.json > gpurun_out/timeline_c2.log 2>&1
echo "timeline rc=$?"
timeout -k 10 200 python bench.py --config c1 --method rk4 --steps 1000 --warmup 50 > gpurun_out/c1.json 2> gpurun_out/c1.err
echo "c1 rc=$?"
