set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s8
timeout -k 10 200 python bench.py --config c2_slab8 --steps 200 --warmup 300 --no-cpu-baseline > gpurun_out/s8/bench.json 2> gpurun_out/s8/bench.err || exit $?
cat gpurun_out/s8/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s8/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c2_slab8 --steps 200 --warmup 300 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/s8/prof.json 2>&1 || exit $?
cat $GRAFT_REPO_ROOT/gpurun_out/s8/prof/run_kernel_stats.csv
