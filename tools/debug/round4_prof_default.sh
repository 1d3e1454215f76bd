#!/bin/bash
# round 4: rocprofv3 kernel stats of the default bench command itself (python bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out/prof_default
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_default" -o run --output-format csv -- \
    python3 "$R/bench.py" > "$R/gpurun_out/prof_default/bench.json" 2> "$R/gpurun_out/prof_default/bench.err"
echo "rocprof rc=$?"; cut -c1-200 "$R/gpurun_out/prof_default/bench.json"
