#!/bin/bash
# rocprofv3 kernel trace of a short config2 bench (timeline gaps between launches)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace" -o tr --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline "$@" > "$R/gpurun_out/trace.log" 2>&1 || { tail -20 "$R/gpurun_out/trace.log"; exit 1; }
find "$R/gpurun_out/trace" -name "*.csv"
