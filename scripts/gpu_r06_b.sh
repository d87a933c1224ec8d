#!/bin/bash
# configs[3]'s full-year oracle test, then the rocprofv3 kernel statistics of the default bench command
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}"; mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 1050 --timeout-method thread -m gpu tests/test_gpu_config4_full.py \
  > "$O/config4_full.txt" 2>&1 || { tail -30 "$O/config4_full.txt"; exit 1; }
tail -3 "$O/config4_full.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o p --output-format csv -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_default.json" 2> "$O/prof_default.err" || { tail -20 "$O/prof_default.err"; exit 1; }
find "$O/prof_default" -name "*kernel_stats.csv"
