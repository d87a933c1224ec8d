#!/bin/bash
# round 3: DQN phase traces + rocprof kernel stats at HEAD
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_tr"; mkdir -p "$O"
bash scripts/gpu_dqn_trace.sh || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
find "$O/prof" -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
