#!/bin/bash
# configs[4] bench line + rocprofv3 kernel stats (into gpurun_out/refresh like gpu_refresh_profiles.sh)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/refresh"; mkdir -p "$O"
timeout -k 10 400 python -u bench.py --workload config5 --steps 5 --warmup 1 > "$O/c5.json" 2> "$O/c5.err" || { tail -20 "$O/c5.err"; exit 1; }
cat "$O/c5.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o c5 --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_c5.log" 2>&1 || { tail -20 "$O/prof_c5.log"; exit 1; }
