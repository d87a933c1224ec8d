#!/bin/bash
# Round 6 closing run: the whole GPU suite (one process), then the driver's default bench command.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}"; mkdir -p "$O"
bash scripts/gpu_tests.sh "${1:-r06}" || exit 1
S=$(date +%s.%N)
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_final.json" 2> "$O/bench_final.err" || { tail -20 "$O/bench_final.err"; exit 1; }
E=$(date +%s.%N)
awk -v s="$S" -v e="$E" "BEGIN{print \"wall_s\", e - s}" > "$O/bench_final.wall"
tail -c 400 "$O/bench_final.json"
