#!/bin/bash
# bench lines of configs[2], [3], [4] at HEAD (each step time-limited, stop at the first failure)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
for W in config3 config4 config5; do
  timeout -k 10 400 python -u bench.py --workload $W > "$O/bench_$W.json" 2> "$O/bench_$W.err" || { tail -20 "$O/bench_$W.err"; exit 1; }
  cat "$O/bench_$W.json"
done
