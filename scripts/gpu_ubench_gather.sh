#!/bin/bash
# dependent row-gather latency floor of the configs[1] / configs[3] geometry (scripts/ubench_gather.hip,
# built in-tree as build/dev/ubench_gather) -> gpurun_out/ubench_gather.jsonl
# args: tables pool rows_per_step steps agents_per_wave launches pair
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"; : > "$O/ubench_gather.jsonl"
B="$R/build/dev/ubench_gather"
for args in "8192 381 5 96 32 20 0" "8192 381 5 96 32 20 1" "8192 381 1 96 32 20 0" "8192 381 1 96 32 20 1" \
            "8192 381 5 96 16 20 0" "8192 381 5 96 16 20 1" "8192 160000 5 96 32 20 0" "1024 381 5 96 32 20 0" \
            "32768 381 5 96 64 20 0" "32768 381 1 96 64 20 0" "32768 381 1 96 32 20 1"; do
  timeout -k 10 120 "$B" $args >> "$O/ubench_gather.jsonl" || { echo "failed: $args"; exit 1; }
  tail -1 "$O/ubench_gather.jsonl" | cut -c 120-
done
