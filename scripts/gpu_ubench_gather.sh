#!/bin/bash
# dependent row-gather latency floor of the configs[1] / configs[3] geometry (scripts/ubench_gather.hip,
# built in-tree as build/dev/ubench_gather:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/dev/ubench_gather scripts/ubench_gather.hip)
# usage: gpu_ubench_gather.sh OUT.jsonl ['tables pool rows_per_step steps agents_per_wave launches pair stages' ...]
# (no argument sets: the round-2 configs[1] sweep)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
OUT="$O/${1:-ubench_gather.jsonl}"; shift; : > "$OUT"
B="$R/build/dev/ubench_gather"
SETS=("$@")
[ ${#SETS[@]} -eq 0 ] && SETS=("8192 381 5 96 32 20 0" "8192 381 5 96 32 20 1" "8192 381 1 96 32 20 0" "8192 381 1 96 32 20 1"
            "8192 381 5 96 16 20 0" "8192 381 5 96 16 20 1" "8192 160000 5 96 32 20 0" "1024 381 5 96 32 20 0"
            "32768 381 5 96 64 20 0" "32768 381 1 96 64 20 0" "32768 381 1 96 32 20 1")
for args in "${SETS[@]}"; do
  timeout -k 10 120 "$B" $args >> "$OUT" || { echo "failed: $args"; exit 1; }
  tail -1 "$OUT" | cut -c 120-
done
