#!/bin/bash
# (1) FETCH_SIZE / WRITE_SIZE calibration on known byte counts (scripts/pmc_calib.hip, one rocprofv3
#     pass per counter); (2) the corrected prefetch probe (scripts/ubench_gather.hip stages=3, the
#     round-4 geometry: 8192 tables, pools of 512 rows, 5 rows per step, 96 steps, 32 agents per wave).
# Binaries built in-tree beforehand:
#   hipcc --offload-arch=gfx950 -O3 -o build/pmc_calib scripts/pmc_calib.hip
#   hipcc --offload-arch=gfx950 -O3 -o build/ubench_gather scripts/ubench_gather.hip
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}/calib"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$R/build/pmc_calib" > "$O/bytes.json" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d "$O/pmc_$c" -o p --output-format csv -- "$R/build/pmc_calib" \
    > "$O/pmc_$c.log" 2>&1 || { tail -20 "$O/pmc_$c.log"; exit 1; }
done
: > "$O/pf.jsonl"
for pool in 512 381; do
  timeout -k 10 120 "$R/build/ubench_gather" 8192 $pool 5 96 32 20 0 3 >> "$O/pf.jsonl" || exit 1
done
timeout -k 10 120 "$R/build/ubench_gather" 8192 512 5 96 32 20 0 1 >> "$O/pf.jsonl" || exit 1
cat "$O/pf.jsonl"
find "$O" -name "*counter_collection.csv"
