#!/bin/bash
# Round-end check at HEAD on one box: the GPU suite in one process, smoke(), then the chained-launch
# profile refresh (scripts/gpu_chain_refresh.sh).  usage: gpu_final.sh ROUND
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
RND="${1:-r05}"
O="$R/gpurun_out/$RND"; mkdir -p "$O"
bash scripts/gpu_tests.sh "$RND" || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -20 "$O/smoke.txt"; exit 1; }
tail -2 "$O/smoke.txt"
bash scripts/gpu_chain_refresh.sh "${RND}_refresh"
