#!/bin/bash
# round 3: quick parity subset on the in-tree library, then interleaved A/B timing
# usage: gpu_r03_ab2.sh "<pytest paths>" WORKLOAD REPS lib1.so lib2.so ...
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab2"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest $1 -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
shift
bash scripts/gpu_ab.sh "$@"
