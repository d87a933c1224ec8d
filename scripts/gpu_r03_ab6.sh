#!/bin/bash
# round 3: configs[1] round-1 argmax precomputed per candidate row: parity on the in-tree library,
# then interleaved A/B against the previous build
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab6"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
bash scripts/gpu_ab.sh config2 3 build/ab/base.so build/ab/candact.so
