#!/bin/bash
# round 3: DQN act: every round's exploration code computed in the prologue; DQN tests (incl. full
# size) on the in-tree library, then interleaved A/B against the previous build
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab17"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/codes.so
