#!/bin/bash
# round 3: DQN train backward with preloaded LDS operands: DQN tests on the in-tree library, A/B, trace
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab8"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/bwd.so || exit 1
bash scripts/gpu_dqn_trace.sh
