#!/bin/bash
# round 3: DQN train kernel wave priority variants (MFMA phases at prio 2 = in-tree; + layer 1; prio 3)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab13"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/prio.so build/ab/l1p.so build/ab/p3.so
