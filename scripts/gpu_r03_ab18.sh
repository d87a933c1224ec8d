#!/bin/bash
# round 3: DQN act with 8 agent slots per workgroup (agw8, 1024 workgroups) vs 16 (agw16 = in-tree);
# DQN tests on both, then interleaved A/B
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab18"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
P2PMG_LIB="$R/build/ab/agw8.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest8.log" 2>&1 || { tail -40 "$O/pytest8.log"; exit 1; }
tail -1 "$O/pytest8.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/agw16.so build/ab/agw8.so
