#!/bin/bash
# round 3: DQN train kernel: target layer-1 action term as a per-column fmaf (l1a), dW1 on VALU
# (dw1v), both; DQN tests on the combined build, then interleaved A/B
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab15"; mkdir -p "$O"
P2PMG_LIB="$R/build/ab/both.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/l1a.so build/ab/dw1v.so build/ab/both.so
