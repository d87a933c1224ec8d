#!/bin/bash
# round 3: DQN train kernel: in-tree (target action fmaf + dW1 on VALU) and the online action term
# as fmaf too (l1o); DQN tests on both, then interleaved A/B against the previous build
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab16"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
P2PMG_LIB="$R/build/ab/l1o.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_l1o.log" 2>&1 || { tail -40 "$O/pytest_l1o.log"; exit 1; }
tail -1 "$O/pytest_l1o.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/cur2.so build/ab/l1o.so build/ab/redp.so
