#!/bin/bash
# round 3: DQN variants: 3 barriers per agent (double-buffered online H1), reduce with 32 loads in
# flight, act MFMA at raised priority; DQN tests on the combined build, then interleaved A/B
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab14"; mkdir -p "$O"
P2PMG_LIB="$R/build/ab/all3.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/bar3.so build/ab/red32.so build/ab/actp.so build/ab/all3.so
