#!/bin/bash
# round 3: parity subset on the in-tree library, then A/B of config3 and config4
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab3"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_config3.py tests/test_gpu_config4.py tests/test_gpu_config4_full.py -m gpu -x -q --timeout 600 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
bash scripts/gpu_ab.sh config3 3 build/ab3/sq_a.so build/ab3/sq_e.so || exit 1
bash scripts/gpu_ab.sh config4 2 build/ab3/sq_e.so build/ab3/cur.so
