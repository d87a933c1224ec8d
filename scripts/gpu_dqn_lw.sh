#!/bin/bash
# DQN train kernel at 3 waves per SIMD (LW layout): the DQN GPU tests, then an interleaved A/B of
# configs[4] against the 2-wave build (build/ab/libp2pmg_occ2.so).  Stops at the first failure.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r04"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -k "dqn or DQN" \
  > "$O/lw_tests.txt" 2>&1 || { tail -40 "$O/lw_tests.txt"; exit 1; }
tail -3 "$O/lw_tests.txt"
bash scripts/gpu_ab.sh config5 2 p2pmicrogrid_amd/libp2pmg.so build/ab/libp2pmg_occ2.so
