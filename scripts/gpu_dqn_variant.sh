#!/bin/bash
# A DQN train-kernel variant library: the DQN GPU tests against it (P2PMG_LIB), then an interleaved
# configs[4] A/B against the main library.  usage: gpu_dqn_variant.sh build/ab/lib.so [REPS]
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r04"; mkdir -p "$O"
L="$1"; n=$(basename "$L" .so)
P2PMG_LIB="$R/$L" timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -k "dqn or DQN" \
  > "$O/${n}_dqn_tests.txt" 2>&1 || { tail -40 "$O/${n}_dqn_tests.txt"; exit 1; }
tail -2 "$O/${n}_dqn_tests.txt"
bash scripts/gpu_ab.sh config5 "${2:-2}" p2pmicrogrid_amd/libp2pmg.so "$L"
