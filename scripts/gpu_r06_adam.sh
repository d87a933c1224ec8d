#!/bin/bash
# Round 6: the shared-DQN split path's forms -- the DQN parity tests ($3: a pytest -k selection), then
# scripts/gpu_dqn_split.sh ($2: the forms; bench lines + kernel stats of each).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}"; mkdir -p "$O"
K=(); [ -n "$3" ] && K=(-k "$3")
timeout -k 10 600 python -u -m pytest -x -v "${K[@]}" --timeout 240 --timeout-method thread -m gpu tests/test_gpu_dqn.py \
  tests/test_gpu_distributed.py "tests/test_gpu_fullsize.py::test_full_size_config5_shared_gradient_segments_against_oracle" \
  > "$O/dqn_adam_tests.txt" 2>&1 || { tail -30 "$O/dqn_adam_tests.txt"; exit 1; }
tail -3 "$O/dqn_adam_tests.txt"
bash scripts/gpu_dqn_split.sh "${1:-r06}" "$2"
