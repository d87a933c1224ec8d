#!/bin/bash
# round 3: the GPU suite on the in-tree library, then interleaved A/B timing of build/ab3/*.so
# usage: gpu_r03_ab.sh [tests|notests] WORKLOAD REPS lib1.so lib2.so ...
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
if [ "$1" = tests ]; then
  bash scripts/gpu_r03_tests.sh || exit 1
fi
shift
bash scripts/gpu_ab.sh "$@"
