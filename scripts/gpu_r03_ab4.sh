#!/bin/bash
# round 3: the full GPU suite on the in-tree library, then A/B of configs[1] (fast kernel) variants
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
bash scripts/gpu_r03_tests.sh || exit 1
bash scripts/gpu_ab.sh config2 3 "$@"
