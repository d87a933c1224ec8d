#!/bin/bash
# round 3: the full GPU suite on the in-tree library, configs[1] A/B (scheduling fence) and
# configs[4] A/B (sample draws fused into the act launch)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
bash scripts/gpu_r03_tests.sh || exit 1
bash scripts/gpu_ab.sh config2 3 build/ab3/base.so build/ab3/sb.so || exit 1
bash scripts/gpu_ab.sh config5 2 build/ab3/base.so build/ab3/dqnf.so
