#!/bin/bash
# round 3: DQN train kernel start skew of the grid's second half (timing experiment)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/skew1.so build/ab/skew2.so build/ab/skew4.so build/ab/prio.so
