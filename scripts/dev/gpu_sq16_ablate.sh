#!/bin/bash
# timing-only variants of episode_sq16_kernel (each build in its own process via P2PMG_LIB)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "" ${SQ_LIBS}; do
  echo "== ${lib:-main}"
  P2PMG_LIB=${lib:+$PWD/$lib} timeout -k 10 200 python -u scripts/probe_sq16.py 125000 "train inkernel,train prepass,greedy" || exit 1
done
