#!/bin/bash
# timing ablation of the episode kernel (main vs no-Q-gather vs compute-only builds)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/latency_ablation.py > gpurun_out/ablation.log 2>&1; rc=$?
cat gpurun_out/ablation.log; exit $rc
