#!/bin/bash
# DQN iteration: device tests for the DQN path (stop on crash)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dqn.py -q -x -rf > gpurun_out/dqn_tests.log 2>&1
rc=$?; tail -40 gpurun_out/dqn_tests.log; exit $rc
