#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -40 gpurun_out/gpu_tests.log; exit $rc
