#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/latency_probe.py > gpurun_out/latency_probe.log 2>&1
rc2=$?; cat gpurun_out/latency_probe.log; exit $rc2
