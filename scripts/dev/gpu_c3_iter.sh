#!/bin/bash
# config3 iteration: shared-table parity tests, then the config3 timing probe
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_config3.py tests/test_gpu_distributed.py -q -x -rf > gpurun_out/c3_tests.log 2>&1
rc=$?; tail -5 gpurun_out/c3_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 800 python scripts/probe_c3.py 125000 > gpurun_out/probe_c3.log 2>&1; rc=$?; cat gpurun_out/probe_c3.log; exit $rc
