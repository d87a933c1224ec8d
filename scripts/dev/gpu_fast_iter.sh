#!/bin/bash
# fast-kernel iteration: parity tests, then bench timings under environment variants (args)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; tail -15 gpurun_out/parity.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_bench_variants.sh "$@"
