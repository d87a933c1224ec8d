#!/bin/bash
# sq16 (configs[2]) iteration: shared-table parity tests, then a short config3 bench + kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_config3.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c3_tests.log 2>&1
rc=$?; tail -15 gpurun_out/c3_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { cat gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
