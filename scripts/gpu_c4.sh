#!/bin/bash
# configs[3] (heterogeneous mixes, 1-year episodes): device tests, bench line, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_config4.py \
  > gpurun_out/c4_tests.log 2>&1 || { tail -30 gpurun_out/c4_tests.log; exit 1; }
tail -3 gpurun_out/c4_tests.log
timeout -k 10 400 python -u bench.py --workload config4 --steps 3 --warmup 1 \
  > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload config4 \
  --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.log 2>&1 || { tail -20 gpurun_out/prof_c4.log; exit 1; }
find gpurun_out/prof_c4 -name "*kernel_stats.csv" | head -3
