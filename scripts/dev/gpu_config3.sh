#!/bin/bash
# GPU tests + both bench workloads + rocprofv3 kernel stats of the config3 bench (stop on crash)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 600 python bench.py --workload config3 --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { cat gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { tail -20 gpurun_out/prof_c3.log; exit 1; }
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -3
