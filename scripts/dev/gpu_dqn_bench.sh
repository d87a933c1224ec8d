#!/bin/bash
# DQN device tests + config5 bench + kernel stats
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -x -v --timeout 300 --timeout-method thread > "$O/dqn_tests.log" 2>&1
rc=$?; tail -15 "$O/dqn_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload config5 --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { tail -30 "$O/bench_c5.err"; exit 1; }
cat "$O/bench_c5.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o c5 --output-format csv -- python "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_c5.log" 2>&1 || { tail -20 "$O/prof_c5.log"; exit 1; }
cut -d, -f1-4 "$O/prof_c5/c5_kernel_stats.csv"
