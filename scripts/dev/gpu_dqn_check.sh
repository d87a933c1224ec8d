#!/bin/bash
# DQN change check: device tests, then configs[4] timing (apb probe + bench line) and kernel stats
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/dqn_tests.log" 2>&1
rc=$?; tail -4 "$O/dqn_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_dqn_apb.py ${APB:-8 16} > "$O/apb.log" 2>&1; rc=$?; cat "$O/apb.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_dqn" -o c5 --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_dqn.log" 2>&1 || { tail -20 "$O/prof_dqn.log"; exit 1; }
head -8 "$O/prof_dqn/c5_kernel_stats.csv" | cut -c1-150
