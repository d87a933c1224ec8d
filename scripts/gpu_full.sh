#!/bin/bash
# Full GPU pass: every -m gpu test, smoke(), both bench workloads, rocprofv3 kernel stats of each.
# Each GPU step has its own time limit; the script stops at the first failing step.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 "$O/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { cat "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 600 python -u bench.py --workload config3 --steps 10 --warmup 2 --cpu-seconds 10 > "$O/bench_c3.json" 2> "$O/bench_c3.err" || { cat "$O/bench_c3.err"; exit 1; }
cat "$O/bench_c3.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_bench" -o bench --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 3 --no-cpu-baseline > "$O/prof_bench.log" 2>&1 || { tail -20 "$O/prof_bench.log"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o c3 --output-format csv -- python3 "$R/bench.py" --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_c3.log" 2>&1 || { tail -20 "$O/prof_c3.log"; exit 1; }
find "$O/prof_bench" "$O/prof_c3" -name "*kernel_stats.csv"
