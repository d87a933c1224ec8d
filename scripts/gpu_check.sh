#!/bin/bash
# Iteration check at the working tree: selected GPU test files (one pytest process), then bench lines
# of the named workloads, each step under its own time limit; output under gpurun_out/<tag>/.
# usage: gpu_check.sh TAG "tests/a.py tests/b.py" "config3 config2 ..."
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/$1"; mkdir -p "$O"
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $2 > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
  tail -3 "$O/tests.txt"
fi
for W in $3; do
  ST=50; [ "$W" = config3 ] && ST=10; [ "$W" = config4 ] && ST=2; [ "$W" = config5 ] && ST=5
  timeout -k 10 400 python -u bench.py --workload "$W" --steps $ST --warmup 2 --no-cpu-baseline --secondary none --schedule-episodes 0 > "$O/bench_$W.json" 2> "$O/bench_$W.err" || { tail -20 "$O/bench_$W.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline'].get('kernel'))" "$O/bench_$W.json" "$W"
done
