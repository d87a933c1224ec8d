#!/bin/bash
# sq16 change check: configs[2] device tests and timing
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_config3.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/c3_tests.log" 2>&1
rc=$?; tail -3 "$O/c3_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload config3 --steps 5 --warmup 2 --no-cpu-baseline > "$O/c3.json" 2> "$O/c3.err" || { tail -20 "$O/c3.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/c3.json').read().splitlines()[-1]); print('c3', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'])"
