#!/bin/bash
# battery paths: config3/config4 device tests, then configs[2] (sq16) and configs[3] (fast, battery) timings
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_config4.py \
  tests/test_gpu_config3.py > "$O/bat_tests.log" 2>&1 || { tail -30 "$O/bat_tests.log"; exit 1; }
tail -2 "$O/bat_tests.log"
timeout -k 10 300 python -u bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > "$O/bat_c3.json" 2> "$O/bat_c3.err" || { tail -20 "$O/bat_c3.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bat_c3.json').read().splitlines()[-1]); print('c3', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python -u bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bat_c4.json" 2> "$O/bat_c4.err" || { tail -20 "$O/bat_c4.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bat_c4.json').read().splitlines()[-1]); print('c4', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
