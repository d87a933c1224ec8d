#!/bin/bash
# sq16 + DQN change check: parity tests, configs[2] timing, DQN apb probe, configs[4] timing
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_config3.py tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/c3c5_tests.log" 2>&1
rc=$?; tail -4 "$O/c3c5_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload config3 --steps 5 --warmup 2 --no-cpu-baseline > "$O/c3.json" 2> "$O/c3.err" || { tail -20 "$O/c3.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/c3.json').read().splitlines()[-1]); print('c3', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'])"
timeout -k 10 300 python -u scripts/probe_dqn_apb.py 4 8 16 32 > "$O/apb.log" 2>&1; rc=$?; cat "$O/apb.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c5.json" 2> "$O/c5.err" || { tail -20 "$O/c5.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/c5.json').read().splitlines()[-1]); print('c5', d['value'], d['roofline']['frac'], d['ms_per_step'])"
