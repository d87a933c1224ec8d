#!/bin/bash
# fast-kernel change check: parity tests of the fast paths, then configs[1] and configs[3] timing
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/fast_tests.log" 2>&1
rc=$?; tail -4 "$O/fast_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$O/fc_c1.json" 2> "$O/fc_c1.err" || { tail -20 "$O/fc_c1.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/fc_c1.json').read().splitlines()[-1]); print('c1', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu-baseline > "$O/fc_c4.json" 2> "$O/fc_c4.err" || { tail -20 "$O/fc_c4.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/fc_c4.json').read().splitlines()[-1]); print('c4', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'])"
