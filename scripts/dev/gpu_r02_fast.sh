#!/bin/bash
# fast-kernel iteration: its parity tests, then the configs[1] bench line
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r02f"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('config2', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'])"
