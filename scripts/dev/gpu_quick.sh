#!/bin/bash
# quick device check: GPU tests (optional), the default bench line and the config3 bench line
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/quick"; mkdir -p "$O"
if [ "${1:-tests}" = tests ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('config2', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench3.json" 2> "$O/bench3.err" || { tail -20 "$O/bench3.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench3.json').read().splitlines()[-1]); print('config3', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'])"
