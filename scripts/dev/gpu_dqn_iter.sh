#!/bin/bash
# DQN iteration: its device tests, then the configs[4] bench line (+ a rocprofv3 kernel-stats pass)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/dqn"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py tests/test_gpu_config4.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench5.json" 2> "$O/bench5.err" || { tail -20 "$O/bench5.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench5.json').read().splitlines()[-1]); print('config5', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof5" -o p --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof5.log" 2>&1 || { tail -20 "$O/prof5.log"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("/root/repo/gpurun_out/dqn/prof5/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
