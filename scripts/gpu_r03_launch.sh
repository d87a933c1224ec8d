#!/bin/bash
# round 3: the new entry-point test, the default bench line and bench.py --gpus 2 through its own launcher
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_launch"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -x -v --timeout 300 --timeout-method thread > "$O/pytest_api.log" 2>&1 || { tail -40 "$O/pytest_api.log"; exit 1; }
tail -3 "$O/pytest_api.log"
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
tail -c 600 "$O/bench.json"; echo
timeout -k 10 300 python -u bench.py --gpus 2 --steps 200 --warmup 10 > "$O/bench_n2.json" 2> "$O/bench_n2.err" || { tail -20 "$O/bench_n2.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_n2.json').read().splitlines()[-1]); print({k: d.get(k) for k in ('value','n_gpus','rccl_nranks','rccl_error','rank_times_s','launcher','ms_per_step')})"
