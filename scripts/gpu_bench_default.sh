#!/bin/bash
# The driver's default bench command at N=1, then the launcher's --gpus 2 rehearsal (two ranks on the
# one GPU, host exchange), each under its own time limit; lines under gpurun_out/<round>/.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r05}"; mkdir -p "$O"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -20 "$O/bench_default.err"; exit 1; }
tail -c 400 "$O/bench_default.json"; echo
timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_n2.json" 2> "$O/bench_n2.err" || { tail -20 "$O/bench_n2.err"; exit 1; }
tail -c 400 "$O/bench_n2.json"; echo
