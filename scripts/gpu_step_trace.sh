#!/bin/bash
# per-step s_memtime split of the fast kernel (P2PMG_TRACE build): wait for rows / chain to the
# next gathers / rest of the step, printed by three waves per launch
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/trace"; mkdir -p "$O"
L="${1:-build/dev/libp2pmg_trace.so}"; W="${2:-config2}"
P2PMG_LIB="$R/$L" timeout -k 10 240 python -u bench.py --workload "$W" --steps ${3:-3} --warmup 1 --no-cpu-baseline > "$O/${W}.out" 2> "$O/${W}.err" || { tail -20 "$O/${W}.err"; exit 1; }
grep TRACE "$O/${W}.out" | tail -9
tail -1 "$O/${W}.out" | cut -c1-300
