#!/bin/bash
# Round 5, chained launches: the driver's default command (line + rocprofv3 kernel stats / trace of
# the same command), a 200-episode configs[1] run, the one-launch-per-episode line beside it, and the
# launcher's --gpus 2 rehearsal.  -> gpurun_out/ROUND/ (scripts/summarize_trace.py splits the trace).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
RND="${1:-r05c}"
O="$R/gpurun_out/$RND"; mkdir -p "$O"
PO="--secondary none --schedule-episodes 0"
run() {  # name timeout args...
  local n=$1 to=$2; shift 2
  timeout -k 10 "$to" python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
  tail -c 300 "$O/$n.json"; echo
}
run c2 400 --gpus 1 --steps 20 --warmup 5
run c2off 300 --steps 20 --warmup 5 --no-cpu-baseline $PO --chain off
run c2long 300 --steps 200 --warmup 10 --no-cpu-baseline $PO
run c2n2 400 --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_c2" -o c2 --output-format csv -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_c2.json" 2> "$O/prof_c2.log" || { tail -20 "$O/prof_c2.log"; exit 1; }
echo done
