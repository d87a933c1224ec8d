#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/latency_probe.py > gpurun_out/latency_probe.log 2>&1
rc=$?; cat gpurun_out/latency_probe.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_quick" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/quick_timing.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_quick.log" 2>&1
rc=$?; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/prof_quick.log"; find "$GRAFT_REPO_ROOT/gpurun_out/prof_quick" -name "*stats*" | head; exit $rc
