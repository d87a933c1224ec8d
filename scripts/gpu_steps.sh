#!/bin/bash
# GPU side: run named steps in order, each under its own time limit, logging to gpurun_out/<dir>/.
# A step that fails normally (a test failure, rc 1/2) does not stop the list; a time limit, abort,
# segfault or kill (124/134/137/139 or > 128) ends the call there.
# usage: gpu_steps.sh DIR 'name|seconds|command' ...
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
D="$R/gpurun_out/$1"; shift; mkdir -p "$D"
worst=0
for step in "$@"; do
  name="${step%%|*}"; rest="${step#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name ($to s): $cmd"
  # heartbeat: a long, quiet step (a CPU-side oracle check) still shows progress every 60 s
  ( while sleep 60; do echo "$(date +%T) $name running" >> "$D/heartbeat.txt"; done ) &
  hb=$!
  timeout -k 10 "$to" bash -c "$cmd" > "$D/$name.out" 2> "$D/$name.err"
  rc=$?
  kill "$hb" 2>/dev/null; wait "$hb" 2>/dev/null
  echo "== $name rc=$rc"; tail -3 "$D/$name.out"
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "fatal rc $rc at $name: stopping"; exit $rc; fi
  [ $rc -ne 0 ] && worst=$rc
done
exit $worst
