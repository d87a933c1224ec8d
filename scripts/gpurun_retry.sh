#!/bin/bash
# Host side: run one gpurun call, re-submitting only while the pod answers "no GPU slot free"
# (exit 3: nothing ran, nothing charged).  usage: gpurun_retry.sh LOG TIMEOUT 'command'
LOG="$1"; TO="$2"; CMD="$3"
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
