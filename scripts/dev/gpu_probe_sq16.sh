#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/probe_sq16.py ${1:-125000} > gpurun_out/probe_sq16.log 2>&1; rc=$?; cat gpurun_out/probe_sq16.log; exit $rc
