#!/bin/bash
# The GPU test suite at HEAD (one process), output to gpurun_out/<round>/gpu_tests.txt.
# $2: extra pytest arguments (e.g. a -k selection)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}"; mkdir -p "$O"
timeout -k 10 1150 python -u -m pytest --maxfail=5 -v --durations=30 --timeout 300 --timeout-method thread -m gpu tests/ $2 > "$O/gpu_tests.txt" 2>&1
rc=$?
tail -5 "$O/gpu_tests.txt"
exit $rc
