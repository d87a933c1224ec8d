#!/bin/bash
# full -m gpu suite (optionally a subset: $1 = pytest path/-k args)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_tests"; mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest ${1:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|SKIPPED" "$O/pytest.log" | tail -15; tail -3 "$O/pytest.log"; exit $rc
