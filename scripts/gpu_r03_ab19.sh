#!/bin/bash
# round 3: DQN replay draws of step t + 1 in step t's reduce launch (smpn = in-tree): DQN + full-size
# tests, then interleaved A/B against the previous build, kernel stats
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03_ab19"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_dqn_api.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash scripts/gpu_ab.sh config5 2 build/ab/cur.so build/ab/smpn.so || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
find "$O/prof" -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
