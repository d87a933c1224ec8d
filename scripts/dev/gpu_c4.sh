#!/bin/bash
# configs[3] (heterogeneous mixes, 1-year episodes): device tests, bench lines, rocprofv3 kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_config4.py \
  tests/test_gpu_config3.py > "$O/c4_tests.log" 2>&1 || { tail -30 "$O/c4_tests.log"; exit 1; }
tail -3 "$O/c4_tests.log"
for S in ${C4_SCEN:-4096}; do
timeout -k 10 400 python -u bench.py --workload config4 --scenarios $S --steps 3 --warmup 1 \
  > "$O/bench_c4_$S.json" 2> "$O/bench_c4_$S.err" || { tail -20 "$O/bench_c4_$S.err"; exit 1; }
cat "$O/bench_c4_$S.json"
done
if [ -n "$C4_PROF" ]; then
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_c4" -o c4 --output-format csv -- python3 "$R/bench.py" \
  --workload config4 --steps 2 --warmup 1 --no-cpu-baseline > "$O/prof_c4.log" 2>&1 || { tail -20 "$O/prof_c4.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_c4_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" \
  --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_c4_fetch.log" 2>&1 || { tail -20 "$O/pmc_c4_fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_c4_write" -o write --output-format csv -- python3 "$R/bench.py" \
  --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_c4_write.log" 2>&1 || { tail -20 "$O/pmc_c4_write.log"; exit 1; }
find "$O/prof_c4" -name "*kernel_stats.csv"
fi
