#!/bin/bash
# config5 (DQN) bench + config3 (sq16) bench, rocprofv3 kernel stats and HBM PMC passes of both
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
timeout -k 10 300 python bench.py --workload config5 --steps 5 --warmup 1 --cpu-seconds 10 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { tail -30 "$O/bench_c5.err"; exit 1; }
cat "$O/bench_c5.json"
timeout -k 10 300 python bench.py --workload config3 --steps 10 --warmup 2 --cpu-seconds 10 > "$O/bench_c3.json" 2> "$O/bench_c3.err" || { tail -30 "$O/bench_c3.err"; exit 1; }
cat "$O/bench_c3.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o c5 --output-format csv -- python "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_c5.log" 2>&1 || { tail -20 "$O/prof_c5.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o c3 --output-format csv -- python "$R/bench.py" --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_c3.log" 2>&1 || { tail -20 "$O/prof_c3.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_c3_fetch" -o fetch --output-format csv -- python "$R/bench.py" --workload config3 --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_c3_fetch.log" 2>&1 || { tail -20 "$O/pmc_c3_fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_c3_write" -o write --output-format csv -- python "$R/bench.py" --workload config3 --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_c3_write.log" 2>&1 || { tail -20 "$O/pmc_c3_write.log"; exit 1; }
find "$O/prof_c5" "$O/prof_c3" -name "*kernel_stats.csv"
