#!/bin/bash
# Round-1 profile refresh: bench lines + rocprofv3 kernel stats for configs[1], [3], [4]; FETCH/WRITE
# PMC passes (separate runs) for the configs[1] and configs[3] fast kernels.  Stops at the first failure.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/refresh"; mkdir -p "$O"
timeout -k 10 300 python -u bench.py > "$O/c1.json" 2> "$O/c1.err" || { tail -20 "$O/c1.err"; exit 1; }
cat "$O/c1.json"
timeout -k 10 400 python -u bench.py --workload config4 --steps 3 --warmup 1 > "$O/c4.json" 2> "$O/c4.err" || { tail -20 "$O/c4.err"; exit 1; }
cat "$O/c4.json"
timeout -k 10 400 python -u bench.py --workload config5 --steps 5 --warmup 1 > "$O/c5.json" 2> "$O/c5.err" || { tail -20 "$O/c5.err"; exit 1; }
cat "$O/c5.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c1" -o c1 --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 3 --no-cpu-baseline > "$O/prof_c1.log" 2>&1 || { tail -20 "$O/prof_c1.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_c1_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_c1_fetch.log" 2>&1 || { tail -20 "$O/pmc_c1_fetch.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_c1_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_c1_write.log" 2>&1 || { tail -20 "$O/pmc_c1_write.log"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_c4" -o c4 --output-format csv -- python3 "$R/bench.py" --workload config4 --steps 2 --warmup 1 --no-cpu-baseline > "$O/prof_c4.log" 2>&1 || { tail -20 "$O/prof_c4.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_c4_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_c4_fetch.log" 2>&1 || { tail -20 "$O/pmc_c4_fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_c4_write" -o write --output-format csv -- python3 "$R/bench.py" --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_c4_write.log" 2>&1 || { tail -20 "$O/pmc_c4_write.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o c5 --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_c5.log" 2>&1 || { tail -20 "$O/prof_c5.log"; exit 1; }
find "$O" -name "*.csv" | head -40
