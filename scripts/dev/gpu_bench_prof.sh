#!/bin/bash
# smoke + bench + rocprofv3 kernel trace + PMC passes (each step time-limited, stop at first failure)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { cat "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_bench" -o bench --output-format csv -- python "$R/bench.py" --steps 30 --warmup 3 --no-cpu-baseline > "$O/prof_bench.log" 2>&1 || { tail -20 "$O/prof_bench.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_fetch" -o fetch --output-format csv -- python "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1 || { tail -20 "$O/pmc_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_write" -o write --output-format csv -- python "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_write.log" 2>&1 || { tail -20 "$O/pmc_write.log"; exit 1; }
find "$O/prof_bench" "$O/pmc_fetch" "$O/pmc_write" -name "*.csv" | head -20
