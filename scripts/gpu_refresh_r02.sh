#!/bin/bash
# Round-2 profile refresh at HEAD: the bench line of every workload (with its CPU baseline), rocprofv3
# kernel stats, FETCH_SIZE / WRITE_SIZE in separate --pmc passes for the configs[1], [2], [3]
# episode kernels.  Stops at the first failure.  scripts/summarize_r02.py -> profiles/.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r02"; mkdir -p "$O"
run() {  # name timeout args...
  local n=$1 to=$2; shift 2
  timeout -k 10 "$to" python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
  tail -c 400 "$O/$n.json"; echo
}
run c2 300
run c3 400 --workload config3 --steps 10 --warmup 2
run c4 500 --workload config4 --steps 3 --warmup 1
run c5 400 --workload config5 --steps 10 --warmup 2
cd /tmp && export TMPDIR=/tmp
prof() {  # name timeout args...
  local n=$1 to=$2; shift 2
  timeout -k 10 "$to" rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o "$n" --output-format csv -- python3 "$R/bench.py" "$@" --no-cpu-baseline > "$O/prof_$n.log" 2>&1 || { tail -20 "$O/prof_$n.log"; exit 1; }
}
pmc() {  # name counter timeout args...
  local n=$1 c=$2 to=$3; shift 3
  timeout -s KILL "$to" rocprofv3 --pmc "$c" --kernel-trace -d "$O/pmc_${n}_$c" -o "$c" --output-format csv -- python3 "$R/bench.py" "$@" --no-cpu-baseline > "$O/pmc_${n}_$c.log" 2>&1 || { tail -20 "$O/pmc_${n}_$c.log"; exit 1; }
}
prof c2 300 --steps 30 --warmup 3
pmc c2 FETCH_SIZE 200 --steps 6 --warmup 1
pmc c2 WRITE_SIZE 200 --steps 6 --warmup 1
prof c3 300 --workload config3 --steps 4 --warmup 1
pmc c3 FETCH_SIZE 300 --workload config3 --steps 2 --warmup 1
pmc c3 WRITE_SIZE 300 --workload config3 --steps 2 --warmup 1
prof c4 500 --workload config4 --steps 2 --warmup 1
pmc c4 FETCH_SIZE 400 --workload config4 --steps 1 --warmup 1
pmc c4 WRITE_SIZE 400 --workload config4 --steps 1 --warmup 1
prof c5 300 --workload config5 --steps 3 --warmup 1
echo done
