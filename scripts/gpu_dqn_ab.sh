#!/bin/bash
# configs[4] train-kernel study: interleaved A/B of library builds (scripts/gpu_ab.sh), per-kernel
# rocprofv3 stats of each, and the per-phase s_memtime traces of the given trace builds.
# usage: gpu_dqn_ab.sh "lib1.so lib2.so ..." ["trace1.so trace2.so ..."]
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/dqn_ab"; mkdir -p "$O"
bash scripts/gpu_ab.sh config5 1 $1 || exit 1
cd /tmp && export TMPDIR=/tmp
for L in $1; do
  n=$(basename "$L" .so)
  P2PMG_LIB="$R/$L" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o "$n" --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_$n.log" 2>&1 || { tail -20 "$O/prof_$n.log"; exit 1; }
  f=$(find "$O/prof_$n" -name "*kernel_stats.csv" | head -1)
  echo "== $n"; cut -d, -f1-4 "$f" | head -5
done
cd "$R"
for T in $2; do
  n=$(basename "$T" .so)
  bash scripts/gpu_dqn_trace.sh "$T" > "$O/trace_$n.txt" || exit 1
  echo "== $n"; head -8 "$O/trace_$n.txt"
done
