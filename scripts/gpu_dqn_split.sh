#!/bin/bash
# configs[4] at one GPU: the fused world-1 path (train + reduce/Adam) against the multi-GPU code path
# (8 gradient segments -> segment fold -> RCCL all-gather on a one-rank communicator -> Adam), bench
# lines and rocprofv3 kernel stats of both.  Output under gpurun_out/<tag>/.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r05}/dqn_split"; mkdir -p "$O"
for V in fused split; do
  A=""; [ $V = split ] && A="--grad-segments 8 --rccl-world1"
  timeout -k 10 300 python -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline $A > "$O/bench_$V.json" 2> "$O/bench_$V.err" || { tail -20 "$O/bench_$V.err"; exit 1; }
  tail -c 300 "$O/bench_$V.json"; echo
done
cd /tmp && export TMPDIR=/tmp
for V in fused split; do
  A=""; [ $V = split ] && A="--grad-segments 8 --rccl-world1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$V" -o "$V" --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline $A > "$O/prof_$V.log" 2>&1 || { tail -20 "$O/prof_$V.log"; exit 1; }
done
echo done
