#!/bin/bash
# configs[4] at one GPU: the fused world-1 path (train + reduce/Adam) against the multi-GPU code path
# (8 gradient segments -> segment fold -> RCCL all-gather on a one-rank communicator -> Adam), bench
# lines and rocprofv3 kernel stats of each form:
#   split        the default split path (fold with 4 runs per thread, standalone Adam launch)
#   splitfold1   the fold on the reduce kernel's 1024-thread form (P2PMG_FOLD_SPT=1, rounds 4-5)
#   splitfoldK   the fold with K = 2, 8 or 16 runs per thread (P2PMG_FOLD_SPT=K)
#   splitact     the Adam step inside the next env step's act launch (P2PMG_DQN_ADAM=act)
#   splitadamK   the standalone Adam launch with K = 64 or 128 threads per workgroup (P2PMG_ADAM_TPB=K)
#   fusednopx    the fused path with the replay draws in each act launch (P2PMG_DQN_SAMPLE_PREPASS=0)
# Output under gpurun_out/<tag>/dqn_split/.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}/dqn_split"; mkdir -p "$O"
FORMS="${2:-fused split splitfold1 splitfold16 splitact}"
setform() {
  unset P2PMG_DQN_ADAM P2PMG_FOLD_SPT P2PMG_ADAM_TPB P2PMG_DQN_SAMPLE_PREPASS
  A="--grad-segments 8 --rccl-world1"
  case $1 in
    fused) A="" ;;
    fusednopx) A=""; export P2PMG_DQN_SAMPLE_PREPASS=0 ;;
    splitfold1) export P2PMG_FOLD_SPT=1 ;;
    splitfold*) export P2PMG_FOLD_SPT=${1#splitfold} ;;
    splitact) export P2PMG_DQN_ADAM=act ;;
    splitadam*) export P2PMG_ADAM_TPB=${1#splitadam} ;;
  esac
}
for V in $FORMS; do
  setform $V
  timeout -k 10 300 python -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline $A > "$O/bench_$V.json" 2> "$O/bench_$V.err" || { tail -20 "$O/bench_$V.err"; exit 1; }
  tail -c 300 "$O/bench_$V.json"; echo
done
cd /tmp && export TMPDIR=/tmp
for V in $FORMS; do
  setform $V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$V" -o "$V" --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline $A > "$O/prof_$V.log" 2>&1 || { tail -20 "$O/prof_$V.log"; exit 1; }
done
echo done
