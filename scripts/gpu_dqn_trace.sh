#!/bin/bash
# per-phase s_memtime split of dqn_train_kernel (P2PMG_TRACE build of the library, env step 50)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/trace"; mkdir -p "$O"
L="${1:-build/dev/libp2pmg_trace.so}"
P2PMG_LIB="$R/$L" timeout -k 10 300 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > "$O/dqn.out" 2> "$O/dqn.err" || { tail -20 "$O/dqn.err"; exit 1; }
grep "DQNTRACE\|ACTTRACE" "$O/dqn.out" | head -24
