#!/bin/bash
# Round 2: GPU tests, the default bench line, and SQ issue/wait counters (two passes of <= 8 SQ
# counters, separate runs) for the configs[1] fast kernel and the configs[2] sq16 kernel.
# P2PMG_NO_SPEC=1 drops the fast kernel's producer blocks so its counters are the episode's own.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/sq"; mkdir -p "$O"
WHAT="${1:-all}"
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
fi
timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
PB="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VALU"
export P2PMG_NO_SPEC=1
for W in config2 config3; do
  ST=8; [ $W = config3 ] && ST=2
  for P in A B; do
    C=$PA; [ $P = B ] && C=$PB
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d "$O/${W}_$P" -o p --output-format csv -- python3 "$R/bench.py" --workload $W --steps $ST --warmup 1 --no-cpu-baseline > "$O/${W}_$P.log" 2>&1 || { tail -20 "$O/${W}_$P.log"; exit 1; }
  done
done
mkdir -p "$O/sq" && python3 "$R/scripts/summarize_sq.py" "$O" "$O/sq" > "$O/sq_summary.json" && cat "$O/sq_summary.json"
