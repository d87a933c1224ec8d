#!/bin/bash
# The configs[2] episode kernel's SQ counter passes (two passes of <= 8 SQ counters, producer blocks
# off), then its standalone bench line.  -> gpurun_out/ROUND/sq/config3_{A,B}, ROUND/c3.json
# (scripts/summarize_sq.py gpurun_out/ROUND/sq profiles/ -> profiles/sq_config3.json)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
RND="${1:-r05}"
O="$R/gpurun_out/$RND"; mkdir -p "$O/sq"
PO="--secondary none --schedule-episodes 0"
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
PB="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VALU"
cd /tmp && export TMPDIR=/tmp
for P in A B; do
  C=$PA; [ $P = B ] && C=$PB
  P2PMG_NO_SPEC=1 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d "$O/sq/config3_$P" -o p --output-format csv -- python3 "$R/bench.py" --workload config3 --steps 2 --warmup 1 --no-cpu-baseline $PO > "$O/sq_config3_$P.log" 2>&1 || { tail -20 "$O/sq_config3_$P.log"; exit 1; }
done
cd "$R"
timeout -k 10 400 python -u bench.py --workload config3 --steps 10 --warmup 2 > "$O/c3.json" 2> "$O/c3.err" || { tail -20 "$O/c3.err"; exit 1; }
echo done
