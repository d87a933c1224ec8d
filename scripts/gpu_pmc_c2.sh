#!/bin/bash
# SQ instruction/cycle counters for the configs[1] fast episode kernel (one counter set per pass)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -d "$O/pmc_c2_$i" -o p --output-format csv -- python "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline > "$O/pmc_c2_$i.log" 2>&1 || { tail -20 "$O/pmc_c2_$i.log"; exit 1; }
done
find "$O" -path "*pmc_c2_*" -name "*counter_collection.csv"
