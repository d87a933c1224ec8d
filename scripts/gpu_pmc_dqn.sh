#!/bin/bash
# DQN train-kernel stall breakdown: one SQ counter pass (8 SQ counters) over a short configs[4] run
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d "$O/pmc_dqn" -o sq --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_dqn.log" 2>&1 || { tail -20 "$O/pmc_dqn.log"; exit 1; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob('/root/repo/gpurun_out/pmc_dqn/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
