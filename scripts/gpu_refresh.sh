#!/bin/bash
# A round's profile refresh at HEAD: the bench line of every workload (with its CPU baseline), the
# launcher's --gpus 2 rehearsal, rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE in separate --pmc
# passes for the configs[1], [2], [3] episode kernels, SQ counter passes (configs[1], [2]) and the
# instruction-rate microbenchmark, and an MFMA-busy pass over configs[4].  Stops at the first failure.  scripts/summarize_refresh.py ROUND
# -> profiles/.
# usage: gpu_refresh.sh ROUND [A|B]  (e.g. r04 A: bench lines, microbenchmark, kernel stats;
#        B: PMC + SQ passes)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
RND="${1:-r05}"
PO="--secondary none --schedule-episodes 0"  # config2 passes that profile the primary episode kernel only
O="$R/gpurun_out/$RND"; mkdir -p "$O"
PART="${2:-A}"
run() {  # name timeout args...
  local n=$1 to=$2; shift 2
  timeout -k 10 "$to" python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
  tail -c 300 "$O/$n.json"; echo
}
if [ "$PART" = A ]; then
run c2 400 --gpus 1 --steps 20 --warmup 5          # the driver's default command (configs[1] + configs[2] secondary)
run c2long 300 --steps 200 --warmup 10 $PO
run c2n2 400 --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
run c3 400 --workload config3 --steps 10 --warmup 2
run c4 500 --workload config4 --steps 3 --warmup 1
run c5 400 --workload config5 --steps 10 --warmup 2
timeout -k 10 120 ./build/ubench_rate > "$O/ubench_rate.jsonl" 2>&1 || { tail -5 "$O/ubench_rate.jsonl"; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp
prof() {  # name timeout args...
  local n=$1 to=$2; shift 2
  timeout -k 10 "$to" rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o "$n" --output-format csv -- python3 "$R/bench.py" "$@" --no-cpu-baseline > "$O/prof_$n.log" 2>&1 || { tail -20 "$O/prof_$n.log"; exit 1; }
}
pmc() {  # name counters timeout args...
  local n=$1 c=$2 to=$3; shift 3
  timeout -s KILL "$to" rocprofv3 --pmc $c --kernel-trace -d "$O/pmc_${n}_${c%% *}" -o "${c%% *}" --output-format csv -- python3 "$R/bench.py" "$@" --no-cpu-baseline > "$O/pmc_${n}_${c%% *}.log" 2>&1 || { tail -20 "$O/pmc_${n}_${c%% *}.log"; exit 1; }
}
if [ "$PART" = A ]; then
prof c2 400 --gpus 1 --steps 20 --warmup 5
prof c3 300 --workload config3 --steps 4 --warmup 1
prof c4 500 --workload config4 --steps 2 --warmup 1
prof c5 300 --workload config5 --steps 3 --warmup 1
echo done A
exit 0
fi
pmc c2 FETCH_SIZE 200 --steps 6 --warmup 1 $PO
pmc c2 WRITE_SIZE 200 --steps 6 --warmup 1 $PO
pmc c3 FETCH_SIZE 300 --workload config3 --steps 2 --warmup 1
pmc c3 WRITE_SIZE 300 --workload config3 --steps 2 --warmup 1
pmc c4 FETCH_SIZE 400 --workload config4 --steps 1 --warmup 1
pmc c4 WRITE_SIZE 400 --workload config4 --steps 1 --warmup 1
# SQ issue counters (two passes of <= 8 SQ counters), producer blocks off (P2PMG_NO_SPEC=1)
export P2PMG_NO_SPEC=1
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
PB="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VALU"
for W in config2 config3; do
  ST=8; [ $W = config3 ] && ST=2
  for P in A B; do
    C=$PA; [ $P = B ] && C=$PB
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d "$O/sq/${W}_$P" -o p --output-format csv -- python3 "$R/bench.py" --workload $W --steps $ST --warmup 1 --no-cpu-baseline $PO > "$O/sq_${W}_$P.log" 2>&1 || { tail -20 "$O/sq_${W}_$P.log"; exit 1; }
  done
done
# configs[4]: the DQN kernels' MFMA busy cycles beside the clock (SQ_BUSY_CYCLES) and the VALU / LDS
# issue that shares the SIMDs with the MFMA stream
PC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
timeout -s KILL 240 rocprofv3 --pmc $PC --kernel-trace -d "$O/sq/config5_C" -o p --output-format csv -- python3 "$R/bench.py" --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > "$O/sq_config5_C.log" 2>&1 || { tail -20 "$O/sq_config5_C.log"; exit 1; }
echo done
