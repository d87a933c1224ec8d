#!/bin/bash
# A/B timing of library builds on one box: bench.py with P2PMG_LIB = each .so in turn, interleaved
# (REPS rounds), kernel ms and ms per step per run.  usage: gpu_ab.sh WORKLOAD REPS lib1.so lib2.so ...
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
W="$1"; REPS="$2"; shift 2
O="$R/gpurun_out/ab"; mkdir -p "$O"
ST=50; [ "$W" = config3 ] && ST=8
for rep in $(seq 1 "$REPS"); do
  for L in "$@"; do
    n=$(basename "$L" .so)
    P2PMG_LIB="$R/$L" timeout -k 10 240 python -u bench.py --workload "$W" --steps $ST --warmup 3 --no-cpu-baseline --secondary none --schedule-episodes 0 > "$O/${W}_${n}_$rep.json" 2> "$O/${W}_${n}_$rep.err" || { tail -20 "$O/${W}_${n}_$rep.err"; exit 1; }
    python -c "import json; d=json.loads(open('$O/${W}_${n}_$rep.json').read().splitlines()[-1]); print('$W', '$n', $rep, round(d['roofline']['kernel_ms']*1e3, 2), 'us kernel', round(d['ms_per_step']*1e3, 2), 'us/step')"
  done
done
