#!/bin/bash
# Interleaved A/B of library builds on the default configs[1] line (chained launches, the epsilon
# schedule on, no secondary): value, ms per episode, kernel us per episode, the windows' kernel us,
# the continuation.  usage: gpu_ab_default.sh REPS lib1.so lib2.so ...
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
REPS="$1"; shift
O="$R/gpurun_out/ab_default"; mkdir -p "$O"
for i in $(seq 1 "$REPS"); do
  for L in "$@"; do
    n=$(basename "$L" .so)
    P2PMG_LIB="$R/$L" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary none \
      > "$O/${n}_$i.json" 2> "$O/${n}_$i.err" || { tail -20 "$O/${n}_$i.err"; exit 1; }
    python -c "
import json; d=json.loads(open('$O/${n}_$i.json').read().splitlines()[-1])
ve=d['value_at_eps']; print('$n', $i, round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), [round(w['kernel_ms']*1e3,2) for w in ve['windows']], round(ve['continuation']['value']/1e9,3))"
  done
done
