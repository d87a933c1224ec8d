#!/bin/bash
# configs[1] with chained launches: scenarios per wave (P2PMG_SPW; 0 = automatic, 16 here) swept,
# interleaved, on the default line without the secondary.  usage: gpu_spw_chain.sh REPS "spw ..."
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
REPS="$1"; SPWS="$2"
O="$R/gpurun_out/spw_chain"; mkdir -p "$O"
for i in $(seq 1 "$REPS"); do
  for W in $SPWS; do
    P2PMG_SPW=$W timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary none $EXTRA \
      > "$O/spw${W}_$i.json" 2> "$O/spw${W}_$i.err" || { tail -20 "$O/spw${W}_$i.err"; exit 1; }
    python -c "
import json; d=json.loads(open('$O/spw${W}_$i.json').read().splitlines()[-1])
ve=d['value_at_eps']; print('spw', $W, $i, round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), [round(w['kernel_ms']*1e3,2) for w in ve['windows']], round(ve['continuation']['value']/1e9,3))"
  done
done
