#!/bin/bash
# configs[1]: scenarios per wave (P2PMG_SPW) sweep, interleaved, bench kernel time
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/spw"; mkdir -p "$O"
for rep in 1 2; do
  for S in ${SPWS:-0 8 4 2}; do
    P2PMG_SPW=$S timeout -k 10 240 python -u bench.py --workload ${W:-config2} --steps ${ST:-50} --warmup 3 --no-cpu-baseline > "$O/spw${S}_$rep.json" 2> "$O/spw${S}_$rep.err" || { tail -20 "$O/spw${S}_$rep.err"; exit 1; }
    python -c "import json; d=json.loads(open('$O/spw${S}_$rep.json').read().splitlines()[-1]); print('spw', $S, $rep, round(d['roofline']['kernel_ms']*1e3, 2), 'us kernel', round(d['ms_per_step']*1e3, 2), 'us/step')"
  done
done
