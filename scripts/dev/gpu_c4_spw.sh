#!/bin/bash
# configs[3]: scenarios per wave (P2PMG_SPW) sweep of the fast battery kernel
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
for W in 0 8 4; do
  P2PMG_SPW=$W timeout -k 10 300 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$O/spw_c4.json" 2> "$O/spw_c4.err" || { tail -20 "$O/spw_c4.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/spw_c4.json').read().splitlines()[-1]); print('spw $W', d['value'], d['roofline']['kernel_ms'])"
done
