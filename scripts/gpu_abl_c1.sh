#!/bin/bash
# configs[1] fast-kernel timing ablation: main build vs fake Q rows (a1: every gather, a8: next-step rows)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
for L in p2pmicrogrid_amd/libp2pmg.so build/abl/libp2pmg_a1.so build/abl/libp2pmg_a8.so; do
  P2PMG_LIB="$R/$L" timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > "$O/abl_c1.json" 2> "$O/abl_c1.err" || { tail -20 "$O/abl_c1.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/abl_c1.json').read().splitlines()[-1]); print('$L', d['roofline']['kernel'], d['roofline']['kernel_ms'], d['ms_per_step'])"
done
