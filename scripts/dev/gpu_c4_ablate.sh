#!/bin/bash
# configs[3] fast-kernel timing ablation: main build vs the round-R gather replaced (P2PMG_ABLATE=7)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
for L in p2pmicrogrid_amd/libp2pmg.so build/abl/libp2pmg_c4a7.so; do
  P2PMG_LIB="$R/$L" timeout -k 10 300 python -u bench.py --workload config4 --scenarios 4096 --steps 2 --warmup 1 \
    --no-cpu-baseline > "$O/abl_c4.json" 2> "$O/abl_c4.err" || { tail -20 "$O/abl_c4.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/abl_c4.json').read().splitlines()[-1]); print('$L', d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
