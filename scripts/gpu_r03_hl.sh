#!/bin/bash
# configs[1]: half-row loads (P2PMG_FAST_HL=1, default) vs two loads per row (=0): parity, then A/B
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/hl"; mkdir -p "$O"
P2PMG_FAST_HL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py > "$O/tests.txt" 2>&1 || { tail -40 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for rep in 1 2 3; do
  for H in 0 1; do
    P2PMG_FAST_HL=$H timeout -k 10 240 python -u bench.py --workload config2 --steps 50 --warmup 3 --no-cpu-baseline > "$O/hl${H}_$rep.json" 2> "$O/hl${H}_$rep.err" || { tail -20 "$O/hl${H}_$rep.err"; exit 1; }
    python -c "import json; d=json.loads(open('$O/hl${H}_$rep.json').read().splitlines()[-1]); print('hl', $H, $rep, round(d['roofline']['kernel_ms']*1e3, 2), 'us kernel', round(d['ms_per_step']*1e3, 2), 'us/step')"
  done
done
