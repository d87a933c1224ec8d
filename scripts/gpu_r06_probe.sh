#!/bin/bash
# Round 6 measurements in one call: PMC calibration + prefetch probe (gpu_calib.sh), the select
# probe, the f32-mode test with its printed error bounds, and the driver's default bench command
# (configs[1] + the configs[2], [4] and [3] records) with its wall time.  $2 = nocalib: skip the first part.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}"; mkdir -p "$O"
[ "$2" = "nocalib" ] || bash scripts/gpu_calib.sh "${1:-r06}" || exit 1
timeout -k 10 60 "$R/build/ubench_select" > "$O/select.jsonl" || exit 1
cat "$O/select.jsonl"
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_f32_mode.py \
  > "$O/f32_mode.txt" 2>&1 || { tail -30 "$O/f32_mode.txt"; exit 1; }
grep "max relative" "$O/f32_mode.txt"
t0=$(date +%s.%N)
timeout -k 10 560 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -30 "$O/bench_default.err"; exit 1; }
t1=$(date +%s.%N)
echo "bench wall_s $(python -c "print($t1 - $t0)")" | tee "$O/bench_default.wall"
python - "$O/bench_default.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("configs[1]", d["value"], d["roofline"]["frac"])
for k in ("secondary", "secondary_dqn", "secondary_year"):
    s = d.get(k, {})
    print(k, s.get("value"), s.get("ms_per_step"), (s.get("roofline") or {}).get("frac"), s.get("setup_s"), s.get("error"))
PY
