#!/bin/bash
# Round 6 A/B: configs[1] with the candidate-row gathers masked by the partner's round-0 code
# (HEAD) against the previous build (build/libp2pmg_base.so via P2PMG_LIB), interleaved, after
# the fast-kernel parity tests.  Output under gpurun_out/<tag>/cand/.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${1:-r06}/cand"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_chain.py > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for i in 1 2 3; do
  for V in base head; do
    if [ $V = base ]; then export P2PMG_LIB="$R/build/libp2pmg_base.so"; else unset P2PMG_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --secondary none --extra "" --no-cpu-baseline \
      --schedule-episodes 0 > "$O/bench_${V}_$i.json" 2> "$O/bench_${V}_$i.err" || { tail -20 "$O/bench_${V}_$i.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_per_launch'])" "$O/bench_${V}_$i.json" "$V $i"
  done
done
