#!/bin/bash
# bench timings of the config2 workload under environment variants given as arguments
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 3 > gpurun_out/b.json 2> gpurun_out/b.err || { cat gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print(sys.argv[1], 'value %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'frac %.4f' % d['roofline']['frac'])" "$cfg"
done
