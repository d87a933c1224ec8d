#!/bin/bash
# iteration loop: GPU tests, ablation probe, bench (each time-limited; stop on crash)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/latency_ablation.py > gpurun_out/ablation.log 2>&1 || { tail gpurun_out/ablation.log; exit 1; }
cat gpurun_out/ablation.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
