#!/bin/bash
# distributed pieces on one GPU: the gloo/RCCL tests, and the bench N>1 path rehearsed with two
# ranks on the one device (P2PMG_BENCH_DEVICE=0; RCCL then runs two ranks on one GPU)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r02d"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -v --timeout 500 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -8 "$O/pytest.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > "$O/b1.json" 2> "$O/b1.err" || { tail -20 "$O/b1.err"; exit 1; }
tail -c 600 "$O/b1.json"
# N = 2 rehearsal on the one GPU (both ranks on device 0): RCCL refuses two ranks on one device,
# so this exercises the gloo fallback of the replicas-only metrics; the 8-GPU node runs RCCL
P2PMG_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline > "$O/b2.json" 2> "$O/b2.err" || { tail -30 "$O/b2.err"; exit 1; }
tail -c 700 "$O/b2.json"
