#!/bin/bash
# configs[1] fast kernel: main build vs gather ablations (a1: every Q gather faked, a8: the
# next-step rows faked), kernel time and SQ wait fraction (timing-only builds, never shipped)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r02abl"; mkdir -p "$O"
for L in p2pmicrogrid_amd/libp2pmg.so build/r02/libp2pmg_a1.so build/r02/libp2pmg_a8.so; do
  n=$(basename $L .so)
  P2PMG_LIB="$R/$L" timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print('$n', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
for L in build/r02/libp2pmg_a1.so build/r02/libp2pmg_a8.so; do
  n=$(basename $L .so)
  P2PMG_NO_SPEC=1 P2PMG_LIB="$R/$L" timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d "$O/sq_$n" -o p --output-format csv -- python3 "$R/bench.py" --steps 8 --warmup 1 --no-cpu-baseline > "$O/sq_$n.log" 2>&1 || { tail -20 "$O/sq_$n.log"; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for n in ("libp2pmg_a1", "libp2pmg_a8"):
    f = glob.glob(f"/root/repo/gpurun_out/r02abl/sq_{n}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "episode_fast" in r["Kernel_Name"]:
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    avg = {c: sum(sorted(d.values())[:]) / len(d) for c, d in per.items()}
    w = avg["SQ_WAVES"]
    print(n, {k: round(v / w) for k, v in avg.items()}, "wait frac", avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"])
PY
