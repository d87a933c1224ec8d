#!/bin/bash
# L2 hit/miss and UTCL1 translation hit/miss of the fast kernel at 4096 vs 512 scenarios
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/pmcfp"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for S in 4096 512; do
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$O/s$S" -o p --output-format csv -- python3 "$R/scripts/probe_fp_one.py" $S > "$O/s$S.log" 2>&1 || { tail -20 "$O/s$S.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --kernel-trace -d "$O/l$S" -o p --output-format csv -- python3 "$R/scripts/probe_fp_one.py" $S > "$O/l$S.log" 2>&1 || { tail -20 "$O/l$S.log"; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob
for d in ("s4096", "s512", "l4096", "l512"):
    f = glob.glob(f"/root/repo/gpurun_out/pmcfp/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "episode_fast" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {k: round(sum(v[1:]) / max(1, len(v) - 1)) for k, v in agg.items()})
PY
