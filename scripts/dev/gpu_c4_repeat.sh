#!/bin/bash
# configs[3] timing repeated (noise check) + configs[1] FETCH/WRITE PMC passes
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out"; mkdir -p "$O"
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu-baseline > "$O/rc4.json" 2> "$O/rc4.err" || { tail -20 "$O/rc4.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/rc4.json').read().splitlines()[-1]); print('c4', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmcq_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmcq_fetch.log" 2>&1 || { tail -20 "$O/pmcq_fetch.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmcq_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmcq_write.log" 2>&1 || { tail -20 "$O/pmcq_write.log"; exit 1; }
python3 - <<'PY'
import csv, collections
for n, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"/root/repo/gpurun_out/pmcq_{n}/{n}_counter_collection.csv")):
        if "episode_fast" in r["Kernel_Name"] and r["Counter_Name"] == c: agg[c].append(float(r["Counter_Value"]))
    print(c, sum(agg[c]) / len(agg[c]), "KB")
PY
