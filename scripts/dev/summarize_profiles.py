"""Turn rocprofv3 outputs under gpurun_out/ into committed summaries under profiles/.

    python scripts/summarize_profiles.py --round 1 [--tag bench]

Writes profiles/r{NN}_{tag}_kernel_stats.csv (the --stats summary, verbatim),
profiles/r{NN}_{tag}_pmc.json (per-kernel FETCH_SIZE / WRITE_SIZE averages, gfx950-corrected) and
profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half of the bytes of coalesced
streaming reads.  Calibrated here on this repo's own known-byte kernels in the same run:
prof_pack_kernel reads exactly A*T*8 bytes (4-B coalesced loads) and its FETCH_SIZE reads half of
it; its writes (A*T*8 B) and the Philox pre-pass writes (T*A*4 B) read exactly.  The episode
kernel's 16-B-per-lane Q-row gathers are a different access shape; the x2 read correction is
applied to them too and flagged as calibrated-on-streams only.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def kernel_avgs(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", type=int, default=1)
    ap.add_argument("--tag", default="bench")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--bench-json", default=None)
    args = ap.parse_args()
    pre = os.path.join(ROOT, "profiles", f"r{args.round:02d}_{args.tag}")
    os.makedirs(os.path.dirname(pre), exist_ok=True)
    o = args.out
    stats = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(o, "prof_bench")) for f in fs
             if f.endswith("kernel_stats.csv")]
    if stats:
        shutil.copy(stats[0], pre + "_kernel_stats.csv")
    fetch = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(o, "pmc_fetch")) for f in fs
             if f.endswith("counter_collection.csv")]
    write = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(o, "pmc_write")) for f in fs
             if f.endswith("counter_collection.csv")]
    if not (fetch and write):
        print("no PMC csv found")
        return
    fk = kernel_avgs(fetch[0], "FETCH_SIZE")
    wk = kernel_avgs(write[0], "WRITE_SIZE")
    rows = {}
    for k in sorted(set(fk) | set(wk)):
        f_kb, w_kb = fk.get(k, 0.0), wk.get(k, 0.0)
        rows[k] = {"fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
                   "read_bytes_corrected": 2 * f_kb * 1024, "write_bytes": w_kb * 1024,
                   "hbm_bytes_corrected": (2 * f_kb + w_kb) * 1024}
    epi = [k for k in rows if "episode_kernel" in k or "episode_fast_kernel" in k]
    summary = {"round": args.round, "counters": "FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes",
               "correction": "reads x2 (gfx950 FETCH_SIZE halving, calibrated on prof_pack_kernel); writes x1",
               "kernels": rows}
    if args.bench_json and os.path.exists(args.bench_json):
        b = json.loads(open(args.bench_json).read().strip().splitlines()[-1])
        summary["bench"] = b
    json.dump(summary, open(pre + "_pmc.json", "w"), indent=1)
    if epi:
        k = epi[0]
        import bench  # noqa: F401  (workload string must match bench.py's)
        b = summary.get("bench", {})
        wl = b.get("config", {}).get("workload")
        traffic = {"workload": wl, "kernel": k, "hbm_bytes_per_launch": rows[k]["hbm_bytes_corrected"],
                   "read_bytes_per_launch": rows[k]["read_bytes_corrected"],
                   "write_bytes_per_launch": rows[k]["write_bytes"],
                   "source": os.path.relpath(pre + "_pmc.json", ROOT)}
        json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
        print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
