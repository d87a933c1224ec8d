"""configs[3] PMC summary: gpurun_out/pmc_c4_{fetch,write} -> profiles/r01_config4_pmc.json and
profiles/pmc_traffic_config4.json (bench.py --workload config4 reads the latter); reads x2 per the
gfx950 FETCH_SIZE rule (MI355X_MICROARCH.md), writes x1.  Also copies the kernel stats and the bench line."""
import collections, csv, json, os, shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out")


def avgs(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


f = avgs(os.path.join(O, "pmc_c4_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
w = avgs(os.path.join(O, "pmc_c4_write", "write_counter_collection.csv"), "WRITE_SIZE")
rows = {k: {"fetch_size_kb_raw": f.get(k, 0.0), "write_size_kb": w.get(k, 0.0),
            "read_bytes_corrected": 2 * f.get(k, 0.0) * 1024, "write_bytes": w.get(k, 0.0) * 1024,
            "hbm_bytes_corrected": (2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024} for k in sorted(set(f) | set(w))}
b = json.loads(open(os.path.join(O, "bench_c4_8192.json")).read().strip().splitlines()[-1])
json.dump({"round": 1, "counters": "FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes "
                                   "(bench.py --workload config4 --steps 1 --warmup 1)",
           "correction": "reads x2 (gfx950 FETCH_SIZE halving); writes x1", "kernels": rows, "bench": b},
          open(os.path.join(ROOT, "profiles", "r01_config4_pmc.json"), "w"), indent=1)
k = [x for x in rows if "episode_fast_kernel" in x][0]
json.dump({"workload": b["config"]["workload"], "kernel": k, "hbm_bytes_per_launch": rows[k]["hbm_bytes_corrected"],
           "read_bytes_per_launch": rows[k]["read_bytes_corrected"], "write_bytes_per_launch": rows[k]["write_bytes"],
           "source": "profiles/r01_config4_pmc.json"},
          open(os.path.join(ROOT, "profiles", "pmc_traffic_config4.json"), "w"), indent=1)
shutil.copy(os.path.join(O, "prof_c4", "c4_kernel_stats.csv"), os.path.join(ROOT, "profiles", "r01_config4_kernel_stats.csv"))
shutil.copy(os.path.join(O, "bench_c4_8192.json"), os.path.join(ROOT, "profiles", "r01_config4_bench.json"))
print(k[:60], {a: round(v / 1e9, 3) for a, v in rows[k].items() if "bytes" in a})
