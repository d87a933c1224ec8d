"""configs[2] PMC summary: gpurun_out/pmc_c3_{fetch,write} -> profiles/r01_config3_pmc.json and
profiles/pmc_traffic_config3.json (bench.py --workload config3 reads the latter), reads x2 per
the gfx950 FETCH_SIZE rule calibrated in the configs[1] run (scripts/summarize_profiles.py)."""
import collections, csv, json, os, shutil, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out")


def avgs(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


f = avgs(os.path.join(O, "pmc_c3_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
w = avgs(os.path.join(O, "pmc_c3_write", "write_counter_collection.csv"), "WRITE_SIZE")
rows = {k: {"fetch_size_kb_raw": f.get(k, 0.0), "write_size_kb": w.get(k, 0.0),
            "read_bytes_corrected": 2 * f.get(k, 0.0) * 1024, "write_bytes": w.get(k, 0.0) * 1024,
            "hbm_bytes_corrected": (2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024} for k in sorted(set(f) | set(w))}
b = json.loads(open(os.path.join(O, "bench_c3.json")).read().strip().splitlines()[-1])
json.dump({"round": 1, "counters": "FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes "
                                   "(bench.py --workload config3 --steps 2 --warmup 1)",
           "correction": "reads x2 (gfx950 FETCH_SIZE halving); writes x1", "kernels": rows, "bench": b},
          open(os.path.join(ROOT, "profiles", "r01_config3_pmc.json"), "w"), indent=1)
k = [x for x in rows if "episode_sq16_kernel" in x][0]
json.dump({"workload": b["config"]["workload"], "kernel": k, "hbm_bytes_per_launch": rows[k]["hbm_bytes_corrected"],
           "read_bytes_per_launch": rows[k]["read_bytes_corrected"], "write_bytes_per_launch": rows[k]["write_bytes"],
           "source": "profiles/r01_config3_pmc.json"},
          open(os.path.join(ROOT, "profiles", "pmc_traffic_config3.json"), "w"), indent=1)
shutil.copy(os.path.join(O, "prof_c3", "c3_kernel_stats.csv"), os.path.join(ROOT, "profiles", "r01_config3_kernel_stats.csv"))
shutil.copy(os.path.join(O, "bench_c3.json"), os.path.join(ROOT, "profiles", "r01_config3_bench.json"))
shutil.copy(os.path.join(O, "prof_c5", "c5_kernel_stats.csv"), os.path.join(ROOT, "profiles", "r01_config5_kernel_stats.csv"))
shutil.copy(os.path.join(O, "bench_c5.json"), os.path.join(ROOT, "profiles", "r01_config5_bench.json"))
print(k[:60], {a: round(v / 1e9, 3) for a, v in rows[k].items() if "bytes" in a})
