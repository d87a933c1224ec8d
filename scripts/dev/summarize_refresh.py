"""gpurun_out/refresh (scripts/gpu_refresh_profiles.sh) -> committed summaries under profiles/.

configs[1] -> r01_bench_{kernel_stats.csv,pmc.json}, r01_bench.json, pmc_traffic.json
configs[3] -> r01_config4_{kernel_stats.csv,pmc.json}, r01_config4_bench.json, pmc_traffic_config4.json
configs[4] -> r01_config5_kernel_stats.csv, r01_config5_bench.json
PMC: FETCH_SIZE and WRITE_SIZE from separate rocprofv3 --pmc passes, reads x2 (gfx950 FETCH_SIZE
halving, MI355X_MICROARCH.md), writes x1.  The bench lines' roofline.traffic is set from the PMC
passes of the same call (bench.py reads pmc_traffic*.json, which this script rewrites).
"""
import collections, csv, json, os, shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out", "refresh")
P = os.path.join(ROOT, "profiles")


def avgs(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def line(name):
    return json.loads(open(os.path.join(O, name)).read().strip().splitlines()[-1])


def do(tag, bench_file, prof, pmc, traffic_name, cmd):
    shutil.copy(os.path.join(O, prof, f"{prof.split('_')[1]}_kernel_stats.csv"), os.path.join(P, f"r01_{tag}_kernel_stats.csv"))
    b = line(bench_file)
    if pmc:
        f = avgs(os.path.join(O, f"pmc_{pmc}_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
        w = avgs(os.path.join(O, f"pmc_{pmc}_write", "write_counter_collection.csv"), "WRITE_SIZE")
        rows = {k: {"fetch_size_kb_raw": f.get(k, 0.0), "write_size_kb": w.get(k, 0.0),
                    "read_bytes_corrected": 2 * f.get(k, 0.0) * 1024, "write_bytes": w.get(k, 0.0) * 1024,
                    "hbm_bytes_corrected": (2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024} for k in sorted(set(f) | set(w))}
        src = f"profiles/r01_{tag}_pmc.json"
        json.dump({"round": 1, "counters": f"FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes ({cmd})",
                   "correction": "reads x2 (gfx950 FETCH_SIZE halving); writes x1", "kernels": rows, "bench": b},
                  open(os.path.join(ROOT, src), "w"), indent=1)
        k = [x for x in rows if "episode_fast_kernel" in x][0]
        json.dump({"workload": b["config"]["workload"], "kernel": k, "hbm_bytes_per_launch": rows[k]["hbm_bytes_corrected"],
                   "read_bytes_per_launch": rows[k]["read_bytes_corrected"], "write_bytes_per_launch": rows[k]["write_bytes"],
                   "source": src}, open(os.path.join(P, traffic_name), "w"), indent=1)
        b["roofline"]["traffic"] = rows[k]["hbm_bytes_corrected"]
        b["roofline"]["traffic_source"] = src
        print(tag, k[:60], "traffic", rows[k]["hbm_bytes_corrected"] / 1e6, "MB vs algorithmic",
              b["roofline"].get("algorithmic_bytes_per_launch", 0) / 1e6, "MB")
    json.dump(b, open(os.path.join(P, f"r01_{tag}_bench.json" if tag != "bench" else "r01_bench.json"), "w"))
    print(tag, b["value"], b["roofline"]["frac"])


do("bench", "c1.json", "prof_c1", "c1", "pmc_traffic.json", "bench.py --steps 6 --warmup 1")
do("config4", "c4.json", "prof_c4", "c4", "pmc_traffic_config4.json", "bench.py --workload config4 --steps 1 --warmup 1")
do("config5", "c5.json", "prof_c5", None, None, "")
