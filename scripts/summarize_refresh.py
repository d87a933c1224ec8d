"""gpurun_out/<round> (scripts/gpu_refresh.sh <round>) -> committed summaries under profiles/.

usage: summarize_refresh.py ROUND   (e.g. r04)

Per workload: <round>_<tag>_bench.json (the bench line, roofline.traffic from this call's PMC passes),
<round>_<tag>_kernel_stats.csv (rocprofv3 --stats), <round>_<tag>_pmc.json and pmc_traffic[_<workload>].json
(which bench.py reads).  PMC: FETCH_SIZE and WRITE_SIZE from separate passes, reads x2 (gfx950
FETCH_SIZE halving, MI355X_MICROARCH.md), writes x1, averaged over the kernel's launches.
"""
import collections, csv, glob, json, os, shutil, sys

RND = sys.argv[1] if len(sys.argv) > 1 else "r04"
ROUND = int(RND.lstrip("r"))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out", RND)
P = os.path.join(ROOT, "profiles")


def avgs(name, counter):
    path = glob.glob(os.path.join(O, f"pmc_{name}_{counter}", "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def line(name):
    return json.loads(open(os.path.join(O, name + ".json")).read().strip().splitlines()[-1])


def do(tag, name, kernel_key, traffic_name):
    stats = glob.glob(os.path.join(O, f"prof_{name}", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(P, f"{RND}_{tag}_kernel_stats.csv"))
    b = line(name)
    if kernel_key:
        f, w = avgs(name, "FETCH_SIZE"), avgs(name, "WRITE_SIZE")
        rows = {k: {"fetch_size_kb_raw": f.get(k, 0.0), "write_size_kb": w.get(k, 0.0),
                    "read_bytes_corrected": 2 * f.get(k, 0.0) * 1024, "write_bytes": w.get(k, 0.0) * 1024,
                    "hbm_bytes_corrected": (2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024} for k in sorted(set(f) | set(w))}
        src = f"profiles/{RND}_{tag}_pmc.json"
        json.dump({"round": ROUND, "counters": "FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes "
                                               "(scripts/gpu_refresh.sh)",
                   "correction": "reads x2 (gfx950 FETCH_SIZE halving); writes x1", "kernels": rows},
                  open(os.path.join(ROOT, src), "w"), indent=1)
        k = [x for x in rows if kernel_key in x][0]
        json.dump({"workload": b["config"]["workload"], "kernel": k, "hbm_bytes_per_launch": rows[k]["hbm_bytes_corrected"],
                   "read_bytes_per_launch": rows[k]["read_bytes_corrected"], "write_bytes_per_launch": rows[k]["write_bytes"],
                   "source": src}, open(os.path.join(P, traffic_name), "w"), indent=1)
        b["roofline"]["traffic"] = rows[k]["hbm_bytes_corrected"]
        b["roofline"]["traffic_source"] = src
        print(tag, k[:70], "traffic", round(rows[k]["hbm_bytes_corrected"] / 1e6, 2), "MB vs algorithmic",
              round(b["roofline"].get("algorithmic_bytes_per_launch", 0) / 1e6, 2), "MB")
    json.dump(b, open(os.path.join(P, f"{RND}_{tag}_bench.json"), "w"))
    print(tag, b["value"], b["roofline"]["frac"], b["roofline"].get("kernel_ms"))


do("bench", "c2", "episode_fast_kernel", "pmc_traffic.json")
do("config3", "c3", "episode_sq16_kernel", "pmc_traffic_config3.json")
do("config4", "c4", "episode_fast_kernel", "pmc_traffic_config4.json")
do("config5", "c5", None, None)

# the launcher's 2-rank rehearsal on the one-GPU box, the instruction-rate microbenchmark, SQ counters
shutil.copy(os.path.join(O, "c2n2.json"), os.path.join(P, f"{RND}_bench_n2_launcher_rehearsal_one_gpu.json"))
if os.path.exists(os.path.join(O, "ubench_rate.jsonl")):
    shutil.copy(os.path.join(O, "ubench_rate.jsonl"), os.path.join(P, f"{RND}_ubench_rate.jsonl"))
import subprocess  # noqa: E402
subprocess.run(["python3", os.path.join(ROOT, "scripts", "summarize_sq.py"), os.path.join(O, "sq"), P], check=True,
               stdout=open(os.path.join(P, f"{RND}_sq_summary.json"), "w"))
