"""Per-launch averages of the SQ counter passes written by scripts/gpu_sq_counters.sh.

usage: summarize_sq.py <gpurun_out dir> [<dest dir>]  (dest: one sq_<workload>.json per workload,
which bench.py reads for roofline.issue)

For each workload, the episode kernel's counters (first launch dropped as warm-up) averaged over
launches, plus derived figures: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md constants table), so cycles = 4 x counter."""
import collections
import csv
import glob
import json
import os
import sys

out_dir = sys.argv[1]
KERNEL = {"config2": "episode_fast_kernel", "config3": "episode_sq16_kernel", "config5": "dqn_train_kernel"}
SQ_ENGINES = 32  # SQ_BUSY_CYCLES sums the shader engines' busy cycles (bench.py issue roofline)
res = {}
for w, kname in KERNEL.items():
    agg = collections.defaultdict(list)
    for p in ("A", "B", "C"):
        files = glob.glob(os.path.join(out_dir, f"{w}_{p}", "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(files[0])):
            if kname in r["Kernel_Name"]:
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for c, d in per.items():
            vals = [d[k] for k in sorted(d)]
            vals = vals[1:] if len(vals) > 1 else vals
            agg[c] = sum(vals) / len(vals)
    if not agg:
        continue
    d = dict(agg)
    waves = d.get("SQ_WAVES", 0) or 1
    wc = d.get("SQ_WAVE_CYCLES", 0)
    der = {
        "wave_cycles_per_wave": 4 * wc / waves,
        "frac_wait_any": d.get("SQ_WAIT_ANY", 0) / wc if wc else None,
        "frac_wait_inst_any": d.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
        "frac_active_inst_any": d.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
        "valu_insts_per_wave": d.get("SQ_INSTS_VALU", 0) / waves,
        "salu_insts_per_wave": d.get("SQ_INSTS_SALU", 0) / waves,
        "vmem_rd_per_wave": d.get("SQ_INSTS_VMEM_RD", 0) / waves,
        "vmem_wr_per_wave": d.get("SQ_INSTS_VMEM_WR", 0) / waves,
        "lds_per_wave": d.get("SQ_INSTS_LDS", 0) / waves,
        # one wave alone issues a VALU every 4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost')
        "valu_issue_frac_of_one_wave_peak": (4 * d.get("SQ_INSTS_VALU", 0) / (4 * wc)) if wc else None,
        "launch_cycles": d.get("SQ_BUSY_CYCLES", 0) / SQ_ENGINES,
    }
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and d.get("SQ_BUSY_CYCLES"):
        # MFMA-busy cycles summed over the 1024 SIMDs, over the SIMD-cycles of the launch
        der["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * der["launch_cycles"])
    res[w] = {"kernel": kname, "workload": w, "counters_per_launch": d, "derived": der,
              "source": "scripts/gpu_sq_counters.sh (rocprofv3 --pmc, two passes of <= 8 SQ counters, P2PMG_NO_SPEC=1)"}
    if len(sys.argv) > 2:
        with open(os.path.join(sys.argv[2], f"sq_{w}.json"), "w") as fh:
            json.dump(res[w], fh, indent=1)
print(json.dumps(res, indent=1))
