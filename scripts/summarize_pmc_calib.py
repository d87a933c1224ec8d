"""gpurun_out/<round>/calib (scripts/gpu_calib.sh) -> profiles/<round>_pmc_calibration.json.

usage: summarize_pmc_calib.py ROUND

For each access pattern of scripts/pmc_calib.hip: the bytes it moves (printed by the probe) and the
FETCH_SIZE / WRITE_SIZE rocprofv3 reports for its launch (KB = 1024 B, separate passes), and their
ratio: counter bytes per byte moved.  MI355X_MICROARCH.md calibrates only 16-B/lane streaming reads
(0.5) and stores (1.0); these are the widths and patterns the episode kernels use.  Then the
configs[1] and configs[2] traffic re-derived from the raw counters with these factors
(profiles/pmc_traffic*.json keep the raw values)."""
import csv
import glob
import json
import os
import sys

RND = sys.argv[1] if len(sys.argv) > 1 else "r06"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out", RND, "calib")


def counter_rows(counter):
    path = glob.glob(os.path.join(O, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0) for r in rows]


def main():
    items = json.loads(open(os.path.join(O, "bytes.json")).read().strip().splitlines()[-1])
    fetch, write = counter_rows("FETCH_SIZE"), counter_rows("WRITE_SIZE")
    out = {"round": RND, "probe": "scripts/pmc_calib.hip (scripts/gpu_calib.sh)",
           "unit": "counter bytes (rocprofv3 KB x 1024) per byte the pattern moves", "patterns": {}}
    for it in items:
        k = it["launch"]  # 0-based position in launch order: fill, fill, then the patterns
        kf, f = fetch[k]
        kw, w = write[k]
        assert kf == kw, (kf, kw)
        out["patterns"][it["pattern"]] = {
            "kernel": kf, "bytes": it["bytes"], "dir": it["dir"], "fetch_size_bytes": f, "write_size_bytes": w,
            "factor": (f if it["dir"] == "read" else w) / it["bytes"]}
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{RND}_pmc_calibration.json"), "w"), indent=1)
    for name, p in out["patterns"].items():
        print(f"{name:10s} {p['dir']:5s} factor {p['factor']:.3f}  (fetch {p['fetch_size_bytes'] / p['bytes']:.3f}, "
              f"write {p['write_size_bytes'] / p['bytes']:.3f})")


if __name__ == "__main__":
    main()
