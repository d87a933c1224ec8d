"""Re-derive the episode kernels' HBM traffic (profiles/pmc_traffic*.json) with the measured counter
factors of profiles/r06_pmc_calibration.json instead of round 1-5's uniform x2 on FETCH_SIZE.

usage: recalibrate_traffic.py [CALIBRATION_JSON]

The calibration (scripts/pmc_calib.hip, known byte counts far past the Infinity Cache) gives, in
counter bytes per byte moved: coalesced 4/8-B reads 0.5 (the guide's streaming halving), 32-B random
row gathers 2.0 (a 64-B tally per row), 16-B row gathers 4.08, coalesced stores 1.0, 8-B scattered
stores 4.0 (the 32-B sector) and 32-B scattered stores 1.05.  A kernel's FETCH_SIZE mixes its streamed
inputs with its row gathers, and only the gathers that miss L2 reach the counter.  So the raw reads
are split by the kernel's own stream bytes per agent-step (bench.py sector_model / SURVEY §8d), taken
as read from the fabric once (counted at 0.5), and the rest is read as row gathers at their factor:

    reads  = stream_bytes + (FETCH_raw - 0.5 * stream_bytes) / f_gather
    writes = WRITE_raw     (exact for coalesced stores; an 8-B scattered store writes its 32-B sector)

The raw counter values stay in each file (`raw`); `hbm_bytes_calibrated_*` is what bench.py reports
as roofline.traffic."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")

# per agent-step: streamed read bytes and the row-gather pattern of each benched kernel
#   config2 episode_fast_kernel<2,f64,2,train>: profile 8 + pre-pass word 8 + code word 4 + round-1 bins 4
#           + the producer blocks' profile re-read for the next episode's pre-pass 8
#   config3 episode_sq16_kernel<f32,...>: step word 8 + its scenario's env row (32 B per 16 agents) 2
#   config4 episode_fast_kernel<4,f64,2,train,battery>: profile 8 + pre-pass word 8 + code word 4 + re-read 8
KERNELS = {
    "pmc_traffic.json": {"stream": 32.0, "gather": "gather32", "agent_steps": 4096 * 2 * 96},
    "pmc_traffic_config3.json": {"stream": 10.0, "gather": "gather16", "agent_steps": 125000 * 16 * 96},
    "pmc_traffic_config4.json": {"stream": 28.0, "gather": "gather32", "agent_steps": 8192 * 4 * 35040},
}


def main():
    cal_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(P, "r06_pmc_calibration.json")
    cal = json.load(open(cal_path))["patterns"]
    f_stream = cal["stream8"]["factor"]
    for name, k in KERNELS.items():
        path = os.path.join(P, name)
        d = json.load(open(path))
        raw = d.get("raw") or {
            # rounds 1-5 stored FETCH x 2 as the read bytes: undo it
            "fetch_size_bytes_per_launch": d["read_bytes_per_launch"] / 2.0,
            "write_size_bytes_per_launch": d["write_bytes_per_launch"],
        }
        if "hbm_bytes_per_episode" in d and "raw_per_episode" not in d:
            raw_ep = {"fetch_size_bytes_per_episode": d["read_bytes_per_episode"] / 2.0,
                      "write_size_bytes_per_episode": d["write_bytes_per_episode"]}
        else:
            raw_ep = d.get("raw_per_episode")
        d["raw"] = raw
        f_g = cal[k["gather"]]["factor"]
        eps_per_launch = d.get("episodes_per_launch", 1)

        def calib(fetch, write, episodes):
            stream = k["stream"] * k["agent_steps"] * episodes
            gathers = max(0.0, fetch - f_stream * stream) / f_g
            return stream + gathers, write, gathers

        r, w, g = calib(raw["fetch_size_bytes_per_launch"], raw["write_size_bytes_per_launch"], eps_per_launch)
        d["hbm_bytes_calibrated_per_launch"] = r + w
        d["read_bytes_calibrated_per_launch"] = r
        d["gather_read_bytes_calibrated_per_launch"] = g
        if raw_ep:
            d["raw_per_episode"] = raw_ep
            r1, w1, g1 = calib(raw_ep["fetch_size_bytes_per_episode"], raw_ep["write_size_bytes_per_episode"], 1)
            d["hbm_bytes_calibrated_per_episode"] = r1 + w1
            d["read_bytes_calibrated_per_episode"] = r1
            d["gather_read_bytes_calibrated_per_episode"] = g1
        single = d.get("one_launch_per_episode")
        if single:  # the one-launch-per-episode figure (rounds 1-5 stored FETCH x 2 there too)
            raw1 = single.get("raw") or {"fetch_size_bytes_per_launch": single["read_bytes_per_launch"] / 2.0,
                                         "write_size_bytes_per_launch": single["write_bytes_per_launch"]}
            single["raw"] = raw1
            r1, w1, g1 = calib(raw1["fetch_size_bytes_per_launch"], raw1["write_size_bytes_per_launch"], 1)
            single["hbm_bytes_calibrated_per_launch"] = r1 + w1
            single["read_bytes_calibrated_per_launch"] = r1
            single["gather_read_bytes_calibrated_per_launch"] = g1
        d["calibration"] = {"source": os.path.relpath(cal_path, ROOT), "stream_read_bytes_per_agent_step": k["stream"],
                            "stream_factor": f_stream, "gather_pattern": k["gather"], "gather_factor": f_g,
                            "model": "reads = stream + (FETCH_raw - f_stream * stream) / f_gather; writes = WRITE_raw"}
        d["counters"] = ("FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes; read_bytes_* / hbm_bytes_* keep "
                         "rounds 1-5's uniform x2 on FETCH_SIZE, *_calibrated_* use the measured factors (round 6)")
        json.dump(d, open(path, "w"), indent=1)
        per = d.get("hbm_bytes_calibrated_per_episode", d["hbm_bytes_calibrated_per_launch"] / eps_per_launch)
        print(f"{name}: calibrated {per / 1e6:.1f} MB per episode (uniform x2: "
              f"{d.get('hbm_bytes_per_episode', d['hbm_bytes_per_launch'] / eps_per_launch) / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
