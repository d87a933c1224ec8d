"""Timing-only ablation of the episode kernel's per-step latency (configs[1] shape).
Runs each library build in its own subprocess (P2PMG_LIB) and prints us/step."""
import os, subprocess, sys, json
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, numpy as np
sys.path.insert(0, %r)
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch, unpack_index
res = {}
for S in (256, 4096):
    for qd in ("f64", "f32"):
        inp = scenario_batch(S, 2, 96)
        e = DeviceCommunityBatch(S, 2, 1, 96, q_dtype=qd)
        e.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        e.set_profiles(inp.load_w, inp.pv_w); e.set_max_in(inp.max_in); e.set_temperatures(inp.t_in0, inp.t_m0)
        for mode in ("train", "greedy"):
            for k in range(3):
                e.run_episode(mode, "philox", episode=k, epsilon=0.5, record=("reward", "cost"))
            e.sync(); e.reset_kernel_times()
            for k in range(10):
                e.run_episode(mode, "philox", episode=3 + k, epsilon=0.5, record=("reward", "cost"))
            ms = float(np.median(e.kernel_times()))
            res[f"S{S} {qd} {mode}"] = ms / 96 * 1e3
        if S == 4096 and qd == "f64":
            e.run_episode("train", "philox", episode=50, epsilon=0.5, record=("index",))
            ip = unpack_index(e.get_record("index"))[:, 1, :, :, 3].ravel()
            res["ip_round1_hist"] = np.bincount(ip, minlength=20).tolist()
        e.close()
print(json.dumps(res))
''' % ROOT

out = {}
for name, lib in (("main", ""), ("noq", "build/libp2pmg_noq.so"), 
                  ("compute", "build/libp2pmg_compute.so")):
    env = dict(os.environ)
    if lib:
        env["P2PMG_LIB"] = os.path.join(ROOT, lib)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(name, "FAILED", r.stderr[-2000:]); sys.exit(1)
    out[name] = json.loads(r.stdout.strip().splitlines()[-1])
for k in out["main"]:
    if k.startswith("ip_"):
        continue
    print(f"{k:24s} " + "  ".join(f"{n}={out[n][k]:6.3f}us" for n in out))
h = np.array(out["main"]["ip_round1_hist"]); h = h / h.sum()
print("round-1 ip histogram:", np.round(h, 3).tolist())
print("P(ip in 8..11) =", h[8:12].sum(), " P(ip in 8..15) =", h[8:16].sum())
