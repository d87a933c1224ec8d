"""Timing probe of episode_sq16_kernel variants at the configs[2] shape (N=16, shared table, battery).
Prints median episode-kernel ms per variant (HIP events stamped by the dispatch)."""
import json, sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch

S = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
inp = scenario_batch(S, 16, 96)
e = DeviceCommunityBatch(S, 16, 1, 96, q_dtype="f32", shared_q=True)
e.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
e.set_profiles(inp.load_w, inp.pv_w); e.set_max_in(inp.max_in); e.set_temperatures(inp.t_in0, inp.t_m0)
e.set_battery(3.6e7)
res = {}
variants = [("train inkernel", dict(mode="train", philox="auto", record=("reward", "cost"))),
            ("train prepass", dict(mode="train", philox="prepass", record=("reward", "cost"))),
            ("train norecord", dict(mode="train", philox="auto", record=())),
            ("greedy", dict(mode="greedy", philox="auto", record=("reward", "cost"))),
            ("train general", dict(mode="train", philox="auto", record=("reward", "cost"), kernel="general"))]
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
for name, kw in variants:
    if only and name not in only:
        continue
    mode = kw.pop("mode")
    for k in range(2):
        e.run_episode(mode, "philox", episode=k, epsilon=0.5, **kw)
        e.apply_q_delta()
    e.sync(); e.reset_kernel_times()
    t0 = time.perf_counter()
    for k in range(4):
        e.run_episode(mode, "philox", episode=3 + k, epsilon=0.5, **kw)
        e.apply_q_delta()
    e.sync()
    res[name + " wall"] = (time.perf_counter() - t0) / 4 * 1e3
    res[name] = float(np.median(e.kernel_times()))
    res[name + " kernel"] = e.last_kernel()
    print(name, res[name], "wall/episode", res[name + " wall"], flush=True)
print(json.dumps(res))
