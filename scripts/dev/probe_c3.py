"""Timing probe of the config3 shape (N=16, shared table, battery): which part costs what.
Each library build runs in its own subprocess (P2PMG_LIB); prints ms per episode kernel."""
import json, os, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, numpy as np
sys.path.insert(0, %r)
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch
S = int(sys.argv[1]); res = {}
inp = scenario_batch(S, 16, 96)
for bat in (True, False):
    e = DeviceCommunityBatch(S, 16, 1, 96, q_dtype="f32", shared_q=True)
    e.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    e.set_profiles(inp.load_w, inp.pv_w); e.set_max_in(inp.max_in); e.set_temperatures(inp.t_in0, inp.t_m0)
    if bat:
        e.set_battery(3.6e7)
    for mode in ("train", "greedy"):
        for k in range(2):
            e.run_episode(mode, "philox", episode=k, epsilon=0.5, record=("reward", "cost"))
        e.sync(); e.reset_kernel_times()
        for k in range(4):
            e.run_episode(mode, "philox", episode=3 + k, epsilon=0.5, record=("reward", "cost"))
        res[f"S{S} bat={bat} {mode}"] = float(np.median(e.kernel_times()))
    if bat:
        d = e.get_q_delta()
        res["distinct_delta_entries"] = int(np.count_nonzero(d))
    e.close()
print(json.dumps(res))
''' % ROOT
out = {}
for name, lib in (("main", ""), ("noatomic", "build/libp2pmg_noatomic.so")):
    env = dict(os.environ)
    if lib:
        env["P2PMG_LIB"] = os.path.join(ROOT, lib)
    for S in sys.argv[1:] or ["125000"]:
        r = subprocess.run([sys.executable, "-c", CHILD, S], env=env, capture_output=True, text=True, timeout=500)
        if r.returncode != 0:
            print(r.stderr[-3000:]); sys.exit(r.returncode)
        out[f"{name} {S}"] = json.loads(r.stdout.strip().splitlines()[-1])
print(json.dumps(out, indent=1))
