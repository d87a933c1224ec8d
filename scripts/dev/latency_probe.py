"""Ablation probe for the episode kernel's per-step latency (config 2 shape)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch
from oracle.restatement import GREEDY

def build(S, q_dtype="f64", bins=(20, 20, 20, 20), N=2, R=1, T=96):
    inp = scenario_batch(S, N, T)
    ov = dict(n_time_states=bins[0], n_temp_states=bins[1], n_balance_states=bins[2], n_p2p_states=bins[3])
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype, **ov)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
    return eng

def timeit(eng, mode="train", rng="philox", eps=0.5, record=("reward", "cost"), reps=8, philox="auto"):
    for e in range(2):
        eng.run_episode(mode, rng, episode=e, epsilon=eps, record=record, philox=philox)
    eng.sync()
    ms = []
    for e in range(reps):
        eng.run_episode(mode, rng, episode=10 + e, epsilon=eps, record=record, philox=philox)
        ms.append(eng.last_kernel_ms())
    return float(np.median(ms))

res = []
def rep(tag, ms, S, N=2, T=96):
    print(f"{tag:48s} {ms:8.3f} ms  {ms/T*1e3:7.2f} us/step  {S*N*T/ms*1e3:.3e} agent-steps/s", flush=True)

e = build(4096)
rep("S4096 f64 philox eps.5", timeit(e), 4096)
rep("S4096 f64 philox-inkernel eps.5", timeit(e, philox="inkernel"), 4096)
rep("S4096 f64 philox eps1", timeit(e, eps=1.0), 4096)
rep("S4096 f64 philox eps0", timeit(e, eps=0.0), 4096)
rep("S4096 f64 greedy", timeit(e, mode="greedy"), 4096)
rep("S4096 f64 philox eps.5 no-record", timeit(e, record=()), 4096)
codes = np.full((96, 2, 4096, 2), GREEDY, np.uint8); codes[np.random.rand(*codes.shape) < 0.5] = 1
e.set_replay_codes(codes)
rep("S4096 f64 replay eps.5", timeit(e, rng="replay"), 4096)
e.close()
e = build(4096, bins=(20, 20, 10, 10))
rep("S4096 f64 philox eps.5 bins 20x20x10x10", timeit(e), 4096); e.close()
e = build(4096, bins=(10, 10, 5, 5))
rep("S4096 f64 philox eps.5 bins 10x10x5x5", timeit(e), 4096); e.close()
for S in (256, 1024, 2048, 8192, 16384):
    e = build(S, q_dtype="f32")
    rep(f"S{S} f32 philox eps.5", timeit(e), S); e.close()
e = build(1024, N=16, R=1)
rep("S1024 N16 f64 philox eps.5", timeit(e), 1024, N=16); e.close()
