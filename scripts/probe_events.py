"""configs[1] wall time per episode with and without dispatch-stamped timing events (P2PMG_NO_EVENTS)."""
import os, sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch

S, N, R, T = 4096, 2, 1, 96
inp = scenario_batch(S, N, T)
eng = DeviceCommunityBatch(S, N, R, T)
eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
for rep in range(2):
    for e in range(5):
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward", "cost"), reset_sigma=0.3)
    eng.sync()
    t0 = time.perf_counter()
    for e in range(5, 205):
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward", "cost"), reset_sigma=0.3)
    eng.sync()
    print(f"events={'off' if os.environ.get('P2PMG_NO_EVENTS') else 'on'}: wall {(time.perf_counter() - t0) / 200 * 1e6:.1f} us/episode", flush=True)
