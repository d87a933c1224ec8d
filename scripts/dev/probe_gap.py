"""configs[1]: gap between back-to-back episode launches (wall per episode - kernel time) vs the
bytes each episode writes (records off / narrow / full)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch

S, N, R, T = 4096, 2, 1, 96
inp = scenario_batch(S, N, T)
eng = DeviceCommunityBatch(S, N, R, T)
eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
for rec in [(), ("reward", "cost"), ("reward", "cost", "grid", "p2p", "t_in", "action", "index")]:
    for rs in (None, 0.3):
        for e in range(5):
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=rec, reset_sigma=rs)
        eng.sync(); eng.reset_kernel_times()
        t0 = time.perf_counter()
        n = 100
        for e in range(5, 5 + n):
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=rec, reset_sigma=rs)
        eng.sync()
        wall = (time.perf_counter() - t0) / n * 1e6
        k = float(np.mean(eng.kernel_times())) * 1e3
        print(f"records={len(rec)} reset={rs}: wall {wall:.1f} us, kernel {k:.1f} us, gap {wall - k:.1f} us", flush=True)
