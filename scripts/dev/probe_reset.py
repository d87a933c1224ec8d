"""configs[1]: episode kernel time with the T0 reset fused, as a separate launch, or absent."""
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
rec = ("reward", "cost")
for variant in ("none", "fused", "separate", "none", "fused"):
    def ep(e):
        if variant == "fused":
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=rec, reset_sigma=0.3)
        else:
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=rec)
            if variant == "separate":
                eng.reset_temperatures_philox(e + 1, 0.3)
    for e in range(5):
        ep(e)
    eng.sync(); eng.reset_kernel_times()
    t0 = time.perf_counter()
    for e in range(5, 105):
        ep(e)
    eng.sync()
    wall = (time.perf_counter() - t0) / 100 * 1e6
    print(f"{variant:9s}: wall {wall:.1f} us/episode, episode kernel {float(np.mean(eng.kernel_times())) * 1e3:.1f} us", flush=True)
