"""Dev probe: host-side cost of one run_episode call (tiny T so the GPU is never the limit)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch
from p2pmicrogrid_amd import _lib

for T in (1, 96):
    S, N, R = 4096, 2, 1
    inp = scenario_batch(S, N, T)
    eng = DeviceCommunityBatch(S, N, R, T)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
    for variant in ("reset_fused", "reset_separate", "no_record", "general"):
        kw = dict(record=("reward", "cost"))
        if variant == "no_record": kw = {}
        if variant == "general": kw["kernel"] = "general"
        for e in range(5):
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, **kw)
        eng.sync()
        n = 200
        t0 = time.perf_counter()
        for e in range(n):
            if variant == "reset_separate":
                eng.run_episode("train", "philox", episode=e, epsilon=0.5, **kw)
                eng.reset_temperatures_philox(e + 1, 0.3)
            else:
                eng.run_episode("train", "philox", episode=e, epsilon=0.5, reset_sigma=0.3, **kw)
        t_host = (time.perf_counter() - t0) / n
        eng.sync()
        t_all = (time.perf_counter() - t0) / n
        print(f"T={T} {variant:15s} host submit {t_host*1e6:7.1f} us/episode, wall {t_all*1e6:7.1f} us/episode", flush=True)
    eng.close()
L = _lib.lib()
t0 = time.perf_counter()
for _ in range(10000):
    L.p2pmg_abi_version()
print(f"ctypes no-op call {(time.perf_counter()-t0)/10000*1e6:.2f} us")
