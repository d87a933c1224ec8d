"""Quick timing probe of the episode kernel (config 2: 4096 scenarios x thesis community)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch

for q_dtype in ("f64", "f32"):
    for S in (4096, 16384):
        N, R, T = 2, 1, 96
        inp = scenario_batch(S, N, T)
        eng = DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype)
        eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
        for e in range(3):
            eng.run_episode("train", "philox", episode=e, epsilon=0.81, record=("reward", "cost"))
        eng.sync()
        ms = []
        t0 = time.perf_counter()
        for e in range(10):
            eng.run_episode("train", "philox", episode=3 + e, epsilon=0.5, record=("reward", "cost"))
            ms.append(eng.last_kernel_ms())
        wall = (time.perf_counter() - t0) / 10
        steps = S * N * T
        print(f"{q_dtype} S={S}: kernel {np.mean(ms):.3f} ms (min {np.min(ms):.3f}), wall/ep {wall*1e3:.3f} ms, "
              f"{steps/np.mean(ms)*1e3:.3e} agent-steps/s", flush=True)
        eng.close()
