"""DQN (configs[4] shape) episode wall time vs agents_per_block (gradient partials per step)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.dqn import DeviceDQNBatch

S, N, R, T = 4096, 2, 1, 96
inp = scenario_batch(S, N, T)
for apb in [int(x) for x in (sys.argv[1:] or ["4", "8", "16"])]:
    eng = DeviceDQNBatch(S, N, R, T, shared=True, agents_per_block=apb, init_seed=0)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
    eng.run_episode("fill", "philox", episode=0, epsilon=1.0, record=("reward", "cost"))
    eng.run_episode("train", "philox", episode=1, epsilon=0.9, record=("reward", "cost"))
    eng.sync()
    t0 = time.perf_counter()
    for e in range(2, 5):
        eng.run_episode("train", "philox", episode=e, epsilon=0.9 ** e, record=("reward", "cost"))
    eng.sync()
    print(f"apb={apb:3d}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms per episode", flush=True)
    eng.close()
