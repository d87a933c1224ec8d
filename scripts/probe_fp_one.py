"""A few fused-reset training episodes at S scenarios (argv[1]) of the configs[1] shape, for PMC passes."""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch

S, N, R, T = int(sys.argv[1]), 2, 1, 96
inp = scenario_batch(S, N, T)
eng = DeviceCommunityBatch(S, N, R, T)
eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
for e in range(6):
    eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward", "cost"), reset_sigma=0.3,
                    scen_per_wave=0 if S >= 4096 else max(1, S // 256))
eng.sync()
print("done", S)
