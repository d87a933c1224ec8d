"""Episode kernel time vs Q-table footprint (configs[1] shape, T0 reset fused): f64 vs f32 tables,
4096 vs 512 scenarios (same per-wave work when every wave has its own CU)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch

N, R, T = 2, 1, 96
for S, qd, spw in ((4096, "f64", 0), (4096, "f32", 0), (512, "f64", 2), (512, "f64", 0), (4096, "f64", 0)):
    inp = scenario_batch(S, N, T)
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype=qd)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w); eng.set_max_in(inp.max_in); eng.set_temperatures(inp.t_in0, inp.t_m0)
    for e in range(5):
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward", "cost"), reset_sigma=0.3, scen_per_wave=spw)
    eng.sync(); eng.reset_kernel_times()
    for e in range(5, 45):
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward", "cost"), reset_sigma=0.3, scen_per_wave=spw)
    eng.sync()
    print(f"S={S} {qd} spw={spw}: episode kernel {float(np.mean(eng.kernel_times())) * 1e3:.1f} us", flush=True)
    eng.close()
