"""Q-row access trace of the configs[1] workload (4096 x 2 agents, R = 1, T = 96, per-agent f64
tables), for the row-cache study of DESIGN.md §8.1: after `--warmup` training episodes (the bench's
epsilon schedule), `--episodes` more are run one launch each with the packed state-index record
(the rows the episode's greedy reads and TD updates touch: every round's state of every step).
Writes the first `--agents` agents' indices, [episodes][T][R+1][agents] int32, to an npz.

    python scripts/trace_rows.py --out gpurun_out/r06/rows.npz

scripts/row_cache_sim.py then replays them through per-agent row caches."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--episodes", type=int, default=12)
    ap.add_argument("--agents", type=int, default=1024)
    a = ap.parse_args()
    import bench
    from p2pmicrogrid_amd.dataset import scenario_batch
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype="f64")
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    eps = [bench.epsilon_at(e) for e in range(a.warmup + a.episodes)]
    if a.warmup:
        eng.run_episodes(0, eps[:a.warmup], reset_sigma=0.3)
    out = np.empty((a.episodes, T, R + 1, a.agents), np.int32)
    for k in range(a.episodes):
        e = a.warmup + k
        eng.run_episode("train", "philox", episode=e, epsilon=eps[e], record=("index",), reset_sigma=0.3)
        out[k] = eng.get_record("index").reshape(T, R + 1, -1)[:, :, :a.agents]
    eng.close()
    np.savez_compressed(a.out, index=out, warmup=a.warmup, epsilons=np.asarray(eps[a.warmup:]))
    print("wrote", a.out, out.shape, flush=True)


if __name__ == "__main__":
    main()
