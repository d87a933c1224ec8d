#!/usr/bin/env python3
"""Where the wall time of a chained configs[1] launch goes: host call, kernel (HIP events), the
wait after it, the metric read-back; pre-pass hits and misses.  One GPU, configs[1] sizes.

    python scripts/probe_chain.py [n_chain] [reps] [chain: 1 | 0 = one launch per episode]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2pmicrogrid_amd.dataset import scenario_batch  # noqa: E402
from p2pmicrogrid_amd.engine import DeviceCommunityBatch  # noqa: E402
from bench import epsilon_at as eps_at  # noqa: E402  the bench's schedule (decay every 50 episodes)


def main(n=20, reps=4, chain=1):
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype="f64")
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    eng.set_timing_period(1)
    e = 0
    eng.run_episodes(e, [eps_at(k) for k in range(e, e + 5)], reset_sigma=0.3, record=("reward", "cost"),
                     next_epsilons=[eps_at(k) for k in range(5, 5 + n)])
    e = 5
    eng.sync()
    for r in range(reps):
        eng.reset_kernel_times()
        h0 = eng.prepass_stats()
        eng.sync()
        t0 = time.perf_counter()
        if chain:
            eng.run_episodes(e, [eps_at(k) for k in range(e, e + n)], reset_sigma=0.3, record=("reward", "cost"),
                             next_epsilons=[eps_at(k) for k in range(e + n, e + 2 * n)])
        else:
            for k in range(e, e + n):
                eng.run_episode("train", "philox", episode=k, epsilon=eps_at(k), record=("reward", "cost"),
                                reset_sigma=0.3, next_epsilon=eps_at(k + 1))
        t1 = time.perf_counter()
        eng.sync()
        t2 = time.perf_counter()
        rew = eng.episode_reward()
        t3 = time.perf_counter()
        kms = eng.kernel_times()
        h1 = eng.prepass_stats()
        if not chain and len(kms) > 1:
            kms = kms[1:] * n / (n - 1)  # the first launch's events also time its host-side start
        print(f"rep {r}: chain {chain} episodes {e}-{e + n - 1} call {1e6 * (t1 - t0):.1f} us, call+sync {1e6 * (t2 - t0):.1f} us, "
              f"read-back {1e6 * (t3 - t2):.1f} us, kernel {[round(1e3 * k, 1) for k in kms]} us, "
              f"per episode wall {1e6 * (t2 - t0) / n:.2f} kernel {1e3 * float(np.sum(kms)) / n:.2f} us, "
              f"pre-pass hits/misses {h1[0] - h0[0]}/{h1[1] - h0[1]}, mean reward {float(np.mean(rew)):.2f}", flush=True)
        e += n


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:4]])
