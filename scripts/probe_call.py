#!/usr/bin/env python3
"""Host-side cost of one chained launch call (configs[1] sizes): the engine wrapper against the bare
ctypes call with prepared arguments, and a bare p2pmg_run_episode for comparison.  The device is
synchronised before each timed call, so each call starts from an idle queue.

    python scripts/probe_call.py
"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import epsilon_at  # noqa: E402
from p2pmicrogrid_amd import _lib  # noqa: E402
from p2pmicrogrid_amd.dataset import scenario_batch  # noqa: E402
from p2pmicrogrid_amd.engine import DeviceCommunityBatch  # noqa: E402


def main():
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype="f64")
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    eng.set_timing_period(1)
    sched = np.array([epsilon_at(e) for e in range(400)])
    e = 0
    n = 20
    eng.run_episodes(e, sched[e:e + n], reset_sigma=0.3, record=("reward", "cost"), next_epsilons=sched[e + n:e + 2 * n])
    e += n
    for rep in range(5):
        eng.sync()
        t0 = time.perf_counter()
        eng.run_episodes(e, sched[e:e + n], reset_sigma=0.3, record=("reward", "cost"),
                         next_epsilons=sched[e + n:e + 2 * n])
        t1 = time.perf_counter()
        eng.sync()
        e += n
        # the bare call with every argument prepared
        args = _lib.EpisodeArgs(_lib.MODE_TRAIN, _lib.RNG_PHILOX, e, _lib.REC["reward"] | _lib.REC["cost"],
                                float(sched[e]), _lib.FLAG_RESET_T0, 0, 0.3, 0.0)
        eps = np.ascontiguousarray(sched[e:e + n])
        nxt = np.ascontiguousarray(sched[e + n:e + 2 * n])
        ref, nptr = C.byref(args), nxt.ctypes.data
        eng.sync()
        t2 = time.perf_counter()
        eng.L.p2pmg_run_episodes(eng._ctx, ref, n, eps, n, nptr)
        t3 = time.perf_counter()
        eng.sync()
        e += n
        print(f"rep {rep}: engine.run_episodes {1e6 * (t1 - t0):.1f} us, bare ctypes call {1e6 * (t3 - t2):.1f} us",
              flush=True)
    for rep in range(3):
        eng.sync()
        t0 = time.perf_counter()
        eng.run_episode("train", "philox", episode=e, epsilon=float(sched[e]), record=("reward", "cost"),
                        reset_sigma=0.3, next_epsilon=float(sched[e + 1]))
        t1 = time.perf_counter()
        eng.sync()
        e += 1
        print(f"single run_episode {1e6 * (t1 - t0):.1f} us", flush=True)


if __name__ == "__main__":
    main()
