#!/usr/bin/env python3
"""configs[1] Q-row working set per agent, from the oracle (CPU only): would an on-chip row cache
take the dependent gather off episode_fast_kernel's chain?

The bench workload (BASELINE configs[1]: thesis community N = 2, R = 1, T = 96, per-agent f64
tables, Philox exploration, the reference's epsilon schedule, T0 reset every episode) is run by
oracle/restatement.py on a sample of its scenarios (every scenario is independent, so per-agent
statistics do not depend on the batch).  For every agent-step the rows the fast kernel gathers are
reconstructed (p2pmg_kernels.hip episode_fast_kernel, N = 2 candidate path):
  * the round-0 row (strip + ip 10) when round 0 is greedy (exploring lanes skip it);
  * the three round-1 candidates, strip + ip(partner's round-0 action a'), a' = 0, 1, 2;
  * the next-state row (next time / balance bins, the same temperature bin, ip 10).
Reported: distinct rows per agent per time bin (it) per episode; the hit rate of a per-agent LRU
cache of C rows (C = 160: 160 KB of LDS / 32 agents per CU / 32-B f64 rows) over the gather stream;
and the hit rate of a "next time bin" bulk load (the rows the agent touched in the same time bin of
the previous episode), with that set's size.  Output: one JSON document.

    python scripts/working_set.py [--scenarios 256] [--episodes 50] [--capacity 160] > profiles/r05_working_set.json
"""
import argparse
import collections
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import philox  # noqa: E402
from oracle.restatement import F32, OracleBatch, state_index  # noqa: E402
from p2pmicrogrid_amd.dataset import scenario_batch  # noqa: E402


def epsilon_at(e, eps0=0.81, decay=0.9, every=50, floor=0.1):
    n = 0 if e == 0 else (e - 1) // every + 1
    eps = eps0
    for _ in range(n):
        eps = max(floor, decay * eps)
    return eps


def rows_of_episode(ob, inp, out, seed, episode, eps, gids):
    """[T, 5, A] int64 rows gathered per agent-step (-1: not gathered), in issue order."""
    S, N, T = ob.S, ob.N, ob.T
    idx = out["idx"]  # [T, R+1, S, N, 4]
    it, iT, ib = idx[:, 0, ..., 0], idx[:, 0, ..., 1], idx[:, 0, ..., 2]
    strip = ((it * 20 + iT) * 20 + ib) * 20  # [T, S, N]
    rows = np.full((T, 5, S, N), -1, np.int64)
    mi = ob.max_in
    lv = ob.hp_levels
    for t in range(T):
        u, _ = philox.decision_draws(seed, episode, gids.ravel(), t, 0, ob.R)
        greedy0 = u.reshape(S, N) >= eps
        rows[t, 0] = np.where(greedy0, strip[t] + 10, -1)
        bal = (ob.load_w[:, :, t] - ob.pv_w[:, :, t]) / mi
        for ap in range(3):  # the partner's round-0 action a'
            out_p = (bal * mi) + lv[:, :, ap]
            ev0_p = (out_p * F32(1)) / F32(N)
            ev0_partner = ev0_p[:, ::-1]  # N = 2: the partner is the other lane
            p2pf = ((-ev0_partner) / F32(N)) / mi
            ip = state_index(p2pf, 20, "plain")
            rows[t, 1 + ap] = strip[t] + ip
        tn = (t + 1) % T
        itn = state_index(np.broadcast_to(inp.time[tn], (S, N)), 20, "time")
        baln = (ob.load_w[:, :, tn] - ob.pv_w[:, :, tn]) / mi
        ibn = state_index(baln, 20, "plain")
        rows[t, 4] = ((itn * 20 + iT[t]) * 20 + ibn) * 20 + 10
    return rows.reshape(T, 5, S * N), it.reshape(T, S * N)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenarios", type=int, default=256)
    ap.add_argument("--episodes", type=int, default=50)
    ap.add_argument("--capacity", type=int, default=160)
    ap.add_argument("--agents-per-wave", type=int, default=32)
    args = ap.parse_args()
    S, N, R, T, seed = args.scenarios, 2, 1, 96, 42
    inp = scenario_batch(S, N, T)
    ob = OracleBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                     env_time=inp.time[None], env_tout=inp.t_out, q_dtype="f64")
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    gids = np.arange(S * N).reshape(S, N)
    A = S * N
    lru = [collections.OrderedDict() for _ in range(A)]
    hits = misses = 0
    prev_bin = [dict() for _ in range(A)]  # time bin -> set of rows touched there last episode
    bin_hits = bin_total = 0
    bin_sizes = []
    step_all_hit = []  # [episode][T, A] every gathered row of the agent-step in the bulk-loaded set
    distinct_per_bin = []
    distinct_per_episode = []
    per_episode = []
    t0 = time.time()
    for e in range(args.episodes):
        eps = epsilon_at(e)
        out = ob.run_episode("train", rng="philox", seed=seed, episode=e, eps=eps, agent_ids=gids)
        rows, itb = rows_of_episode(ob, inp, out, seed, e, eps, gids)
        ta, tm = philox.t0_draws(seed, e + 1, gids.ravel(), sigma=0.3)  # agent.reset() (heating.py:145-152)
        ob.t_in, ob.t_m = ta.reshape(S, N).astype(F32), tm.reshape(S, N).astype(F32)
        eh = em = 0
        allhit = np.ones((T, A), bool)
        for a in range(A):
            c = lru[a]
            cur_bin = collections.defaultdict(set)
            ra, ia = rows[:, :, a], itb[:, a]
            for t in range(T):
                b = int(ia[t])
                pb = prev_bin[a].get(b, set())
                for k in range(5):
                    r = int(ra[t, k])
                    if r < 0:
                        continue
                    if r in c:
                        c.move_to_end(r)
                        eh += 1
                    else:
                        em += 1
                        c[r] = None
                        if len(c) > args.capacity:
                            c.popitem(last=False)
                    if e > 0:
                        bin_total += 1
                        h = (r in pb) or (r in cur_bin[b])
                        bin_hits += h
                        allhit[t, a] &= h
                    cur_bin[b].add(r)
            distinct_per_bin.extend(len(v) for v in cur_bin.values())
            distinct_per_episode.append(len(set().union(*cur_bin.values())))
            if e > 0:
                bin_sizes.extend(len(prev_bin[a].get(b, ())) for b in cur_bin)
            prev_bin[a] = dict(cur_bin)
        hits += eh
        misses += em
        if e > 0:
            step_all_hit.append(allhit)
        per_episode.append({"episode": e, "epsilon": eps, "lru_hit_rate": eh / max(1, eh + em)})
        print(f"episode {e} eps {eps:.3f} lru hit {eh / max(1, eh + em):.3f} ({time.time() - t0:.0f} s)",
              file=sys.stderr, flush=True)

    def q(x):
        x = np.asarray(x)
        return {"mean": float(x.mean()), "p50": float(np.percentile(x, 50)), "p90": float(np.percentile(x, 90)),
                "max": int(x.max())}

    late = [p["lru_hit_rate"] for p in per_episode[len(per_episode) // 2:]]
    ah = np.stack(step_all_hit)  # [E-1, T, A]
    wave = ah.reshape(ah.shape[0], T, A // args.agents_per_wave, args.agents_per_wave).all(axis=-1)
    print(json.dumps({
        "workload": f"configs[1] bench workload sample: {S} scenarios x N={N} (R={R}, T={T}), per-agent f64 tables, "
                    f"Philox exploration, epsilon schedule of community.py:279-286, T0 reset per episode; "
                    f"oracle/restatement.py, {args.episodes} training episodes",
        "rows_gathered_per_agent_step": "round-0 row (greedy round 0 only) + 3 round-1 candidates + next-state row",
        "gathers": hits + misses,
        "distinct_rows_per_agent_per_time_bin_per_episode": q(distinct_per_bin),
        "distinct_rows_per_agent_per_episode": q(distinct_per_episode),
        "lru_capacity_rows": args.capacity,
        "lru_hit_rate_all": hits / max(1, hits + misses),
        "lru_hit_rate_second_half": float(np.mean(late)),
        "next_bin_bulk_load": {"hit_rate": bin_hits / max(1, bin_total),
                               "rows_loaded_per_agent_per_bin": q(bin_sizes) if bin_sizes else None,
                               "agent_steps_all_rows_hit": float(ah.mean()),
                               "wave_steps_all_rows_hit": float(wave.mean()),
                               "agents_per_wave": args.agents_per_wave,
                               "note": "rows of the same time bin in the previous episode, loaded ahead; "
                                       "rows missed once in the current bin count as hits afterwards.  A wave "
                                       "waits for its slowest lane's rows (one vmcnt per wave): only wave-steps "
                                       "whose every row hits leave the HBM round trip off the chain"},
        "per_episode": per_episode,
        "seconds": time.time() - t0}, indent=1))


if __name__ == "__main__":
    main()
