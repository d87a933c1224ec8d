"""Replay the configs[1] Q-row trace (scripts/trace_rows.py) through per-agent row caches.

Every agent's table is private (one writer: the agent itself), so a per-agent software cache of
its rows in LDS would be coherent by construction.  What decides whether it pays is the wave:
all lanes of a gather wait for the slowest, so a wave-step avoids the MALL/HBM round trip only
when EVERY lane's rows hit.  For cache capacities C (rows per agent) this prints the per-access
hit rate and the fraction of wave-steps with all lanes hitting, for waves of k agents
(consecutive agents, as the kernel packs scenarios), under LRU (an upper bound) and a 4-way
set-associative cache (what an LDS table would implement).  Accesses per step: the round-0 row,
then the round-1 row (the TD update writes the final round's row, already present).  The first
episode warms the caches and is not counted.

    python scripts/row_cache_sim.py rows.npz > profiles/r06_row_cache_sim.json"""
import json
import sys
from collections import OrderedDict

import numpy as np


def simulate(seq, cap, ways):
    """seq [n_access] row ids of one agent -> hit flags.  ways = 0: fully associative LRU."""
    hits = np.zeros(seq.size, bool)
    if ways == 0:
        c = OrderedDict()
        for i, r in enumerate(seq.tolist()):
            if r in c:
                hits[i] = True
                c.move_to_end(r)
            else:
                c[r] = None
                if len(c) > cap:
                    c.popitem(last=False)
        return hits
    sets = max(1, cap // ways)
    c = [OrderedDict() for _ in range(sets)]
    for i, r in enumerate(seq.tolist()):
        s = c[(r * 2654435761 >> 7) % sets]
        if r in s:
            hits[i] = True
            s.move_to_end(r)
        else:
            s[r] = None
            if len(s) > ways:
                s.popitem(last=False)
    return hits


def main(path):
    z = np.load(path)
    idx = z["index"]  # [E][T][R1][A]
    E, T, R1, A = idx.shape
    seq = idx.transpose(3, 0, 1, 2).reshape(A, -1)  # per agent, in access order
    per_ep = T * R1
    out = {"trace": path, "episodes": int(E), "agents": int(A), "warmup_episodes_before_trace": int(z["warmup"]),
           "distinct_rows_per_agent_per_episode": float(np.mean([len(np.unique(seq[a, e * per_ep:(e + 1) * per_ep]))
                                                                 for a in range(0, A, 7) for e in range(E)])),
           "results": []}
    for ways in (0, 4):
        for cap in (64, 128, 160, 256, 512):
            h = np.stack([simulate(seq[a], cap, ways) for a in range(A)])[:, per_ep:]  # drop the warm-up episode
            step = h.reshape(A, -1, R1).all(axis=2)  # [A][steps]: both rounds' rows hit
            res = {"ways": ways or "lru", "rows_per_agent": cap, "kb_per_agent_f64": cap * 32 / 1024,
                   "access_hit": float(h.mean()), "agent_step_hit": float(step.mean())}
            for k in (2, 8, 16, 32, 64):
                g = step[:A - A % k].reshape(-1, k, step.shape[1]).all(axis=1)
                res[f"wave_step_all_hit_k{k}"] = float(g.mean())
            out["results"].append(res)
            print(json.dumps(res), file=sys.stderr, flush=True)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
