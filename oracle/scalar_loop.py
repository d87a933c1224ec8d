"""Reference-shaped per-object CPU loop of the hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg import this module: it is the checker's
second form and the "per-object eager-style" CPU baseline of SURVEY.md §8(d).  The product
(``p2pmicrogrid_amd``) never imports anything under ``oracle/``.

``oracle/restatement.py`` vectorises the path over scenarios; this module keeps the reference's
object structure and loop nesting instead: one object per agent with its own (20,20,20,20,3)
float64 table, and ``train_episode`` walks t -> round -> agent with scalar float32 arithmetic,
as ``CommunityMicrogrid.train_episode`` (community.py:149-182) does with eager TF ops:

    CommunityMicrogrid._run            community.py:67-93    ScalarCommunity._negotiate
    RLAgent.__call__ / _get_balance    agent.py:172-213      ScalarQAgent.__call__
    RLAgent._divide_power              agent.py:186-195      ScalarQAgent._divide_power
    QActor.select_action / greedy      rl.py:89-117          ScalarQAgent._act
    CommunityMicrogrid._assign_powers  community.py:45-54    ScalarCommunity._assign_powers
    CommunityMicrogrid._compute_costs  community.py:56-65    ScalarCommunity._costs
    RLAgent.get_reward                 agent.py:225-232      ScalarQAgent.get_reward
    QAgent.train -> QActor.train       agent.py:293-298, rl.py:119-129   ScalarQAgent.train
    HPHeating.step                     heating.py:37-56,138-143          ScalarQAgent.step

Exploration is either replayed (codes [T, R+1, N], 255 = greedy) or drawn from a
``np.random.RandomState`` in the reference's consumption order (per t, round, agent:
``rand() < eps`` then ``choice(3)``, rl.py:100-111).  tests/test_cpu_scalar_loop.py pins it to
the reference-driven fixtures (tests/golden/loop_*.npz) bit for bit.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .restatement import GREEDY, OracleParams, prices, state_index, temperature_step

F32 = np.float32


def _sgn(x) -> F32:
    """tf.math.sign on a float32 scalar (sign of +-0 is 0)."""
    return F32(int(x > 0) - int(x < 0))


class ScalarQAgent:
    """QAgent (agent.py:255-298) on RLAgent (agent.py:156-252): one agent, its own QActor table."""

    def __init__(self, load_w, pv_w, max_in, t_in, t_m, p: OracleParams = OracleParams()):
        self.p = p
        self.load_w = np.asarray(load_w, F32)
        self.pv_w = np.asarray(pv_w, F32)
        self.max_in = F32(max_in)
        self.t_in, self.t_m = F32(t_in), F32(t_m)
        self.q = np.zeros((p.n_time, p.n_temp, p.n_bal, p.n_p2p, p.n_actions))
        self.levels = p.hp_levels
        self.hp = F32(0)

    def _indices(self, time, tnorm, bal, p2p):
        """QActor._get_state_indices rl.py:89-95."""
        p = self.p
        return (int(state_index(time, p.n_time, "time")), int(state_index(tnorm, p.n_temp, "temp")),
                int(state_index(bal, p.n_bal, "plain")), int(state_index(p2p, p.n_p2p, "plain")))

    def _tnorm(self) -> F32:
        return F32(F32(self.t_in - F32(self.p.setpoint)) / F32(self.p.margin))  # heating.py:118-120

    def _act(self, s, code: int) -> int:
        """QActor.select_action / greedy_action rl.py:100-117 (first max on ties)."""
        if code != GREEDY:
            return int(code)
        return int(self.q[s].argmax())

    def _divide_power(self, out: F32, powers) -> list:
        """RLAgent._divide_power agent.py:186-195."""
        n = len(powers)
        so = _sgn(out)
        filt = [powers[j] if so != _sgn(powers[j]) else F32(0) for j in range(n)]
        tot = F32(0)
        for j in range(n):
            tot = F32(tot + filt[j])
        tot = F32(abs(tot))
        if tot == F32(0):
            return [F32(F32(out * F32(1)) / F32(n))] * n
        return [F32(F32(out * F32(abs(filt[j]))) / tot) for j in range(n)]

    def __call__(self, t: int, time: F32, powers, code: int):
        """RLAgent.__call__ agent.py:200-213: observation, action, the agent's row of P."""
        n = len(powers)
        acc = F32(0)
        for j in range(n):
            acc = F32(acc + powers[j])
        p2p = F32(F32(acc / F32(n)) / self.max_in)
        bal = F32(F32(self.load_w[t] - self.pv_w[t]) / self.max_in)
        s = self._indices(time, self._tnorm(), bal, p2p)
        a = self._act(s, code)
        self.hp = self.levels[a]
        out = F32(F32(bal * self.max_in) + self.hp)
        return self._divide_power(out, powers), a, s

    def get_reward(self, cost: F32) -> F32:
        """RLAgent.get_reward agent.py:225-232 (pre-update T_in)."""
        p, t = self.p, self.t_in
        pen = max(max(F32(0), F32(F32(p.lower) - t)), max(F32(0), F32(t - F32(p.upper))))
        pen = F32(pen + F32(1)) if pen > 0 else F32(0)
        return F32(-F32(cost + F32(F32(p.penalty_weight) * pen)))

    def train(self, s, a: int, r: F32, tn: int, time_n: F32) -> None:
        """QAgent.train agent.py:293-298 -> QActor.train rl.py:119-129: next state = next slot,
        same T_in, p2p = 0; the TD arithmetic in float64."""
        p = self.p
        baln = F32(F32(self.load_w[tn] - self.pv_w[tn]) / self.max_in)
        ns = self._indices(time_n, self._tnorm(), baln, F32(F32(0) / self.max_in))
        qmax = self.q[ns].max()
        sa = s + (a,)
        self.q[sa] = self.q[sa] + p.alpha * ((float(r) + p.gamma * qmax) - self.q[sa])

    def step(self, t_out: F32) -> None:
        """HPHeating.step heating.py:138-143 -> temperature_simulation heating.py:37-56."""
        a, b = temperature_step(t_out, self.t_in, self.t_m, self.hp, self.p)
        self.t_in, self.t_m = F32(a), F32(b)


class ScalarCommunity:
    """CommunityMicrogrid (community.py:35-188) over ScalarQAgents, one scenario."""

    def __init__(self, agents, time, t_out, R: int, price_table=None, p: OracleParams = OracleParams()):
        self.agents, self.R, self.p = list(agents), int(R), p
        self.time = np.asarray(time, F32)
        self.t_out = np.asarray(t_out, F32)
        self.T = len(self.time)
        self.buy, self.inj, self.p2pp = price_table if price_table is not None else prices(self.time, p)

    def _assign_powers(self, P):
        """community.py:45-54 on the final P (diagonal kept): opposite signs exchange the min."""
        n = len(self.agents)
        g, pp = [F32(0)] * n, [F32(0)] * n
        for i in range(n):
            ag, ap = F32(0), F32(0)
            for j in range(n):
                pij, pji = P[i][j], P[j][i]
                e = F32(_sgn(pij) * min(abs(pij), abs(pji))) if _sgn(pij) != _sgn(pji) else F32(0)
                ag = F32(ag + F32(pij - e))
                ap = F32(ap + e)
            g[i], pp[i] = ag, ap
        return g, pp

    def _costs(self, t: int, g: F32, pp: F32) -> F32:
        """community.py:56-65."""
        p = self.p
        c = F32(g * self.buy[t]) if g >= 0 else F32(g * self.inj[t])
        c = F32(c + F32(pp * self.p2pp[t]))
        return F32(F32(F32(c * F32(p.time_slot)) / F32(p.minutes_per_hour)) * F32(1e-3))

    def _negotiate(self, t: int, codes_t):
        """community.py:67-93: R + 1 Jacobi rounds; each round every agent sees -P[:, i]."""
        n = len(self.agents)
        P = [[F32(0)] * n for _ in range(n)]
        acts, states = [0] * n, [None] * n
        rec_a = np.zeros((self.R + 1, n), np.int64)
        rec_s = np.zeros((self.R + 1, n, 4), np.int64)
        for r in range(self.R + 1):
            for i in range(n):
                P[i][i] = F32(0)
            rows = []
            for i, ag in enumerate(self.agents):
                powers = [F32(-P[j][i]) for j in range(n)]
                row, a, s = ag(t, self.time[t], powers, int(codes_t[r][i]))
                rows.append(row)
                acts[i], states[i] = a, s
                rec_a[r, i], rec_s[r, i] = a, s
            P = rows
        return P, acts, states, rec_a, rec_s

    def train_episode(self, codes: Optional[np.ndarray] = None, rs: Optional[np.random.RandomState] = None,
                      eps: float = 0.0, training: bool = True) -> Dict[str, np.ndarray]:
        """community.py:149-182 (training=False: CommunityMicrogrid.run, community.py:95-123).
        codes: [T, R+1, N] replay codes, or None to draw them from ``rs`` as the reference does."""
        n, T, R = len(self.agents), self.T, self.R
        out = {k: np.zeros((T, n), F32) for k in ("grid", "p2p", "cost", "reward", "t_in", "t_m", "hp")}
        out["action"] = np.zeros((T, R + 1, n), np.int64)
        out["idx"] = np.zeros((T, R + 1, n, 4), np.int64)
        ep = F32(0)
        for t in range(T):
            if not training:
                ct = np.full((R + 1, n), GREEDY, np.uint8)
            elif codes is not None:
                ct = codes[t]
            else:
                ct = np.full((R + 1, n), GREEDY, np.uint8)
                for r in range(R + 1):
                    for i in range(n):
                        if rs.rand() < eps:
                            ct[r, i] = rs.choice(3)
            P, acts, states, out["action"][t], out["idx"][t] = self._negotiate(t, ct)
            g, pp = self._assign_powers(P)
            rewards = []
            for i, ag in enumerate(self.agents):
                cost = self._costs(t, g[i], pp[i])
                rw = ag.get_reward(cost)
                out["grid"][t, i], out["p2p"][t, i], out["cost"][t, i], out["reward"][t, i] = g[i], pp[i], cost, rw
                out["t_in"][t, i], out["t_m"][t, i], out["hp"][t, i] = ag.t_in, ag.t_m, ag.hp
                rewards.append(rw)
            if training:
                tn = (t + 1) % T
                for i, ag in enumerate(self.agents):
                    ag.train(states[i], acts[i], rewards[i], tn, self.time[tn])
            m = F32(0)
            for rw in rewards:
                m = F32(m + rw)
            ep = F32(ep + F32(m / F32(n)))
            for ag in self.agents:  # CommunityMicrogrid._step community.py:184-188
                ag.step(self.t_out[t])
        out["episode_reward"] = ep
        return out
