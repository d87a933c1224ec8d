"""CPU restatement of the DQN variant (config 5) — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The product (``p2pmicrogrid_amd``) never imports ``oracle/``.

Restates, in float32 NumPy (paths relative to /root/reference/microgrid):

    QNetwork                         rl.py:135-148   concat(state[4], action[1]) -> 64 ReLU -> 64 ReLU -> 1
    ActorModel.select_action         rl.py:174-183   explore if u < epsilon: action values (0, .5, 1)
    ActorModel.greedy_action         rl.py:188-196   argmax over the 3 action values (first max)
    ReplayBuffer.add/sample_batch    rl.py:200-248   deque(maxlen=5000), random.sample of 32
    Trainer._train                   rl.py:307-333   y = r + gamma * max_a' Q_target(ns, a');
                                                     loss = mean((y - Q(s, a))^2); clip grad[0]
                                                     (first kernel) to [-1, 1]; Adam(lr=1e-5)
    Trainer._soft_update             rl.py:335-359   target <- (1 - tau) target + tau online
    DQNAgent                         agent.py:301-350 buffer 5000, batch 32, gamma .95, tau .005
    CommunityMicrogrid.train_episode community.py:149-182 (agent.train after every step)
    CommunityMicrogrid.init_buffers  community.py:125-147 (5 episodes of memory, no training)

Parameter layout (Keras ``trainable_weights`` order, packed):
    W1 [5][64] | b1 [64] | W2 [64][64] | b2 [64] | W3 [64][1] | b3 [1]   = 4609 floats.

Parity: TensorFlow is absent, so the Keras initialisation, TF's Adam kernel and TF's matmul
summation order cannot be reproduced or run: initial weights are an INPUT shared by the
oracle and the device, Adam follows the published Keras form (below), and device results are
compared within a float32 tolerance (1e-5 relative on Q values / weights, north_star),
actions exactly.  Parity with the reference itself: unpinned (no TF fixtures exist).

Adam (Keras ``Adam`` / TF ``ResourceApplyAdam``, beta1 .9, beta2 .999, epsilon 1e-7):
    lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)            (host, float64 -> float32)
    m += (g - m) * (1 - beta1);  v += (g*g - v) * (1 - beta2)
    w -= (m * lr_t) / (sqrt(v) + epsilon)
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

import numpy as np

from . import philox
from .restatement import (GREEDY, OracleParams, assign_powers, compute_costs, divide_power, prices, reward,
                          seq_sum, temperature_step)

F32 = np.float32
H = 64
N_IN = 5
N_PARAMS = N_IN * H + H + H * H + H + H + 1  # 4609
ACTION_VALUES = np.array([0.0, 0.5, 1.0], dtype=F32)  # rl.py:153
OFF = {"W1": 0, "b1": 320, "W2": 384, "b2": 4480, "W3": 4544, "b3": 4608}


@dataclass
class DQNParams:
    gamma: float = 0.95    # agent.py:309
    tau: float = 0.005     # agent.py:309
    lr: float = 1e-5       # agent.py:310
    beta1: float = 0.9     # Keras Adam defaults
    beta2: float = 0.999
    adam_eps: float = 1e-7
    batch: int = 32        # agent.py:308
    capacity: int = 5000   # agent.py:308
    clip: float = 1.0      # rl.py:329


def unpack(theta):
    """theta [..., 4609] -> dict of views (Keras shapes)."""
    t = np.asarray(theta, dtype=F32)
    lead = t.shape[:-1]
    return {"W1": t[..., 0:320].reshape(*lead, N_IN, H), "b1": t[..., 320:384],
            "W2": t[..., 384:4480].reshape(*lead, H, H), "b2": t[..., 4480:4544],
            "W3": t[..., 4544:4608].reshape(*lead, H, 1), "b3": t[..., 4608:4609]}


def glorot_init(n_nets: int, seed: int = 0) -> np.ndarray:
    """Keras Dense defaults in distribution (glorot_uniform kernels, zero biases), from a NumPy
    seed: the build's initial weights (TF's own init stream is not reproducible)."""
    rs = np.random.RandomState(seed)
    th = np.zeros((n_nets, N_PARAMS), dtype=F32)
    for name, (fi, fo) in (("W1", (N_IN, H)), ("W2", (H, H)), ("W3", (H, 1))):
        lim = np.sqrt(6.0 / (fi + fo))
        o = OFF[name]
        th[:, o:o + fi * fo] = rs.uniform(-lim, lim, size=(n_nets, fi * fo)).astype(F32)
    return th


def forward(theta, x):
    """QNetwork.call (rl.py:147-148).  theta [n, 4609] (or [4609]); x [n, B, 5] (or [B, 5]).
    Returns q [.., B] and the cache for backward."""
    p = unpack(theta)
    x = np.asarray(x, dtype=F32)
    z1 = np.matmul(x, p["W1"]) + p["b1"][..., None, :]
    h1 = np.maximum(z1, F32(0))
    z2 = np.matmul(h1, p["W2"]) + p["b2"][..., None, :]
    h2 = np.maximum(z2, F32(0))
    q = (np.matmul(h2, p["W3"]) + p["b3"][..., None, :])[..., 0]
    return q.astype(F32), (x, z1, h1, z2, h2)


def q_values(theta, obs):
    """Q(obs, a) for the three action values: obs [n, M, 4] -> [n, M, 3] (rl.py:188-193)."""
    obs = np.asarray(obs, dtype=F32)
    M = obs.shape[-2]
    x = np.concatenate([np.repeat(obs[..., :, None, :], 3, axis=-2),
                        np.broadcast_to(ACTION_VALUES[:, None], obs.shape[:-1] + (3, 1))], axis=-1)
    q, _ = forward(theta, x.reshape(obs.shape[:-2] + (M * 3, N_IN)))
    return q.reshape(obs.shape[:-2] + (M, 3))


def gradients(theta, s, a, r, ns, target, gamma: float, clip: float = 1.0):
    """Trainer._train (rl.py:307-333) up to the optimizer: per-net gradient of
    mean_b (y_b - Q(s_b, a_b))^2 with y = r + gamma * max_a' Q_target(ns, a').
    s, ns [n, B, 4]; a, r [n, B].  Returns (grad [n, 4609], loss [n]) - grad[0] NOT clipped
    (the clip is applied to the gradient the optimizer receives, see adam_step)."""
    s = np.asarray(s, F32)
    B = s.shape[-2]
    qn = q_values(target, ns)                               # [n, B, 3]
    y = np.asarray(r, F32) + F32(gamma) * qn.max(axis=-1)   # [n, B]
    x = np.concatenate([s, np.asarray(a, F32)[..., None]], axis=-1)
    q, (x, z1, h1, z2, h2) = forward(theta, x)
    diff = q - y
    loss = (diff * diff).mean(axis=-1, dtype=F32)
    dq = (F32(2.0 / B) * diff).astype(F32)                  # d mean((y - q)^2) / dq
    p = unpack(theta)
    gW3 = np.matmul(np.swapaxes(h2, -1, -2), dq[..., None])  # [n, 64, 1]
    gb3 = dq.sum(axis=-1, dtype=F32)[..., None]
    dz2 = (dq[..., None] * np.swapaxes(p["W3"], -1, -2)) * (z2 > 0)
    gW2 = np.matmul(np.swapaxes(h1, -1, -2), dz2)
    gb2 = dz2.sum(axis=-2, dtype=F32)
    dz1 = np.matmul(dz2, np.swapaxes(p["W2"], -1, -2)) * (z1 > 0)
    gW1 = np.matmul(np.swapaxes(x, -1, -2), dz1)
    gb1 = dz1.sum(axis=-2, dtype=F32)
    n = s.shape[:-2]
    g = np.concatenate([gW1.reshape(*n, -1), gb1, gW2.reshape(*n, -1), gb2, gW3.reshape(*n, -1), gb3], axis=-1)
    return g.astype(F32), loss.astype(F32)


def adam_lr(step: int, dp: DQNParams = DQNParams()) -> np.float32:
    """lr * sqrt(1 - beta2^t) / (1 - beta1^t), t = step (1-based), in float64 -> float32."""
    t = np.asarray(step, np.float64)
    return (dp.lr * np.sqrt(1.0 - dp.beta2 ** t) / (1.0 - dp.beta1 ** t)).astype(F32)


def adam_step(theta, m, v, grad, step: int, dp: DQNParams = DQNParams()):
    """Clip the first kernel's gradient (rl.py:329) and apply one Adam update in place."""
    g = np.array(grad, dtype=F32, copy=True)
    g[..., 0:320] = np.clip(g[..., 0:320], F32(-dp.clip), F32(dp.clip))
    lr_t = adam_lr(step, dp)
    if np.ndim(lr_t):  # one Adam iteration count per network (rows of theta)
        lr_t = np.asarray(lr_t, F32)[:, None]
    m += (g - m) * (F32(1) - F32(dp.beta1))
    v += (g * g - v) * (F32(1) - F32(dp.beta2))
    theta -= (m * lr_t) / (np.sqrt(v) + F32(dp.adam_eps))


RED_SLICES = 16  # dqn_reduce_adam_kernel: 16 waves per parameter fold a segment's partials


def block_layout(n_agents: int, segments: int = 1, agents_per_block: int = 0):
    """The shared network's gradient layout (p2pmg_dqn_setup, include/p2pmg.h grad_segments): the
    agents split into `segments` contiguous segments, each into blocks of `agents_per_block` agents
    (0: one block per segment here; the device's automatic choice depends on its CU count).
    Returns (seg_agents, apb, bps, [(first agent, count)] per block in launch order)."""
    if n_agents % segments:
        raise ValueError("grad_segments must divide the agents (whole scenarios)")
    seg_agents = n_agents // segments
    apb = agents_per_block if agents_per_block > 0 else seg_agents
    bps = -(-seg_agents // apb)
    blocks = []
    for g in range(segments):
        for j in range(bps):
            a0 = g * seg_agents + j * apb
            blocks.append((a0, min(apb, (g + 1) * seg_agents - a0)))
    return seg_agents, apb, bps, blocks


def fold_segments(partials, bps: int):
    """dqn_reduce_adam_kernel's order for each segment (rows of `partials` [segments * bps, P]):
    16 slices of ceil(bps / 16) consecutive partials, each summed from +0.0 in partial order, then
    slice 0 + slice 1 + ... + slice 15.  Returns [segments, P] float32."""
    partials = np.asarray(partials, F32)
    n_seg = partials.shape[0] // bps
    per = -(-bps // RED_SLICES)
    out = np.zeros((n_seg, partials.shape[1]), F32)
    for g in range(n_seg):
        blk = partials[g * bps:(g + 1) * bps]
        parts = []
        for sl in range(RED_SLICES):
            acc = np.zeros(partials.shape[1], F32)
            for b in range(sl * per, min(bps, sl * per + per)):
                acc = acc + blk[b]
            parts.append(acc)
        t = parts[0]
        for r in range(1, RED_SLICES):
            t = t + parts[r]
        out[g] = t
    return out


def sum_segments(segs):
    """dqn_adam_shared_kernel: the segments of every rank summed in global segment order."""
    segs = np.asarray(segs, F32)
    t = segs[0].copy()
    for g in range(1, segs.shape[0]):
        t = t + segs[g]
    return t


def soft_update(target, theta, tau: float):
    """Trainer._soft_update (rl.py:335-354) with tau != 1: t <- (1 - tau) * t + tau * w."""
    target[...] = (F32(1) - F32(tau)) * target + F32(tau) * theta


def reference_dqn_replay(py_rng, np_rng, T: int, R: int, N: int, eps, counts=None, k: int = 32):
    """Draws of one DQN community episode in the reference's consumption order: per (t, round,
    agent) ``random.random() < eps`` (rl.py:175, Python's ``random``) then, when exploring,
    ``np.random.choice([0, 1, 2])`` (rl.py:186); then per agent ``random.sample(buffer, 32)``
    (rl.py:238, after the step's transition was added) when ``counts`` (buffer sizes before the
    episode) is given.  Returns (codes uint8 [T, R+1, N], samples int64 [T, N, k] or None)."""
    eps = np.broadcast_to(np.asarray(eps, np.float64), (N,))
    codes = np.full((T, R + 1, N), GREEDY, np.uint8)
    samples = None if counts is None else np.zeros((T, N, k), np.int64)
    cnt = None if counts is None else np.array(counts, np.int64)
    for t in range(T):
        for r in range(R + 1):
            for i in range(N):
                if py_rng.random() < eps[i]:
                    codes[t, r, i] = np_rng.choice([0, 1, 2])
        if samples is not None:
            for i in range(N):
                cnt[i] = min(cnt[i] + 1, 5000)
                n = int(cnt[i])
                samples[t, i] = py_rng.sample(range(n), min(n, k))
    return codes, samples


@dataclass
class OracleDQNBatch:
    """S scenarios x N DQN agents (per-agent networks, or ONE shared network when
    ``shared=True``: the per-agent batch gradients are averaged over every agent and one Adam
    step is taken per env step - the data-parallel config 5, build-defined)."""
    S: int
    N: int
    R: int
    load_w: np.ndarray
    pv_w: np.ndarray
    max_in: np.ndarray
    env_time: np.ndarray
    env_tout: np.ndarray
    theta0: np.ndarray                 # [n_nets, 4609] initial online weights (= target)
    shared: bool = False
    params: OracleParams = field(default_factory=OracleParams)
    dqn: DQNParams = field(default_factory=DQNParams)
    price_table: Optional[tuple] = None
    # shared network: the gradient layout (p2pmg_dqn_config) and, over several ranks, the host
    # all-gather of every rank's segments ([world, segments * P] rows, this rank's filled in)
    agents_per_block: int = 0
    grad_segments: int = 1
    rank: int = 0
    world: int = 1
    exchange: Optional[Callable] = None

    def __post_init__(self):
        self.T = self.load_w.shape[-1]
        S, N, T = self.S, self.N, self.T
        self.load_w = np.asarray(self.load_w, F32).reshape(S, N, T)
        self.pv_w = np.asarray(self.pv_w, F32).reshape(S, N, T)
        self.max_in = np.asarray(self.max_in, F32).reshape(S, N)
        self.env_time = np.asarray(self.env_time, F32).reshape(-1, T)
        self.env_tout = np.asarray(self.env_tout, F32).reshape(-1, T)
        n_nets = 1 if self.shared else S * N
        th = np.asarray(self.theta0, F32).reshape(-1, N_PARAMS)
        self.theta = np.ascontiguousarray(np.broadcast_to(th, (n_nets, N_PARAMS))).copy()
        self.target = self.theta.copy()
        self.m = np.zeros_like(self.theta)
        self.v = np.zeros_like(self.theta)
        self.step = 0              # Adam iterations: one count for all nets, or an [n_nets] array
        cap = self.dqn.capacity
        self.buf = np.zeros((S, N, cap, 10), F32)                # (s[4], a, r, ns[4]) per slot
        self.added = np.zeros((S, N), np.int64)
        p = self.params
        self.t_in = np.full((S, N), F32(p.setpoint), F32)
        self.t_m = np.full((S, N), F32(p.setpoint), F32)
        if self.price_table is None:
            self.buy, self.inj, self.p2p = prices(self.env_time, p)
        else:
            self.buy, self.inj, self.p2p = (np.asarray(x, F32).reshape(-1, T) for x in self.price_table)

    def _shared_gradient(self, gr):
        """Mean gradient of every agent of every rank in the device's summation structure: block
        partials (agents in order), each segment folded by fold_segments, every rank's segments
        gathered (exchange) and summed in global order, times 1 / (agents over all ranks)."""
        A = gr.shape[0]
        _, _, bps, blocks = block_layout(A, self.grad_segments, self.agents_per_block)
        partials = np.zeros((len(blocks), N_PARAMS), F32)
        for k, (a0, n) in enumerate(blocks):
            acc = np.zeros(N_PARAMS, F32)
            for a in range(a0, a0 + n):
                acc = acc + gr[a]
            partials[k] = acc
        segs = fold_segments(partials, bps)
        if self.world > 1:
            rows = np.zeros((self.world, segs.size), F32)
            rows[self.rank] = segs.ravel()
            self.exchange(rows)
            segs = rows.reshape(-1, N_PARAMS)
        return sum_segments(segs) * (F32(1) / F32(A * self.world))

    def _env(self, arr, t):
        return arr[:, t] if arr.shape[0] == self.S else np.broadcast_to(arr[0, t], (self.S,))

    def count(self):
        return np.minimum(self.added, self.dqn.capacity)

    def slots(self, idx):
        """deque index (0 = oldest) -> ring slot.  idx [S, N, k]."""
        cap = self.dqn.capacity
        first = (self.added - self.count())[..., None]
        return (first + idx) % cap

    def _nets(self, x):
        """Per-agent view of [n_nets, ...] arrays: [S, N, ...]."""
        if self.shared:
            return np.broadcast_to(x[0], (self.S, self.N) + x.shape[1:])
        return x.reshape((self.S, self.N) + x.shape[1:])

    def run_episode(self, mode: str = "train", codes=None, samples=None, rng: str = "replay", seed: int = 42,
                    episode: int = 0, eps=1.0, agent_ids=None) -> Dict:
        """mode 'train' (community.py:149-182 with DQNAgent.train), 'fill' (init_buffers,
        community.py:125-147: memory only) or 'greedy' (community.py:95-123).
        Replay: codes uint8 [T, R+1, S, N], samples [T, S, N, 32] deque indices."""
        p, dp = self.params, self.dqn
        S, N, R, T = self.S, self.N, self.R, self.T
        A = S * N
        gids = np.arange(A).reshape(S, N) if agent_ids is None else np.asarray(agent_ids).reshape(S, N)
        mi = self.max_in
        lv = p.hp_levels
        eps_arr = np.broadcast_to(np.asarray(eps, np.float64), (S, N))
        tr = {k: [] for k in ("action", "reward", "cost", "grid", "p2p", "t_in", "hp", "q", "loss")}
        for t in range(T):
            tn = (t + 1) % T
            time_t, tout, time_n = self._env(self.env_time, t), self._env(self.env_tout, t), self._env(self.env_time, tn)
            buy, inj, p2pp = self._env(self.buy, t), self._env(self.inj, t), self._env(self.p2p, t)
            bal = (self.load_w[:, :, t] - self.pv_w[:, :, t]) / mi        # agent.py:172-176
            baln = (self.load_w[:, :, tn] - self.pv_w[:, :, tn]) / mi
            tnorm = (self.t_in - F32(p.setpoint)) / F32(p.margin)         # heating.py:118-120
            P = np.zeros((S, N, N), F32)
            acts = np.zeros((R + 1, S, N), np.int64)
            qs = np.zeros((R + 1, S, N, 3), F32)
            obs = None
            for r in range(R + 1):
                d = np.arange(N)
                P[:, d, d] = F32(0)
                powers = -np.swapaxes(P, 1, 2)
                p2pf = (seq_sum(powers) / F32(N)) / mi                     # agent.py:203
                obs = np.stack([np.broadcast_to(time_t[:, None], (S, N)), tnorm, bal, p2pf], -1).astype(F32)
                th = self._nets(self.theta).reshape(A, N_PARAMS) if not self.shared else self.theta
                if self.shared:
                    q = q_values(self.theta[0], obs.reshape(A, 4)).reshape(S, N, 3)
                else:
                    q = q_values(th, obs.reshape(A, 1, 4)).reshape(S, N, 3)
                greedy = np.argmax(q, axis=-1)
                if mode == "greedy":
                    a = greedy
                elif rng == "replay":
                    c = codes[t, r]
                    a = np.where(c == GREEDY, greedy, c.astype(np.int64))
                else:
                    u, ra = philox.decision_draws(seed, episode, gids.ravel(), t, r, R)
                    a = np.where(u.reshape(S, N) < eps_arr, ra.reshape(S, N), greedy)
                hp = lv[a]
                out = (bal * mi) + hp                                      # agent.py:210
                P = divide_power(out, powers, N)
                acts[r] = a
                qs[r] = q
            g, pp = assign_powers(P)
            cost = compute_costs(g, pp, buy[:, None], inj[:, None], p2pp[:, None], p)
            rew = reward(cost, self.t_in, p)
            loss = np.zeros((S, N), F32)
            if mode in ("train", "fill"):
                # DQNAgent.save_memory agent.py:332-336: (s of the last round, its action value, r, ns)
                ns = np.stack([np.broadcast_to(time_n[:, None], (S, N)), tnorm, baln,
                               np.zeros((S, N), F32) / mi], -1).astype(F32)
                slot = self.added % dp.capacity
                rec = np.concatenate([obs, ACTION_VALUES[acts[R]][..., None], rew[..., None], ns], -1)
                self.buf[np.arange(S)[:, None], np.arange(N)[None, :], slot] = rec
                self.added += 1
            if mode == "train":
                cnt = self.count()
                if rng == "replay":
                    idx = np.asarray(samples[t], np.int64)
                else:
                    idx = philox.sample_draws(seed, episode, gids.ravel(), t, cnt.ravel(), dp.batch).reshape(S, N, -1)
                b = self.buf[np.arange(S)[:, None, None], np.arange(N)[None, :, None], self.slots(idx)]  # [S,N,k,10]
                b = b.reshape(A, -1, 10)
                self.step += 1
                if self.shared:
                    gr, ls = gradients(np.broadcast_to(self.theta[0], (A, N_PARAMS)), b[..., 0:4], b[..., 4],
                                       b[..., 5], b[..., 6:10], np.broadcast_to(self.target[0], (A, N_PARAMS)),
                                       dp.gamma, dp.clip)
                    adam_step(self.theta, self.m, self.v, self._shared_gradient(gr)[None], self.step, dp)
                else:
                    gr, ls = gradients(self.theta, b[..., 0:4], b[..., 4], b[..., 5], b[..., 6:10], self.target,
                                       dp.gamma, dp.clip)
                    adam_step(self.theta, self.m, self.v, gr, self.step, dp)
                soft_update(self.target, self.theta, dp.tau)               # Trainer.update_targets
                loss = ls.reshape(S, N)
            tr["action"].append(acts)
            tr["reward"].append(rew)
            tr["cost"].append(cost)
            tr["grid"].append(g)
            tr["p2p"].append(pp)
            tr["t_in"].append(self.t_in.copy())
            tr["hp"].append(hp)
            tr["q"].append(qs)
            tr["loss"].append(loss)
            self.t_in, self.t_m = temperature_step(tout[:, None], self.t_in, self.t_m, hp, p)
        out = {k: np.stack(v) for k, v in tr.items()}
        mean_t = seq_sum(out["reward"], axis=-1) / F32(N)
        out["episode_reward"] = seq_sum(mean_t, axis=0)
        return out
