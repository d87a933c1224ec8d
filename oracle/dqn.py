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


# ----------------------------------------------------------------------------- device order
# The same arithmetic in the summation order of the HIP kernels (p2pmg_dqn.hip), so the device
# can be held to it bit for bit.  The f32 MFMA is exactly a k-ordered fmaf chain (MI355X guide,
# FP32-input MFMA numerics), DPP / permlane sums are the pairwise trees spelled out below, and
# every other op rounds on its own (-ffp-contract=off).  forward()/gradients() above (NumPy
# matmul order) stay as the independent second check, within the north_star tolerance.

def fmaf(a, b, c):
    """float32 fused multiply-add with ONE rounding: a * b is exact in float64 (24 + 24 bits);
    the float64 sum is taken with round-to-odd (TwoSum error folded into the last bit), which
    rounds correctly to float32 afterwards (53 >= 24 + 2 bits)."""
    a, b, c = (np.asarray(x, F32) for x in (a, b, c))
    p = a.astype(np.float64) * b.astype(np.float64)
    cc = c.astype(np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        sm = p + cc
        bb = sm - p
        err = (p - (sm - bb)) + (cc - bb)
        odd = np.frombuffer(np.ascontiguousarray(sm, np.float64).tobytes(), np.int64).reshape(sm.shape) & 1
        fix = (err != 0) & (odd == 0) & np.isfinite(sm)
        sm = np.where(fix, np.nextafter(sm, np.where(err > 0, np.inf, -np.inf)), sm)
    return sm.astype(F32)


def tree_sum(v, axis=-1):
    """Pairwise tree of adjacent elements (v0 + v1) + (v2 + v3) ... over a power-of-two axis: the
    DPP quad_perm / row_half_mirror / row_mirror + permlane16 / permlane32 swap sums (x + swap(x)
    adds the same two operands in both lanes)."""
    v = np.moveaxis(np.asarray(v, F32), axis, -1)
    while v.shape[-1] > 1:
        v = (v[..., 0::2] + v[..., 1::2]).astype(F32)
    return v[..., 0]


def relu32(x):
    x = np.asarray(x, F32)
    return np.where(x > 0, x, F32(0)).astype(F32)


def act_q(theta, obs):
    """Greedy Q values of dqn_act_kernel / dqn_act_shared_kernel (ActorModel.greedy_action
    rl.py:188-196): layer 1 as p2p * W1[3], then fmaf with bal, tnorm, time (features 3, 2, 1, 0),
    the action term added per action value; layer 2 as an fmaf chain over k = 0..63 from +0;
    layer 3 as the pairwise tree over the 64 units (wave_sum), then + b3.
    theta [4609]; obs [..., 4] -> q [..., 3]."""
    p = unpack(theta)
    obs = np.asarray(obs, F32)
    W1, b1, W2, b2, w3, b3 = p["W1"], p["b1"], p["W2"], p["b2"], p["W3"][:, 0], p["b3"][0]
    o = obs[..., None, :]
    z = (o[..., 3] * W1[3]).astype(F32)
    z = fmaf(o[..., 2], W1[2], z)
    z = fmaf(o[..., 1], W1[1], z)
    z = fmaf(o[..., 0], W1[0], z)
    hs = [relu32(z + b1), relu32(fmaf(F32(0.5), W1[4], z) + b1), relu32((z + W1[4]).astype(F32) + b1)]
    out = []
    for h in hs:
        acc = np.zeros(h.shape, F32)
        for k in range(H):
            acc = fmaf(h[..., k:k + 1], W2[k], acc)
        out.append(tree_sum((relu32(acc + b2) * w3).astype(F32)) + b3)
    return np.stack(out, -1).astype(F32)


def api_forward(theta, x):
    """dqn_forward_kernel (QNetwork.call on explicit rows, rl.py:147-148): layer 1 as an fmaf
    chain over the 5 inputs, layer 2 over k = 0..63, layer 3 as an fmaf chain over the units,
    + b3.  theta [4609]; x [..., 5] -> q [...]."""
    p = unpack(theta)
    x = np.asarray(x, F32)
    z = np.zeros(x.shape[:-1] + (H,), F32)
    for k in range(N_IN):
        z = fmaf(x[..., k:k + 1], p["W1"][k], z)
    h1 = relu32(z + p["b1"])
    acc = np.zeros(h1.shape, F32)
    for k in range(H):
        acc = fmaf(h1[..., k:k + 1], p["W2"][k], acc)
    h2 = relu32(acc + p["b2"])
    out = np.zeros(x.shape[:-1], F32)
    for j in range(H):
        out = fmaf(h2[..., j], p["W3"][j, 0], out)
    return (out + p["b3"][0]).astype(F32)


def _chain_k(h, W2):
    """fmaf chain over k = 0..63 from +0: h [..., rows, 64] x W2 [..., 64, 64] (rows of W2 = k)."""
    acc = np.zeros(h.shape[:-1] + (W2.shape[-1],), F32)
    for k in range(W2.shape[-2]):
        acc = fmaf(h[..., k:k + 1], W2[..., None, k, :], acc)
    return acc


def _train_layer23(h1, W2, b2, w3):
    """dqn_train_kernel layers 2-3 of one network: Z2^T = W2^T H1^T on MFMA (fmaf chain over
    k = 0..63), ReLU, then each wave's 16 units as the pairwise tree (in-lane pairs, reduce4_groups)
    and the 4 waves added in wave order (qpart), + b3 by the caller.  Returns (z2 pre-ReLU, q sum).
    h1 [..., 32, 64]; W2 [..., 64, 64]; b2, w3 [..., 64]."""
    pre = (_chain_k(h1, W2) + b2[..., None, :]).astype(F32)
    v = (relu32(pre) * w3[..., None, :]).astype(F32)
    q = tree_sum(v[..., 0:16])
    for w in range(1, 4):
        q = (q + tree_sum(v[..., 16 * w:16 * w + 16])).astype(F32)
    return pre, q


def train_block(theta, target, batches, gamma: float, counts=None):
    """dqn_train_kernel workgroups (Trainer._train rl.py:307-333 up to the optimizer), in the
    kernel's order, for nb blocks at once.  theta / target [4609] (a shared network) or [nb, 4609]
    (one network per block); batches [nb, n_ag, 32, 10] (s[4], a, r, ns[4]) or [n_ag, 32, 10] (one
    block); counts [nb]: agents of each block (default n_ag; a shorter block's trailing slots are
    ignored).  The gradient accumulators run ACROSS a block's agents as the kernel's registers do:
    dW2 as the MFMA chain over (agent, q = 0..7, b = 8 k + q); dW1 / db1 per row group g4 over
    (agent, r, rt) rows b = 16 rt + 4 g4 + r, then the 4 groups pairwise; dW3 / db2 per data-row
    lane c over (agent, rt) rows b = 16 rt + c, then the 16 lanes pairwise; db3 per agent pairwise
    over the lanes of dq[c] + dq[16 + c], chained over agents.
    Returns (gradient partials [nb, 4609] f32 (W1 not clipped), loss [nb, n_ag]); without a block
    axis in `batches`, ([4609], [n_ag])."""
    bt = np.asarray(batches, F32)
    single = bt.ndim == 3
    if single:
        bt = bt[None]
    nb, n_ag = bt.shape[0], bt.shape[1]
    cnt = np.full(nb, n_ag) if counts is None else np.asarray(counts)
    P, T = unpack(theta), unpack(target)
    if np.ndim(theta) == 1:  # one shared network: a block axis of length 1 broadcasts
        P = {k: v[None] for k, v in P.items()}
        T = {k: v[None] for k, v in T.items()}
    gW2 = np.zeros((nb, H, H), F32)
    gx1 = np.zeros((nb, 4, N_IN, H), F32)      # [block][row group g4][input k][unit]
    gb1 = np.zeros((nb, 4, H), F32)
    gW3 = np.zeros((nb, 16, H), F32)           # [block][lane c][unit]
    gb2 = np.zeros((nb, 16, H), F32)
    gb3 = np.zeros(nb, F32)
    losses = np.zeros((nb, n_ag), F32)
    b3t, b3o = T["b3"][:, 0], P["b3"][:, 0]
    rows_g = [[16 * rt + 4 * np.arange(4) + rr for rt in range(2)] for rr in range(4)]
    for ag in range(n_ag):
        on = (ag < cnt)                          # blocks that still have an agent at this slot
        x = bt[:, ag]                            # [nb, 32, 10]
        s5, r, ns = x[..., 0:5], x[..., 5], x[..., 6:10]
        # target network on (ns, a') for the 3 action values
        z = np.zeros((nb, 32, H), F32)
        for k in range(4):
            z = fmaf(ns[..., k:k + 1], T["W1"][:, None, k, :], z)
        qt = []
        for av in ACTION_VALUES:
            h1t = relu32(fmaf(av, T["W1"][:, None, 4, :], z) + T["b1"][:, None, :])
            _, qs = _train_layer23(h1t, T["W2"], T["b2"], T["W3"][..., 0])
            qt.append((qs + b3t[:, None]).astype(F32))
        # online network on (s, a): features 0..3 then the action input (second MFMA)
        z = np.zeros((nb, 32, H), F32)
        for k in range(N_IN):
            z = fmaf(s5[..., k:k + 1], P["W1"][:, None, k, :], z)
        pre1 = (z + P["b1"][:, None, :]).astype(F32)
        h1 = relu32(pre1)
        pre2, qs = _train_layer23(h1, P["W2"], P["b2"], P["W3"][..., 0])
        h2 = relu32(pre2)
        q = (qs + b3o[:, None]).astype(F32)
        y = (r + F32(gamma) * np.maximum(np.maximum(qt[0], qt[1]), qt[2])).astype(F32)
        diff = (q - y).astype(F32)
        dq = (F32(2.0 / 32) * diff).astype(F32)                       # [nb, 32]
        sq = (diff * diff).astype(F32)
        losses[:, ag] = tree_sum((sq[:, 0:16] + sq[:, 16:32]).astype(F32)) / F32(32)
        gb3 = np.where(on, (gb3 + tree_sum((dq[:, 0:16] + dq[:, 16:32]).astype(F32))).astype(F32), gb3)
        # backward: dZ2, dW3, db2 (lane c holds rows c and 16 + c)
        w3o = P["W3"][..., 0][:, None, :]
        dz2 = np.where(pre2 > 0, (dq[..., None] * w3o).astype(F32), F32(0)).astype(F32)
        prod3 = (h2 * dq[..., None]).astype(F32)
        m = on[:, None, None]
        for rt in range(2):
            gW3 = np.where(m, (gW3 + prod3[:, 16 * rt:16 * rt + 16]).astype(F32), gW3)
            gb2 = np.where(m, (gb2 + dz2[:, 16 * rt:16 * rt + 16]).astype(F32), gb2)
        # dW2 = H1^T dZ2, MFMA K order b = 8 k + q
        for qq in range(8):
            for k in range(4):
                b = 8 * k + qq
                gW2 = np.where(m, fmaf(h1[:, b, :, None], dz2[:, b, None, :], gW2), gW2)
        # dH1 = dZ2 W2^T, K order j = 16 g + kk; dZ1 = dH1 [pre1 > 0]
        dh1 = np.zeros((nb, 32, H), F32)
        for kk in range(16):
            for g in range(4):
                j = 16 * g + kk
                dh1 = fmaf(dz2[..., j:j + 1], P["W2"][:, None, :, j], dh1)
        dz1 = np.where(pre1 > 0, dh1, F32(0)).astype(F32)
        m4 = on[:, None, None, None]
        for rr in range(4):
            for rt in range(2):
                rows = rows_g[rr][rt]                                   # one row per group g4
                gb1 = np.where(m, (gb1 + dz1[:, rows]).astype(F32), gb1)
                for k in range(N_IN):
                    gx1[:, :, k] = np.where(m4[..., 0], fmaf(s5[:, rows, k][..., None], dz1[:, rows], gx1[:, :, k]),
                                            gx1[:, :, k])
    g1 = ((gx1[:, 0] + gx1[:, 1]).astype(F32) + (gx1[:, 2] + gx1[:, 3]).astype(F32)).astype(F32)
    gb1s = ((gb1[:, 0] + gb1[:, 1]).astype(F32) + (gb1[:, 2] + gb1[:, 3]).astype(F32)).astype(F32)
    g = np.concatenate([g1.reshape(nb, -1), gb1s, gW2.reshape(nb, -1), tree_sum(gb2, axis=1),
                        tree_sum(gW3, axis=1), gb3[:, None]], axis=1).astype(F32)
    if single:
        return g[0], losses[0]
    return g, losses


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
    # "device": the HIP kernels' summation order (act_q, train_block: bit-exact target);
    # "matmul": NumPy matmul order (q_values, gradients: the independent second check)
    order: str = "device"

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

    def _train_device(self, b, dp):
        """The train launch(es) of one env step in the kernels' order: shared network = one
        train_block per workgroup (block_layout), then the segment reduction + Adam; per-agent
        networks = one train_block per agent with its own Adam step."""
        A = b.shape[0]
        if self.shared:
            _, apb, bps, blocks = block_layout(A, self.grad_segments, self.agents_per_block)
            bb = np.zeros((len(blocks), apb) + b.shape[1:], F32)
            for k, (a0, n) in enumerate(blocks):
                bb[k, :n] = b[a0:a0 + n]
            counts = np.array([n for _, n in blocks])
            partials, lb = train_block(self.theta[0], self.target[0], bb, dp.gamma, counts)
            ls = np.concatenate([lb[k, :n] for k, (_, n) in enumerate(blocks)])
            adam_step(self.theta, self.m, self.v, self._reduce_partials(partials, bps)[None], self.step, dp)
            return ls
        gr, ls = train_block(self.theta, self.target, b[:, None], dp.gamma)
        adam_step(self.theta, self.m, self.v, gr, self.step, dp)
        return ls[:, 0]

    def _reduce_partials(self, partials, bps):
        """fold_segments -> (exchange over ranks) -> sum_segments -> mean over all agents."""
        segs = fold_segments(partials, bps)
        A_local = self.S * self.N
        if self.world > 1:
            rows = np.zeros((self.world, segs.size), F32)
            rows[self.rank] = segs.ravel()
            self.exchange(rows)
            segs = rows.reshape(-1, N_PARAMS)
        return sum_segments(segs) * (F32(1) / F32(A_local * self.world))

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
        return self._reduce_partials(partials, bps)

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
                if self.order == "device":
                    if self.shared:
                        q = act_q(self.theta[0], obs.reshape(A, 4)).reshape(S, N, 3)
                    else:
                        q = np.stack([act_q(th[k], obs.reshape(A, 4)[k]) for k in range(A)]).reshape(S, N, 3)
                elif self.shared:
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
                    u, ra = philox.decision_draws(seed, episode, gids.ravel(), t, r, R, eps=philox.launch_eps(eps_arr))
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
                if self.order == "device":
                    ls = self._train_device(b, dp)
                elif self.shared:
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
