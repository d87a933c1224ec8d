"""Philox4x32-10 counter-based RNG in NumPy — TEST INFRASTRUCTURE ONLY.

This module is part of ``oracle/``: it is the checker for the device-side Philox
exploration stream, never imported by the product (``p2pmicrogrid_amd``).

The reference draws exploration from the global legacy ``np.random`` MT19937 stream
(``microgrid/rl.py:101-111``); that order is reproduced by replay mode
(``oracle/restatement.py``).  Philox mode is the build-defined, counter-keyed stream of
SURVEY.md §3.5 (ii): one Philox block per (seed, episode, agent, t, round, tag), so the
result is independent of how scenarios are sharded over GPUs.

Block layout (must match ``p2pmicrogrid_amd/csrc/p2pmg_device.h::philox_step_codes``): one 32-bit
word per negotiation round, so one block serves four rounds (two agent-steps at R = 1):
    key  = (seed_lo, seed_hi)
    k    = t * (R + 1) + r
    ctr  = (k // 4, episode, agent_global, TAG_DECISION)
    w    = x[k % 4]
    u    = w / 2**32                                           (exact in f64)
    explore <=> u < epsilon   (f64 compare, as rl.py:101)
    act  = w % 3   when thr = ceil(epsilon * 2**32) >= 2**24 (used only when exploring: given
                   u < epsilon, w is uniform on [0, thr), so w % 3 is uniform up to 1 / thr <= 2**-24);
           v % 3   when thr < 2**24 (small epsilon: w itself is below thr, so w % 3 would be biased),
                   v = word k % 4 of the block ctr = (k // 4, episode, agent_global, TAG_ACTION),
                   independent of the explore test (rl.py:110-111 draws the action separately)
T0 draws at an episode start (tag TAG_T0, ctr = (0, episode, agent, TAG_T0)):
    Box-Muller in f64 on u1 = (x0 + 0.5) / 2**32, u2 = (x1 + 0.5) / 2**32;
    T_in = f32(setpoint + 0.3 * z0), T_m = f32(setpoint + 0.3 * z1)   (heating.py:149-152)
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

TAG_DECISION = 0x5EED0004  # one word per round, four rounds per block (0x5EED0003: two rounds per block)
TAG_T0 = 0x5EED0002
TAG_ACTION = 0x5EED0005    # small epsilon: the explore actions' own block
SMALL_EPS_THR = 1 << 24


def eps_threshold(eps: float):
    """(thr, all): w / 2**32 < eps  <=>  all or w < thr (p2pmg_internal.h::eps_threshold)."""
    c = np.ceil(float(eps) * 4294967296.0)
    if not c > 0.0:
        c = 0.0
    all_ = c >= 4294967296.0
    return (0xFFFFFFFF if all_ else int(c)), bool(all_)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Random123 definition). All args uint32-valued arrays."""
    c0 = np.asarray(c0, dtype=np.uint64) & MASK32
    c1 = np.asarray(c1, dtype=np.uint64) & MASK32
    c2 = np.asarray(c2, dtype=np.uint64) & MASK32
    c3 = np.asarray(c3, dtype=np.uint64) & MASK32
    k0 = np.asarray(k0, dtype=np.uint64) & MASK32
    k1 = np.asarray(k1, dtype=np.uint64) & MASK32
    c0, c1, c2, c3, k0, k1 = np.broadcast_arrays(c0, c1, c2, c3, k0, k1)
    c0, c1, c2, c3, k0, k1 = (x.copy() for x in (c0, c1, c2, c3, k0, k1))
    for rnd in range(10):
        if rnd > 0:
            k0 = (k0 + W0) & MASK32
            k1 = (k1 + W1) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
    return c0, c1, c2, c3


def launch_eps(eps_arr) -> float:
    """The one epsilon of a Philox-mode launch (the device takes a single threshold per launch)."""
    e = np.asarray(eps_arr, dtype=np.float64)
    if not np.all(e == e.flat[0]):
        raise ValueError("Philox mode draws with one epsilon per launch")
    return float(e.flat[0])


def decision_draws(seed: int, episode: int, agents, t: int, r: int, rounds: int, eps=None):
    """(u f64, action int) for each agent id in ``agents`` at (episode, t, r); ``rounds`` = R.
    eps (the launch's epsilon, one value): below 2**-8 (thr < 2**24) the action comes from the
    TAG_ACTION block; None = the large-epsilon layout (action = w % 3)."""
    agents = np.asarray(agents, dtype=np.uint64)
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    k = t * (rounds + 1) + r
    x = philox4x32_10(k // 4, episode, agents, TAG_DECISION, k0, k1)
    w = x[k % 4]
    u = w.astype(np.float64) / 4294967296.0
    aw = w
    if eps is not None:
        thr, all_ = eps_threshold(eps)
        if not all_ and thr < SMALL_EPS_THR:
            aw = philox4x32_10(k // 4, episode, agents, TAG_ACTION, k0, k1)[k % 4]
    act = (aw % np.uint64(3)).astype(np.int64)
    return u, act


def t0_draws(seed: int, episode: int, agents, setpoint: float = 21.0, sigma: float = 0.3):
    """(T_in f32, T_m f32) initial temperatures for an episode start in Philox mode."""
    agents = np.asarray(agents, dtype=np.uint64)
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    x0, x1, _, _ = philox4x32_10(0, episode, agents, TAG_T0, k0, k1)
    u1 = (x0.astype(np.float64) + 0.5) / 4294967296.0
    u2 = (x1.astype(np.float64) + 0.5) / 4294967296.0
    rad = np.sqrt(-2.0 * np.log(u1))
    ang = 6.283185307179586 * u2
    z0 = rad * np.cos(ang)
    z1 = rad * np.sin(ang)
    return (setpoint + sigma * z0).astype(np.float32), (setpoint + sigma * z1).astype(np.float32)


TAG_SAMPLE = 0x5EED0100  # + j, j < 32: replay-buffer sample draws (DQN)


def sample_draws(seed: int, episode: int, agents, t: int, count, k: int = 32):
    """Build-defined replay-buffer sampling in Philox mode (DQN, rl.py:226-241 semantics:
    k distinct indices of [0, count), 0 = oldest).  Floyd's algorithm: for j = 0..k-1,
    m = count - k + j, r = (x0_j * (m + 1)) >> 32 with x0_j the first word of the Philox block
    ctr = (t, episode, agent, TAG_SAMPLE + j); take r unless already taken, else m.
    Returns int64 [len(agents), k] in draw order."""
    agents = np.asarray(agents, dtype=np.uint64).ravel()
    count = np.broadcast_to(np.asarray(count, dtype=np.int64), agents.shape)
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    out = np.zeros((len(agents), k), dtype=np.int64)
    for j in range(k):
        x0, _, _, _ = philox4x32_10(t, episode, agents, TAG_SAMPLE + j, k0, k1)
        m = count - k + j
        r = ((x0 * (m + 1).astype(np.uint64)) >> np.uint64(32)).astype(np.int64)
        taken = (out[:, :j] == r[:, None]).any(axis=1) if j else np.zeros(len(agents), bool)
        out[:, j] = np.where(taken, m, r)
    return out
