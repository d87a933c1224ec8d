"""Exploration streams.

Replay mode reproduces the reference's use of the global legacy ``np.random`` (MT19937)
exactly, in its consumption order:

  get_community (community.py:210-211): normal(0.7,0.2,N) load ratings, normal(4,0.2,N) PV ratings
  HPHeating.__init__ (heating.py:101-104): per agent T_m first, then T_in  ~ N(setpoint, 0.3)
  train_episode: per (t, round, agent): rand(); if < eps: choice(3)   (rl.py:101-111)
  agent.reset at episode end (heating.py:149-152): per agent T_in first, then T_m

The per-decision draws are decoded natively (``p2pmg_replay_decode``) from a block of raw
32-bit MT words; the RandomState is then advanced by exactly the words consumed, so the
stream continues bit-identically for the normals that follow.

Philox mode (counter-keyed on seed, episode, global agent, t, round) is generated on the
device; nothing is drawn on the host.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib


def global_random_state() -> np.random.RandomState:
    """The RandomState behind ``np.random.*`` (what the reference's module-level seeds set)."""
    return np.random.mtrand._rand


class ReferenceRNG:
    """The reference's exploration/initialisation stream over one legacy RandomState."""

    def __init__(self, rs: Optional[np.random.RandomState] = None):
        self.rs = rs if rs is not None else global_random_state()

    # -- get_community + HPHeating.__init__
    def community_ratings(self, n_agents: int, homogeneous: bool):
        if homogeneous:
            return np.array([0.7] * n_agents), np.array([4] * n_agents)
        return self.rs.normal(0.7, 0.2, n_agents), self.rs.normal(4, 0.2, n_agents)

    def initial_temperature(self, setpoint: float, homogeneous: bool):
        """One HPHeating.__init__: returns (t_in, t_m) after drawing T_m first, then T_in."""
        if homogeneous:
            return np.float32(setpoint), np.float32(setpoint)
        t_m = np.float32(self.rs.normal(setpoint, 0.3, 1)[0])
        t_in = np.float32(self.rs.normal(setpoint, 0.3, 1)[0])
        return t_in, t_m

    def reset_temperature(self, setpoint: float, homogeneous: bool):
        """One HPHeating.reset: returns (t_in, t_m) drawing T_in first, then T_m."""
        if homogeneous:
            return np.float32(setpoint), np.float32(setpoint)
        t_in = np.float32(self.rs.normal(setpoint, 0.3, 1)[0])
        t_m = np.float32(self.rs.normal(setpoint, 0.3, 1)[0])
        return t_in, t_m

    # -- train_episode exploration
    def episode_codes(self, T: int, R: int, N: int, eps: Sequence[float]) -> np.ndarray:
        """uint8 codes [T, R+1, N]: 255 = greedy, else the explored action."""
        n_dec = T * (R + 1) * N
        eps = np.ascontiguousarray(np.broadcast_to(np.asarray(eps, dtype=np.float64), (N,)))
        codes = np.empty(n_dec, dtype=np.uint8)
        st = self.rs.get_state()
        k = int(n_dec * (2 + 1.5 * float(eps.max(initial=0.0)))) + 256
        L = _lib.lib()
        while True:
            self.rs.set_state(st)
            words = np.ascontiguousarray(self.rs.randint(0, 2 ** 32, size=k, dtype=np.uint32))
            used = C.c_size_t(0)
            status = L.p2pmg_replay_decode(words.ctypes.data, words.size, n_dec, eps.ctypes.data, N,
                                           codes.ctypes.data, C.byref(used))
            if status == _lib.P2PMG_OK:
                break
            k *= 2
        self.rs.set_state(st)
        if used.value:
            self.rs.randint(0, 2 ** 32, size=used.value, dtype=np.uint32)
        return codes.reshape(T, R + 1, N)


def python_random():
    """The module-level ``random`` generator the reference seeds in rl.py:25 and draws from in
    ActorModel.select_action (rl.py:175) and ReplayBuffer.sample_batch (rl.py:238)."""
    import random
    return random._inst


def dqn_episode_draws(py_rng, np_rs: np.random.RandomState, T: int, R: int, N: int, eps: Sequence[float],
                      counts: Optional[Sequence[int]] = None, capacity: int = 5000, batch: int = 32):
    """One DQN community episode's draws in the reference's consumption order:
    per (t, round, agent): ``random.random() < eps`` then, exploring, ``np.random.choice([0, 1, 2])``
    (rl.py:175-186); then per agent, after its transition was stored, ``random.sample(buffer, 32)``
    (rl.py:238, only when ``counts`` - buffer sizes before the episode - is given).
    Returns (codes uint8 [T, R+1, N], samples uint16 [T, N, 32] or None)."""
    eps = np.broadcast_to(np.asarray(eps, np.float64), (N,))
    codes = np.full((T, R + 1, N), _lib.GREEDY, np.uint8)
    samples = None if counts is None else np.zeros((T, N, batch), np.uint16)
    cnt = None if counts is None else [int(c) for c in counts]
    for t in range(T):
        for r in range(R + 1):
            for i in range(N):
                if py_rng.random() < eps[i]:
                    codes[t, r, i] = np_rs.choice([0, 1, 2])
        if samples is not None:
            for i in range(N):
                cnt[i] = min(cnt[i] + 1, capacity)
                samples[t, i] = py_rng.sample(range(cnt[i]), min(cnt[i], batch))
    return codes, samples
