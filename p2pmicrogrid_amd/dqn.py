"""DeviceDQNBatch — the DQN variant (BASELINE.json configs[4]) of the batched community.

S scenarios x N ``DQNAgent``s (agent.py:301-350) resident in HBM: per agent (or ONE shared
network, the data-parallel config 5) an online and a target ``QNetwork`` (rl.py:135-148,
5 -> 64 -> 64 -> 1 ReLU), Adam state and a replay ring of 5000 transitions (rl.py:200-248).
One ``run_episode`` call runs T environment steps on the device; each step is an act launch
(negotiation rounds with the Q-MLP, market, reward, memory append, RC update) followed in
TRAIN mode by the train launch (sample 32, target/online forward + backward on f32 MFMA,
clip, Adam, soft update; p2pmg_dqn.hip).

    mode 'fill'   CommunityMicrogrid.init_buffers (community.py:125-147): act + remember
    mode 'train'  CommunityMicrogrid.train_episode (community.py:149-182) with DQNAgent.train
    mode 'greedy' CommunityMicrogrid.run (community.py:95-123)

Weights use the Keras ``trainable_weights`` order packed into 4609 floats:
W1[5][64] | b1[64] | W2[64][64] | b2[64] | W3[64][1] | b3[1].
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .engine import DeviceCommunityBatch

F32 = np.float32
N_PARAMS = _lib.DQN_PARAMS
WHICH = {"online": _lib.DQN_ONLINE, "target": _lib.DQN_TARGET, "adam_m": _lib.DQN_ADAM_M, "adam_v": _lib.DQN_ADAM_V}
MODES = {"train": _lib.MODE_TRAIN, "greedy": _lib.MODE_GREEDY, "fill": _lib.MODE_FILL}
ACTION_VALUES = np.array([0.0, 0.5, 1.0], dtype=F32)  # ActorModel.actions rl.py:153


def glorot_init(n_nets: int, seed: int = 0) -> np.ndarray:
    """Keras Dense defaults in distribution (glorot_uniform kernels, zero biases) from a NumPy
    seed.  TF's own initialiser stream cannot be reproduced without TF."""
    rs = np.random.RandomState(seed)
    th = np.zeros((n_nets, N_PARAMS), dtype=F32)
    off = 0
    for fi, fo in ((5, 64), (64, 64), (64, 1)):
        lim = np.sqrt(6.0 / (fi + fo))
        th[:, off:off + fi * fo] = rs.uniform(-lim, lim, size=(n_nets, fi * fo)).astype(F32)
        off += fi * fo + fo
    return th


class DeviceDQNBatch(DeviceCommunityBatch):
    """Device-resident batch of S communities of DQN agents.  All compute runs in libp2pmg.so."""

    def __init__(self, n_scenarios: int, n_agents: int, rounds: int, horizon: int, shared: bool = False,
                 device: int = 0, seed: int = 42, scenario_offset: int = 0, gamma: float = 0.95, tau: float = 0.005,
                 lr: float = 1e-5, capacity: int = 5000, agents_per_block: int = 0, grad_segments: int = 1,
                 init_seed: Optional[int] = 0, **overrides):
        super().__init__(n_scenarios, n_agents, rounds, horizon, q_dtype="f32", device=device, seed=seed,
                         scenario_offset=scenario_offset, shared_q=shared, learner=_lib.LEARNER_DQN, **overrides)
        dc = _lib.DqnConfig()
        _lib.check(self.L.p2pmg_dqn_config_default(C.byref(dc)), what="dqn_config_default")
        dc.gamma, dc.tau, dc.lr, dc.capacity, dc.agents_per_block = gamma, tau, lr, capacity, agents_per_block
        dc.grad_segments = grad_segments
        self._chk(self.L.p2pmg_dqn_setup(self._ctx, C.byref(dc)), "dqn_setup")
        self.dcfg = dc
        self.shared = bool(shared)
        self.n_nets = 1 if shared else self.A
        self.capacity = capacity
        self._xfn = None          # the host exchange's ctypes callback (kept alive while installed)
        self._xerr = None
        if init_seed is not None:
            th = glorot_init(self.n_nets, init_seed)
            self.set_weights("online", th)
            self.set_weights("target", th)

    # ----------------------------------------------------------------- networks
    def set_weights(self, which: str, arr, first: int = 0):
        a = np.ascontiguousarray(np.asarray(arr, dtype=F32).reshape(-1, N_PARAMS))
        self._chk(self.L.p2pmg_dqn_set_weights(self._ctx, WHICH[which], first, a.shape[0], a.ctypes.data),
                  f"dqn_set_weights({which})")

    def get_weights(self, which: str, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        count = self.n_nets - first if count is None else count
        out = np.empty((count, N_PARAMS), F32)
        self._chk(self.L.p2pmg_dqn_get_weights(self._ctx, WHICH[which], first, count, out.ctypes.data),
                  f"dqn_get_weights({which})")
        return out

    def initialize_target(self):
        """Trainer.initialize_target (rl.py:274-278): target <- online (soft update with tau = 1)."""
        self.set_weights("target", self.get_weights("online"))

    @property
    def step(self) -> int:
        v = C.c_int64(0)
        self._chk(self.L.p2pmg_dqn_get_step(self._ctx, C.byref(v)), "dqn_get_step")
        return int(v.value)

    @step.setter
    def step(self, value: int):
        self._chk(self.L.p2pmg_dqn_set_step(self._ctx, int(value)), "dqn_set_step")

    def net_steps(self, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        """Adam iterations of each network (one optimizer per DQNAgent, agent.py:310)."""
        count = self.n_nets - first if count is None else count
        out = np.empty(count, np.int64)
        self._chk(self.L.p2pmg_dqn_get_net_steps(self._ctx, first, count, out.ctypes.data), "dqn_get_net_steps")
        return out

    # ----------------------------------------------------------------- multi-rank shared network
    def grad_layout(self) -> dict:
        """Shared network: gradient segments of this context, agents per train workgroup, train
        workgroups per env step (the summation structure the result depends on)."""
        g, a, b = C.c_int(0), C.c_int(0), C.c_int(0)
        self._chk(self.L.p2pmg_dqn_grad_layout(self._ctx, C.byref(g), C.byref(a), C.byref(b)), "dqn_grad_layout")
        return {"segments": g.value, "agents_per_block": a.value, "blocks": b.value}

    def set_grad_exchange(self, gather, rank: int, world: int):
        """Host exchange of the shared network's gradient segments (no RCCL communicator):
        ``gather(segs)`` gets the [world, floats_per_rank] f32 host array with this rank's row
        filled in and must fill the other rows (an all-gather, e.g. over gloo); called once per
        training env step from inside run_episode.  gather=None removes it."""
        if gather is None:
            self._chk(self.L.p2pmg_dqn_set_exchange(self._ctx, _lib.EXCHANGE_FN(), None, 0, 1), "dqn_set_exchange")
            self._xfn = None
            return

        def cb(_user, ptr, per, rk, nr):
            try:
                segs = np.ctypeslib.as_array(ptr, shape=(nr * per,)).reshape(nr, per)
                gather(segs)
                return 0
            except BaseException as e:  # noqa: BLE001  (re-raised by run_episode)
                self._xerr = e
                return 1

        fn = _lib.EXCHANGE_FN(cb)
        self._chk(self.L.p2pmg_dqn_set_exchange(self._ctx, fn, None, int(rank), int(world)), "dqn_set_exchange")
        self._xfn = fn

    # ----------------------------------------------------------------- replay memory
    def set_samples(self, samples):
        """Replay-mode sample indices: deque indices (0 = oldest) of random.sample(buffer, 32)
        (rl.py:238), [T, S, N, 32] or [T, A, 32]."""
        s = np.ascontiguousarray(np.asarray(samples).reshape(self.T, self.A, 32).astype(np.uint16))
        self._chk(self.L.p2pmg_dqn_set_samples(self._ctx, s.ctypes.data), "dqn_set_samples")

    def get_buffer(self, first: int = 0, count: Optional[int] = None):
        """(ring [count, capacity, 10] f32, added [count] int32) of agents [first, first + count)."""
        count = self.A - first if count is None else count
        buf = np.empty((count, self.capacity, 10), F32)
        added = np.empty(count, np.int32)
        self._chk(self.L.p2pmg_dqn_get_buffer(self._ctx, first, count, buf.ctypes.data, added.ctypes.data),
                  "dqn_get_buffer")
        return buf, added

    def set_buffer(self, buf, added, first: int = 0):
        b = np.ascontiguousarray(np.asarray(buf, F32).reshape(-1, self.capacity, 10))
        a = np.ascontiguousarray(np.asarray(added, np.int32).reshape(-1))
        self._chk(self.L.p2pmg_dqn_set_buffer(self._ctx, first, b.shape[0], b.ctypes.data, a.ctypes.data),
                  "dqn_set_buffer")

    # ----------------------------------------------------------------- the hot path
    def run_episode(self, mode: str = "train", rng: str = "philox", episode: int = 0, epsilon: float = 1.0,
                    record: Sequence[str] = (), philox: str = "auto"):
        """One episode of T steps for every scenario (asynchronous, stream-ordered)."""
        mask = 0
        for r in record:
            mask |= _lib.REC[r]
        args = _lib.EpisodeArgs(MODES[mode], _lib.RNG_REPLAY if rng == "replay" else _lib.RNG_PHILOX,
                                int(episode), mask, float(epsilon), 0, 0)
        self._xerr = None
        st = self.L.p2pmg_run_episode(self._ctx, C.byref(args))
        if st != _lib.P2PMG_OK and self._xerr is not None:
            raise _lib.P2PMGError(f"run_episode: the gradient exchange raised {self._xerr!r}") from self._xerr
        self._chk(st, "run_episode")
        self._recorded = mask

    # ----------------------------------------------------------------- object-API primitives
    def forward(self, x, net: int = 0) -> np.ndarray:
        """QNetwork.call (rl.py:147-148) on rows x = concat(state, action) [n, 5]."""
        x = np.ascontiguousarray(np.asarray(x, F32).reshape(-1, 5))
        q = np.empty(x.shape[0], F32)
        self._chk(self.L.p2pmg_dqn_forward(self._ctx, net, x.shape[0], x.ctypes.data, q.ctypes.data), "dqn_forward")
        return q

    def q_values(self, obs, net: int = 0) -> np.ndarray:
        """Q(obs, a) for the three action values (ActorModel.greedy_action rl.py:188-193): [n, 3]."""
        obs = np.asarray(obs, F32).reshape(-1, 4)
        x = np.concatenate([np.repeat(obs, 3, axis=0), np.tile(ACTION_VALUES, len(obs))[:, None]], axis=1)
        return self.forward(x, net).reshape(-1, 3)

    def train_batch(self, s, a, r, ns, net: int = 0) -> float:
        """Trainer._train + update_targets (rl.py:307-359) on one batch of 32 transitions."""
        b = np.concatenate([np.asarray(s, F32).reshape(32, 4), np.asarray(a, F32).reshape(32, 1),
                            np.asarray(r, F32).reshape(32, 1), np.asarray(ns, F32).reshape(32, 4)], axis=1)
        b = np.ascontiguousarray(b)
        loss = C.c_float(0)
        self._chk(self.L.p2pmg_dqn_train_batch(self._ctx, net, b.ctypes.data, C.byref(loss)), "dqn_train_batch")
        return float(loss.value)
