"""Learners (mirrors microgrid/rl.py:36-132 for the tabular actor).

``QActor`` keeps the reference's constructor, attributes and methods.  Its table lives in HBM:
inside a ``CommunityMicrogrid`` it is the agent's slot of the community's device tables
(the episode kernel reads and updates it); a standalone actor owns a private one-agent device
context.  ``q_table`` / ``set_qtable`` copy to / from the reference layout
(n_time, n_temp, n_balance, n_p2p, n_actions) float64, and ``load_from_file`` /
``save_to_file`` read / write the reference's ``.npy`` checkpoints (rl.py:83-87).
Per-call ``select_action`` / ``greedy_action`` / ``train`` run on the device (p2pmg_q_calls);
the exploration draws use the global np.random exactly as rl.py:101-111 does.
"""
from __future__ import annotations

import os
from abc import ABC, abstractmethod
from typing import Optional, Tuple

import numpy as np

from . import setup

MODELS_DIR = os.environ.get("P2PMG_MODELS_DIR", "..")  # the reference uses ../models_{implementation}/


def _as_obs(state) -> np.ndarray:
    x = state.numpy() if hasattr(state, "numpy") else state
    return np.asarray(x, dtype=np.float32).reshape(-1, 4)


class ActorInterface(ABC):
    @abstractmethod
    def __call__(self, state, *args, **kwargs): ...

    @abstractmethod
    def select_action(self, state): ...

    @abstractmethod
    def greedy_action(self, state): ...

    @abstractmethod
    def load_from_file(self, setting: str, implementation: str) -> None: ...

    @abstractmethod
    def save_to_file(self, setting: str, implementation: str) -> None: ...

    @abstractmethod
    def decay_exploration(self) -> None: ...


class QActor(ActorInterface):

    def __init__(self, num_time_states: int, num_temperature_states: int, num_balance_states: int,
                 num_p2p_states: int, num_actions: int = 3, gamma: float = 0.9,
                 alpha: float = 1e-5, epsilon: float = 1, decay: float = 0.9) -> None:
        self._time_states = num_time_states
        self._temp_states = num_temperature_states
        self._balance_states = num_balance_states
        self._p2p_states = num_p2p_states
        self._num_actions = num_actions
        self._epsilon = epsilon
        self._decay = decay
        self._gamma = gamma
        self._alpha = alpha
        self._shape = (num_time_states, num_temperature_states, num_balance_states, num_p2p_states, num_actions)
        self._host_table: Optional[np.ndarray] = None  # pending table while unbound (None = zeros)
        self._engine = None
        self._slot = 0

    # ------------------------------------------------------------ device binding
    def bind(self, engine, slot: int) -> None:
        """Attach to agent ``slot`` of a DeviceCommunityBatch (uploads any pending table)."""
        if (engine.cfg.alpha, engine.cfg.gamma) != (self._alpha, self._gamma):
            raise ValueError("QActor alpha/gamma differ from the device context's")
        if engine.q_shape != self._shape:
            raise ValueError(f"QActor table shape {self._shape} != device {engine.q_shape}")
        table = self._host_table if self._engine is None else self.q_table
        self._engine, self._slot = engine, slot
        self._host_table = None
        if table is not None:
            engine.set_q(np.asarray(table)[None], first=slot)

    def _device(self):
        if self._engine is None:
            from .engine import DeviceCommunityBatch
            nt, nT, nb, np_, na = self._shape
            eng = DeviceCommunityBatch(1, 1, 0, 1, q_dtype=setup.q_dtype, device=setup.device,
                                       alpha=self._alpha, gamma=self._gamma, n_time_states=nt,
                                       n_temp_states=nT, n_balance_states=nb, n_p2p_states=np_)
            self.bind(eng, 0)
        return self._engine, self._slot

    # ------------------------------------------------------------ table access (rl.py:76-87)
    @property
    def q_table(self) -> np.ndarray:
        if self._engine is None:
            return np.zeros(self._shape) if self._host_table is None else self._host_table
        return self._engine.get_q(first=self._slot, count=1)[0]

    def set_qtable(self, q_table: np.ndarray) -> None:
        q_table = np.asarray(q_table)
        if q_table.shape != self._shape:
            raise ValueError(f"q_table shape {q_table.shape} != {self._shape}")
        if self._engine is None:
            self._host_table = np.array(q_table, dtype=np.float64)
        else:
            self._engine.set_q(q_table[None], first=self._slot)

    def load_from_file(self, setting: str, implementation: str) -> None:
        self.set_qtable(np.load(os.path.join(MODELS_DIR, f"models_{implementation}", f"{setting}.npy")))

    def save_to_file(self, setting: str, implementation: str) -> None:
        d = os.path.join(MODELS_DIR, f"models_{implementation}")
        os.makedirs(d, exist_ok=True)
        np.save(os.path.join(d, f"{setting}.npy"), self.q_table)

    # ------------------------------------------------------------ per-call API (rl.py:89-132)
    def _get_state_indices(self, state) -> Tuple[int, int, int, int]:
        eng, _ = self._device()
        idx = eng.state_indices(_as_obs(state)[:1])[0]
        return int(idx[0]), int(idx[1]), int(idx[2]), int(idx[3])

    def __call__(self, state, *args, **kwargs):
        return self.select_action(state)

    def select_action(self, state) -> Tuple[int, float]:
        if np.random.rand() < self._epsilon:
            return self.random_action()
        return self.greedy_action(state)

    def random_action(self) -> Tuple[int, float]:
        return np.random.choice(self._num_actions), 0.

    def greedy_action(self, state) -> Tuple[int, float]:
        eng, slot = self._device()
        acts, qv = eng.q_calls([slot], _as_obs(state)[:1], [255])
        return int(acts[0]), float(qv[0])

    def train(self, state, action: int, reward, next_state) -> None:
        eng, slot = self._device()
        r = reward.numpy() if hasattr(reward, "numpy") else reward
        eng.q_calls([slot], _as_obs(state)[:1], [int(action)], rewards=np.asarray(r, np.float32).ravel()[:1],
                    ns_obs=_as_obs(next_state)[:1], train=True)

    def decay_exploration(self) -> None:
        self._epsilon = max(0.1, self._decay * self._epsilon)
