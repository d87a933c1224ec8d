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


# ============================================================================ DQN (rl.py:135-359)
import collections  # noqa: E402
import random  # noqa: E402
from dataclasses import dataclass  # noqa: E402

random.seed(setup.seed)  # rl.py:25 seeds Python's random for select_action / sample_batch

_KERAS_SHAPES = (("kernel", (5, 64)), ("bias", (64,)), ("kernel", (64, 64)), ("bias", (64,)),
                 ("kernel", (64, 1)), ("bias", (1,)))
_N_PARAMS = 4609
_net_counter = [0]


@dataclass
class Adam:
    """Stand-in for ``tf.optimizers.Adam`` (agent.py:310): its hyper-parameters, applied on the
    device in the Keras form (oracle/dqn.py documents the update)."""
    learning_rate: float = 1e-3
    beta_1: float = 0.9
    beta_2: float = 0.999
    epsilon: float = 1e-7


def _flat(weights) -> np.ndarray:
    return np.concatenate([np.asarray(w, np.float32).ravel() for w in weights]).astype(np.float32)


def _unflat(theta) -> list:
    out, o = [], 0
    for _, shp in _KERAS_SHAPES:
        n = int(np.prod(shp))
        out.append(np.asarray(theta[o:o + n], np.float32).reshape(shp))
        o += n
    return out


class QNetwork:
    """rl.py:135-148: concat(state[4], action[1]) -> Dense(64, relu) -> Dense(64, relu) -> Dense(1).

    Weights live in a device context slot (``bind``); until then on the host.  Keras creates
    its weights lazily with glorot_uniform from TF's seed; this build draws the same
    distribution from a private NumPy stream (the global np.random is not consumed)."""

    def __init__(self):
        _net_counter[0] += 1
        from .dqn import glorot_init
        self._host = glorot_init(1, seed=setup.seed * 1000 + _net_counter[0])[0]
        self._engine, self._which, self._slot = None, "online", 0

    def bind(self, engine, which: str, slot: int) -> None:
        th = self.flat_weights()
        self._engine, self._which, self._slot = engine, which, slot
        engine.set_weights(which, th[None], first=slot)

    def unbind(self) -> None:
        self._host = self.flat_weights()
        self._engine = None

    def flat_weights(self) -> np.ndarray:
        if self._engine is None:
            return self._host.copy()
        return self._engine.get_weights(self._which, first=self._slot, count=1)[0]

    def set_flat_weights(self, theta) -> None:
        theta = np.asarray(theta, np.float32).reshape(_N_PARAMS)
        if self._engine is None:
            self._host = theta.copy()
        else:
            self._engine.set_weights(self._which, theta[None], first=self._slot)

    @property
    def trainable_weights(self) -> list:
        return _unflat(self.flat_weights())

    def get_weights(self) -> list:
        return self.trainable_weights

    def set_weights(self, weights) -> None:
        self.set_flat_weights(_flat(weights))

    def _device(self):
        if self._engine is None or self._which != "online":
            from .dqn import DeviceDQNBatch
            eng = DeviceDQNBatch(1, 1, 0, 1, device=setup.device, init_seed=None)
            eng.set_weights("online", self.flat_weights()[None])
            return eng, 0, True
        return self._engine, self._slot, False

    def __call__(self, state, action) -> np.ndarray:
        s = np.asarray(state.numpy() if hasattr(state, "numpy") else state, np.float32).reshape(-1, 4)
        a = np.asarray(action.numpy() if hasattr(action, "numpy") else action, np.float32).reshape(-1, 1)
        eng, slot, tmp = self._device()
        try:
            return eng.forward(np.concatenate([s, a], axis=1), slot)[:, None]
        finally:
            if tmp:
                eng.close()

    def save_weights(self, path: str) -> None:
        """Keras ``save_weights`` replacement: an .npz of the six arrays in Keras order."""
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        np.savez(path if path.endswith(".npz") else path + ".npz",
                 **{f"w{k}": w for k, w in enumerate(self.trainable_weights)})

    def load_weights(self, path: str) -> None:
        with np.load(path if path.endswith(".npz") else path + ".npz", allow_pickle=False) as f:
            self.set_weights([f[f"w{k}"] for k in range(6)])


class ActorModel(ActorInterface):
    """rl.py:151-197: epsilon-greedy over the action values (0, .5, 1) with a Q-network."""

    def __init__(self, epsilon: float = 0.1):
        self.actions = np.array([0., 0.5, 1.], dtype=np.float32)
        self._epsilon = epsilon
        self._decay = 0.9
        self._q_network = QNetwork()

    @property
    def q_network(self) -> QNetwork:
        return self._q_network

    def load_from_file(self, setting: str, implementation: str) -> None:
        self._q_network.load_weights(os.path.join(MODELS_DIR, f"models_{implementation}", setting))

    def save_to_file(self, setting: str, implementation: str) -> None:
        self._q_network.save_weights(os.path.join(MODELS_DIR, f"models_{implementation}", setting))

    def __call__(self, state, *args, **kwargs):
        return self.select_action(state)

    def select_action(self, state):
        if random.random() < self._epsilon:
            return self.random_action()
        return self.greedy_action(state)

    def random_action(self):
        return np.expand_dims(self.actions[np.random.choice([0, 1, 2])], axis=0), np.array([0.], np.float32)

    def greedy_action(self, state):
        s = np.asarray(state.numpy() if hasattr(state, "numpy") else state, np.float32).reshape(1, 4)
        q = self._q_network(np.repeat(s, 3, axis=0), self.actions[:, None])   # (3, 1)
        return np.expand_dims(self.actions[int(np.argmax(q[:, 0]))], axis=0), q

    def decay_exploration(self) -> None:
        self._epsilon *= self._decay  # no floor for the DQN actor (rl.py:196-197)


class ReplayBuffer:
    """rl.py:200-248.  Host deque for standalone use; inside a community the memory is the
    device ring of the agent (``bind``) and sampling reads it back."""

    def __init__(self, buffer_size: int, batch_size: int):
        self.buffer_size = buffer_size
        self.batch_size = batch_size
        self.count = 0
        self.buffer = collections.deque(maxlen=buffer_size)
        self._engine, self._slot = None, 0

    def bind(self, engine, slot: int) -> None:
        self._engine, self._slot = engine, slot

    def _device_rows(self):
        ring, added = self._engine.get_buffer(self._slot, 1)
        n = int(added[0])
        cnt = min(n, self.buffer_size)
        order = (n - cnt + np.arange(cnt)) % self.buffer_size
        return ring[0][order]

    def add(self, s, a, r, ns) -> None:
        if self._engine is not None:
            raise RuntimeError("this agent's memory is device-resident (filled by the community kernels)")
        self.count = min(self.count + 1, self.buffer_size)
        self.buffer.append((s, a, r, ns))

    def add_batch(self, s, a, r, ns) -> None:
        for i in range(np.shape(s)[0]):
            self.add(s[i, :], a[i], r[i], ns[i, :])

    def size(self) -> int:
        if self._engine is not None:
            return len(self._device_rows())
        return min(self.count, self.buffer_size)

    def sample_batch(self):
        if self._engine is not None:
            rows = self._device_rows()
            idx = random.sample(range(len(rows)), min(len(rows), self.batch_size))
            b = rows[idx]
            return b[:, 0:4], b[:, 4:5], b[:, 5:6], b[:, 6:10]
        batch = random.sample(self.buffer, min(self.count, self.batch_size))
        return tuple(np.stack([np.asarray(x[k], np.float32) for x in batch]) for k in range(4))

    def clear(self):
        self.buffer.clear()
        self.count = 0


class Trainer:
    """rl.py:251-359: TD targets from a target network, MSE loss, first-kernel gradient clip,
    Adam, soft target update - one device launch per ``train`` (p2pmg_dqn_train_batch)."""

    def __init__(self, actor: ActorModel, buffer_size: int, batch_size: int, gamma: float, tau: float,
                 optimizer: Adam):
        self._batch_size = batch_size
        self._gamma = gamma
        self._tau = tau
        self.actor = actor
        self.target_network = ActorModel().q_network
        self.optimizer = optimizer
        self.buffer = ReplayBuffer(buffer_size, batch_size)
        self._engine, self._slot = None, 0

    def bind(self, engine, slot: int) -> None:
        """Attach actor (online), target network and memory to agent ``slot`` of a DeviceDQNBatch."""
        self.actor.q_network.bind(engine, "online", slot)
        self.target_network.bind(engine, "target", slot)
        self.buffer.bind(engine, slot)
        self._engine, self._slot = engine, slot

    def _device(self):
        if self._engine is None:
            from .dqn import DeviceDQNBatch
            eng = DeviceDQNBatch(1, 1, 0, 1, device=setup.device, gamma=self._gamma, tau=self._tau,
                                 lr=self.optimizer.learning_rate, capacity=self.buffer.buffer_size, init_seed=None)
            self.actor.q_network.bind(eng, "online", 0)
            self.target_network.bind(eng, "target", 0)
            self._engine, self._slot = eng, 0
        return self._engine, self._slot

    def initialize_target(self) -> None:
        self.buffer.sample_batch()  # the reference draws a batch to build the Keras models (rl.py:275)
        self._soft_update(self.actor.q_network, self.target_network, tau=1.0)

    def load_from_file(self, setting: str, implementation: str) -> None:
        self.target_network.load_weights(os.path.join(MODELS_DIR, f"models_{implementation}", f"{setting}_target"))

    def save_to_file(self, setting: str, implementation: str) -> None:
        self.target_network.save_weights(os.path.join(MODELS_DIR, f"models_{implementation}", f"{setting}_target"))

    def train(self) -> float:
        s, a, r, ns = self.buffer.sample_batch()
        return self._train(s, a, r, ns)

    def _train(self, states, actions, rewards, next_states) -> float:
        """One Trainer._train + update_targets on the device (the soft update is fused)."""
        eng, slot = self._device()
        return eng.train_batch(states, actions, rewards, next_states, net=slot)

    def _soft_update(self, source: QNetwork, target: QNetwork, tau: float = 1.0) -> None:
        ts, tt = source.flat_weights(), target.flat_weights()
        target.set_flat_weights(ts if tau == 1.0 else (np.float32(1 - tau) * tt + np.float32(tau) * ts))

    def update_targets(self) -> None:
        """Applied inside every device train step (rl.py:356-359 follows each _train)."""
