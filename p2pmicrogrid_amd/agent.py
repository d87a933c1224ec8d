"""Agents (mirrors microgrid/agent.py:23-350).

Agents keep the reference's constructors and attributes.  Inside ``CommunityMicrogrid`` their
per-step work is fused: one device launch per episode runs the negotiation, market, reward,
TD update and RC step of every agent (p2pmg_run_episode).

The per-agent step methods also exist, for callers that step agents themselves
(``__call__``, ``take_decision``, ``get_reward``, ``train``, ``save_memory``, ``step``, ``reset``;
agent.py:111-136, 200-250, 271-298, 312-342).  They run the reference's op order on f32 host
values and call the device for the learner (QActor / Q-network calls, p2pmg_q_calls /
p2pmg_dqn_*) and for the RC update (p2pmg_rc_step).  Each call is a handful of tiny launches:
correct, but the batched community path is the one to use for throughput.
"""
from __future__ import annotations

import re
from abc import ABC, abstractmethod
from typing import Optional, Tuple

import numpy as np

from . import setup
from .dataset import ProfileDataset
from .heating import Heating
from .production import Production
from . import rl
from .rl import QActor
from .storage import Storage

F32 = np.float32


def _f32(x) -> np.ndarray:
    return np.asarray(x.numpy() if hasattr(x, "numpy") else x, dtype=F32)


def reduce_sum(v) -> np.float32:
    """tf.math.reduce_sum of a small f32 vector in the build's canonical order, sequential from
    +0.0 (the order the kernels and the oracle use)."""
    acc = F32(0.0)
    for x in _f32(v).ravel():
        acc = F32(acc + x)
    return acc


def reduce_mean(v) -> np.float32:
    v = _f32(v).ravel()
    return F32(reduce_sum(v) / F32(v.size))


def divide_power(out, powers) -> np.ndarray:
    """RLAgent._divide_power (agent.py:186-195): keep the peers' powers of the opposite sign,
    split ``out`` in proportion to them, or evenly over all N entries when none is kept."""
    out = _f32(out).reshape(-1)
    powers = _f32(powers).ravel()
    filtered = np.where(np.sign(out) != np.sign(powers), powers, F32(0.0)).astype(F32)
    total = np.abs(reduce_sum(filtered))
    if total == F32(0.0):
        return ((out * np.ones(powers.shape, F32)) / F32(powers.shape[0])).astype(F32)
    return ((out * np.abs(filtered)) / total).astype(F32)


class Agent(ABC):

    __last_id = -1

    def __init__(self):
        self.id = Agent.__last_id + 1
        Agent.__last_id += 1
        self.time: int = 0

    @classmethod
    def reset_ids(cls) -> None:
        Agent.__last_id = -1

    @abstractmethod
    def take_decision(self, *args, **kwargs): ...

    def step(self) -> None:
        self.time += 1

    def reset(self) -> None:
        self.time = 0


class GridAgent(Agent):
    """Time-of-use grid prices (agent.py:46-67).  ``take_decision(state)`` returns the f32
    (buy, injection) pair for the state's normalised time; the community precomputes the whole
    table once per environment (engine.price_table)."""

    def __init__(self):
        super().__init__()
        self._cost_avg = setup.GRID_COST_AVG
        self._cost_amplitude = setup.GRID_COST_AMPLITUDE
        self._cost_phase = setup.GRID_COST_PHASE
        self._cost_frequency = 2 * np.pi * setup.HOURS_PER_DAY / setup.GRID_COST_PERIOD
        self._cost_normalization = setup.CENTS_PER_EURO
        self._injection_price = np.array([setup.GRID_INJECTION_PRICE], np.float32)

    def take_decision(self, state, **kwargs) -> Tuple[np.ndarray, np.ndarray]:
        from .engine import price_table
        x = state.numpy() if hasattr(state, "numpy") else state
        buy, _, _ = price_table(np.asarray(x, np.float32).reshape(-1)[:1])
        return buy[0], self._injection_price


class ActingAgent(Agent, ABC):

    def __init__(self, load: ProfileDataset, production: Production, storage: Storage, heating: Heating,
                 max_in: float, max_out: float, *args, **kwargs):
        super().__init__()
        self.max_in = max_in
        self.max_out = max_out  # stored, never read (community.py:228)
        self._load = load
        self._load_pos = 0  # position of the reference's ``self.load`` generator (agent.py:79)
        self.pv = production
        self.storage = storage
        self.heating = heating

    def _next_load_item(self):
        """next(self.load): (x_t, x_{t+1}) of the load stream; StopIteration at its end."""
        d = self._load
        if self._load_pos >= len(d):
            raise StopIteration
        k = self._load_pos
        self._load_pos += 1
        return F32(np.asarray(d.data[k]).reshape(-1)[0]), F32(np.asarray(d.rolled[k]).reshape(-1)[0])

    @abstractmethod
    def __call__(self, *args, **kwargs): ...

    def load_series(self, T: int) -> np.ndarray:
        return np.asarray(self._load.data, dtype=np.float32).reshape(-1)[:T]

    def step(self) -> None:
        super().step()
        self.pv.step()
        self.storage.step()
        self.heating.step()

    def reset(self) -> None:
        super().reset()
        self._load_pos = 0
        self.pv.reset()
        self.storage.reset()
        self.heating.reset()

    def set_profiles(self, load: ProfileDataset, pv_gen: ProfileDataset) -> None:
        """agent.py:100-103: new load / PV series (re-uploaded by the community) and a reset."""
        self._load = load
        self.pv.pv.production = pv_gen
        self.reset()


class RuleAgent(ActingAgent):
    """Rule-based baseline (agent.py:106-153): the heat pump follows a hysteresis on the indoor
    temperature (on at T_in <= setpoint - 1, off at T_in >= setpoint + 1), the net power is
    (load - pv) + heat-pump power, and nothing is learned.  Inside a CommunityMicrogrid
    (``get_rule_based_community``) a whole run is one device launch (rule_episode_kernel)."""

    def __call__(self, *args, **kwargs):
        return self.take_decision(*args, **kwargs)

    def take_decision(self, *args, **kwargs) -> Tuple[np.ndarray, np.ndarray]:
        """agent.py:116-128: hysteresis on the pre-step T_in, then (load - pv) + heat-pump power."""
        t = F32(self.heating.temperature[0])
        if t <= F32(self.heating.lower_bound):
            self.heating.set_power(1)
        elif t >= F32(self.heating.upper_bound):
            self.heating.set_power(0)
        current_load, _ = self._next_load_item()
        current_pv, _ = self.pv.production
        balance = F32(current_load - F32(current_pv))
        return (np.array([balance], F32) + self.heating.power).astype(F32), np.array([0.], F32)

    def _update_storage(self, balance: float) -> float:
        """agent.py:138-153 (never called by the reference's communities): the greedy battery
        rule on one net balance (W), run on the device by the agent's storage (p2pmg_battery_seq)."""
        return float(self.storage.apply_rule([balance])[0])


class RLAgent(ActingAgent):
    """agent.py:156-252.  The per-step methods run the reference's TF op order on f32 host
    values; the learner calls (select/greedy action, TD update) run on the device."""

    def __init__(self, actor, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.actor = actor
        self._next_load = self._next_load_item()        # agent.py:163-164
        self._next_production = self.pv.production
        self._current_balance = None
        self._next_balance = None
        self._current_state = None
        self._action = None

    def _get_balance(self) -> Tuple[np.ndarray, np.ndarray]:
        """agent.py:172-176: (load - pv) / max_in of this step and of the next one."""
        load, pv = self._next_load, self._next_production
        mi = F32(self.max_in)
        return (np.array([F32(load[0]) - F32(pv[0])], F32) / mi).astype(F32), \
               (np.array([F32(load[1]) - F32(pv[1])], F32) / mi).astype(F32)

    def _get_observation_state(self, state, balance, p2p) -> np.ndarray:
        """agent.py:178-184: [time, normalised T_in, balance, p2p] as a (1, 4) f32 row."""
        st = _f32(state)
        time = st.reshape(-1)[:1] if st.ndim <= 1 else st[:, 0]
        return np.concatenate([time, self.heating.normalized_temperature, _f32(balance).reshape(-1),
                               _f32(p2p).reshape(1)]).astype(F32)[None, :]

    def _divide_power(self, out, powers) -> np.ndarray:
        return divide_power(out, powers)

    def _act(self):
        raise NotImplementedError

    def __call__(self, state, powers, *args, **kwargs):
        """agent.py:200-213: exploring decision for one negotiation round."""
        powers = _f32(powers).ravel()
        p2p = F32(reduce_mean(powers) / F32(self.max_in))
        self._current_balance, self._next_balance = self._get_balance()
        self._current_state = self._get_observation_state(state, self._current_balance, p2p)
        q_val = self._act()
        p_out = self._divide_power(self._current_balance * F32(self.max_in) + self.heating.power, powers)
        return p_out, q_val

    def take_decision(self, state, powers, *args, **kwargs):
        raise NotImplementedError

    def get_reward(self, cost) -> np.ndarray:
        """agent.py:225-232: -(cost + 10 * penalty), penalty = distance outside the comfort band + 1."""
        t = _f32(self.heating.temperature)
        lo, hi = F32(self.heating.lower_bound), F32(self.heating.upper_bound)
        pen = np.maximum(np.maximum(F32(0.0), lo - t), np.maximum(F32(0.0), t - hi)).astype(F32)
        pen = np.where(pen > F32(0.0), pen + F32(1.0), F32(0.0)).astype(F32)
        return (-(_f32(cost) + F32(10.0) * pen)).astype(F32)

    def save_memory(self, reward, next_state, powers) -> None:
        pass

    def train(self, reward, next_state, powers) -> float:
        raise NotImplementedError

    def step(self) -> None:
        """agent.py:234-241: advance the assets and the profile streams (None at their end)."""
        super().step()
        try:
            self._next_load = self._next_load_item()
            self._next_production = self.pv.production
        except StopIteration:
            self._next_load = None
            self._next_production = None

    def reset(self) -> None:
        super().reset()
        self._next_load = self._next_load_item()
        self._next_production = self.pv.production

    def load_from_file(self, setting: str, implementation: str) -> None:
        self.actor.load_from_file(f'{re.sub("-", "_", setting)}_{self.id}', implementation)

    def save_to_file(self, setting: str, implementation: str) -> None:
        self.actor.save_to_file(f'{re.sub("-", "_", setting)}_{self.id}', implementation)


class QAgent(RLAgent):
    """Tabular Q-learning agent (agent.py:255-298): 20 x 20 x 20 x 20 states, 3 heat-pump levels,
    epsilon 0.81 decayed x0.9."""

    def __init__(self, *args, **kwargs):
        self._num_time_states = 20
        self._num_temp_states = 20
        self._num_balance_states = 20
        self._num_p2p_states = 20
        actor = QActor(self._num_time_states, self._num_temp_states, self._num_balance_states,
                       self._num_p2p_states, epsilon=0.81, decay=0.9)
        super().__init__(actor, *args, **kwargs)
        self._actions = np.array([0., 0.5, 1.])
        self._last_action: int = -1

    def _act(self):
        """agent.py:271-275: epsilon-greedy on the device table, then the heat-pump set-point."""
        self._last_action, q = self.actor.select_action(self._current_state)
        self.heating.set_power(float(self._actions[self._last_action]))
        return q

    def take_decision(self, state, powers, *args, **kwargs):
        """agent.py:277-289: greedy decision (evaluation)."""
        powers = _f32(powers).ravel()
        p2p = F32(reduce_mean(powers) / F32(self.max_in))
        current_balance = self._get_balance()[0]
        new_state = self._get_observation_state(state, current_balance, p2p)
        action, q = self.actor.greedy_action(new_state)
        self.heating.set_power(float(self._actions[action]))
        p_out = self._divide_power(current_balance * F32(self.max_in) + self.heating.power, powers)
        return p_out, q

    def train(self, reward, next_state, powers) -> float:
        """agent.py:293-298: TD update of the last round's (state, action) towards the next state
        (p2p from ``powers``, the same pre-update T_in)."""
        p2p = F32(reduce_mean(powers) / F32(self.max_in))
        ns = self._get_observation_state(next_state, self._next_balance, p2p)
        self.actor.train(self._current_state, self._last_action, reward, ns)
        return 0.


class DQNAgent(RLAgent):
    """Deep Q-learning agent (agent.py:301-350): ActorModel(epsilon=1), Trainer with a 5000-entry
    memory, batch 32, gamma 0.95, tau 0.005, Adam(1e-5).  Inside a CommunityMicrogrid its
    networks, Adam state and memory are slot ``i`` of the community's DeviceDQNBatch."""

    def __init__(self, *args, **kwargs) -> None:
        super().__init__(rl.ActorModel(1), *args, **kwargs)
        self.trainer = rl.Trainer(self.actor, buffer_size=5 * 1000, batch_size=32, gamma=0.95, tau=0.005,
                                  optimizer=rl.Adam(learning_rate=1e-5))

    def _act(self):
        """agent.py:312-316"""
        self._action, q_val = self.actor.select_action(self._current_state)
        self.heating.set_power(float(self._action[0]))
        return q_val

    def take_decision(self, state, powers, *args, **kwargs):
        """agent.py:318-331: greedy action of the Q-network (evaluation)."""
        powers = _f32(powers).ravel()
        p2p = F32(reduce_mean(powers) / F32(self.max_in))
        current_balance = self._get_balance()[0]
        new_state = self._get_observation_state(state, current_balance, p2p)
        action, q = self.actor.greedy_action(new_state)
        self.heating.set_power(float(action[0]))
        p_out = self._divide_power(current_balance * F32(self.max_in) + self.heating.power, powers)
        return p_out, q[:, 0]

    def save_memory(self, reward, next_state, powers) -> None:
        """agent.py:333-336: (s, a, r, s') into the agent's replay memory."""
        p2p = F32(reduce_mean(powers) / F32(self.max_in))
        ns = self._get_observation_state(next_state, self._next_balance, p2p)
        self.trainer.buffer.add(self._current_state[0, :], self._action, _f32(reward), ns[0, :])

    def train(self, reward, next_state, powers) -> float:
        """agent.py:338-342"""
        self.save_memory(reward, next_state, powers)
        return self.trainer.train()

    def load_from_file(self, setting: str, implementation: str) -> None:
        super().load_from_file(setting, implementation)
        self.trainer.load_from_file(f'{re.sub("-", "_", setting)}_{self.id}', implementation)

    def save_to_file(self, setting: str, implementation: str) -> None:
        super().save_to_file(setting, implementation)
        self.trainer.save_to_file(f'{re.sub("-", "_", setting)}_{self.id}', implementation)


def agent_kind(agent) -> Optional[str]:
    if isinstance(agent, QAgent):
        return "tabular"
    if isinstance(agent, DQNAgent):
        return "dqn"
    if isinstance(agent, RuleAgent):
        return "rule"
    return None
