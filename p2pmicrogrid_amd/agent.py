"""Agents (mirrors microgrid/agent.py:23-298).

Agents are parameter holders with the reference's constructors and attributes.  Their per-step
methods (``__call__``, ``take_decision``, ``get_reward``, ``train``) are not called one agent at
a time: ``CommunityMicrogrid`` fuses the whole negotiation / market / reward / TD / RC step of
every agent into one device launch per episode (p2pmg_run_episode).  Calling them directly
raises with a pointer to that path.
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

_FUSED = ("per-agent step calls are fused into the community episode kernel; use "
          "CommunityMicrogrid.train_episode() / run() (p2pmg_run_episode)")


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
        self.pv = production
        self.storage = storage
        self.heating = heating

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
        raise NotImplementedError(_FUSED)

    def take_decision(self, *args, **kwargs):
        raise NotImplementedError(_FUSED)

    def _update_storage(self, balance: float) -> float:
        """agent.py:138-153: greedy battery rule on the net balance (W); returns the remainder.
        The reference never calls it from a community; kept for scripts that do."""
        energy = balance * setup.SECONDS_PER_MINUTE * setup.TIME_SLOT
        if balance > 0 and self.storage.available_energy > 0:
            to_extract = min(energy, self.storage.available_energy)
            self.storage.discharge(self.storage.to_soc(to_extract))
            balance -= to_extract / (setup.SECONDS_PER_MINUTE * setup.TIME_SLOT)
        elif balance < 0 and not self.storage.is_full:
            to_store = min(-energy, self.storage.available_space)
            self.storage.charge(self.storage.to_soc(to_store))
            balance += to_store / (setup.SECONDS_PER_MINUTE * setup.TIME_SLOT)
        return balance


class RLAgent(ActingAgent):

    def __init__(self, actor, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.actor = actor

    def __call__(self, state, powers, *args, **kwargs):
        raise NotImplementedError(_FUSED)

    def take_decision(self, state, powers, *args, **kwargs):
        raise NotImplementedError(_FUSED)

    def get_reward(self, cost):
        raise NotImplementedError(_FUSED)

    def train(self, reward, next_state, powers) -> float:
        raise NotImplementedError(_FUSED)

    def save_memory(self, reward, next_state, powers) -> None:
        raise NotImplementedError(_FUSED)

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


class DQNAgent(RLAgent):
    """Deep Q-learning agent (agent.py:301-350): ActorModel(epsilon=1), Trainer with a 5000-entry
    memory, batch 32, gamma 0.95, tau 0.005, Adam(1e-5).  Inside a CommunityMicrogrid its
    networks, Adam state and memory are slot ``i`` of the community's DeviceDQNBatch."""

    def __init__(self, *args, **kwargs) -> None:
        super().__init__(rl.ActorModel(1), *args, **kwargs)
        self.trainer = rl.Trainer(self.actor, buffer_size=5 * 1000, batch_size=32, gamma=0.95, tau=0.005,
                                  optimizer=rl.Adam(learning_rate=1e-5))

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
