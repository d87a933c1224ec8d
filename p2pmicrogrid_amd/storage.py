"""Storage assets: the interface of the reference's microgrid/storage.py (storage.py:12-116).

Here a battery is a parameter holder.  Its state of charge evolves on the device: the battery
rule of the reference (RuleAgent._update_storage, agent.py:138-153, with BatteryStorage's
sqrt(efficiency) bookkeeping, storage.py:36-76) runs inside the episode kernels
(``battery_rule_r`` in p2pmg_kernels.hip) for communities whose agents carry a battery, and on
explicit balance sequences through ``p2pmg_battery_seq`` (``BatteryStorage.apply_rule``).
``CommunityMicrogrid`` uploads capacities and SoC with ``p2pmg_set_battery`` before a launch and
reads the SoC back with ``p2pmg_get_soc`` after it, as it does for the temperatures.
The reference's RL communities use ``NoStorage`` only (community.py:225).
"""
from __future__ import annotations

from abc import abstractmethod
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from .electrical_asset import ElectricalAsset

RESET_SOC = 0.5  # BatteryStorage.reset (storage.py:73)


@dataclass
class Battery:
    """storage.py:108-116 (capacity in J, peak power in W, SoC bounds and round-trip efficiency)."""
    capacity: float
    peak_power: float
    min_soc: float
    max_soc: float
    efficiency: float
    soc: float


class Storage(ElectricalAsset):
    """storage.py:12-33 (plus ``soc`` / ``capacity``, which the device upload reads)."""

    @property
    @abstractmethod
    def soc(self) -> float: ...

    @property
    @abstractmethod
    def capacity(self) -> float: ...

    @property
    @abstractmethod
    def is_full(self) -> bool: ...

    @property
    @abstractmethod
    def available_space(self) -> float: ...

    @property
    @abstractmethod
    def available_energy(self) -> float: ...

    @abstractmethod
    def to_soc(self, energy: float) -> float: ...

    @abstractmethod
    def charge(self, amount: float) -> None: ...

    @abstractmethod
    def discharge(self, amount: float) -> None: ...


class BatteryStorage(Storage):
    """A battery whose state of charge the device updates (see the module docstring)."""

    def __init__(self, battery: Battery):
        self.battery = battery
        self._time = 0
        self._history: List[float] = []

    @property
    def soc(self) -> float:
        return float(self.battery.soc)

    def set_soc(self, soc: float) -> None:
        """The SoC the device reported after a launch (CommunityMicrogrid pulls it)."""
        self.battery.soc = float(soc)

    @property
    def capacity(self) -> float:
        return float(self.battery.capacity)

    @property
    def is_full(self) -> bool:  # storage.py:41-43
        return self.battery.soc >= self.battery.max_soc

    # The per-call bookkeeping of storage.py:45-64, host-side f64 in the reference's op order, for
    # callers that step a battery themselves (e.g. a ported RuleAgent._update_storage).
    @property
    def available_space(self) -> float:  # storage.py:47-50
        b = self.battery
        return max(0.0, b.max_soc - b.soc) * b.capacity / np.sqrt(b.efficiency)

    @property
    def available_energy(self) -> float:  # storage.py:52-55
        b = self.battery
        return max(0.0, b.soc - b.min_soc) * b.capacity * np.sqrt(b.efficiency)

    def to_soc(self, energy: float) -> float:  # storage.py:57-58
        return energy / self.battery.capacity

    def charge(self, amount: float) -> None:  # storage.py:60-61
        self.battery.soc += np.sqrt(self.battery.efficiency) * amount

    def discharge(self, amount: float) -> None:  # storage.py:63-64
        self.battery.soc -= amount / np.sqrt(self.battery.efficiency)

    def apply_rule(self, balances: Sequence[float]) -> np.ndarray:
        """RuleAgent._update_storage (agent.py:138-153) over a sequence of net balances (W), on the
        device (p2pmg_battery_seq): returns the balances left after the battery, updates the SoC."""
        from .heating import _primitives
        b = self.battery
        out, _, soc = _primitives().battery_seq(np.asarray(balances, np.float64)[None], b.soc, b.capacity,
                                                b.min_soc, b.max_soc, b.efficiency)
        b.soc = float(soc[0])
        return out[0]

    def step(self) -> None:  # storage.py:66-68
        self._history.append(self.soc)
        self._time += 1

    def reset(self) -> None:  # storage.py:70-73
        self._time = 0
        self._history = []
        self.battery.soc = RESET_SOC

    def get_history(self) -> List[float]:
        return self._history


class NoStorage(Storage):
    """storage.py:79-105: no battery (capacity 0 on the device: the kernels skip the rule)."""

    @property
    def soc(self) -> float:
        return 0.0

    @property
    def capacity(self) -> float:
        return 0.0

    @property
    def is_full(self) -> bool:
        return True

    @property
    def available_space(self) -> float:
        return 0

    @property
    def available_energy(self) -> float:
        return 0

    def to_soc(self, energy: float) -> float:
        return 0

    def charge(self, amount: float) -> None: ...

    def discharge(self, amount: float) -> None: ...

    def apply_rule(self, balances: Sequence[float]) -> np.ndarray:
        return np.asarray(balances, np.float64)

    def step(self) -> None: ...

    def reset(self) -> None: ...

    def get_history(self) -> List[float]:
        return []
