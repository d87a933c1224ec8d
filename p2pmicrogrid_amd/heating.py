"""Heat-pump heating and the 2-node RC thermal model (mirrors microgrid/heating.py:17-163).

``temperature_simulation`` keeps the reference signature but runs batched on the device
(p2pmg_rc_step): scalars or arrays of any matching shape.  ``HPHeating`` holds an agent's
thermal parameters and its T_in / T_m between episodes; during an episode the state lives in
the kernel's registers.
"""
from __future__ import annotations

import threading
from abc import abstractmethod
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from . import setup
from .electrical_asset import ElectricalAsset

# Simulator parameters (heating.py:23-29)
Ci = 2.44e6 * 2
Cm = 9.4e7
Ri = 8.64e-4
Re = 1.05e-2
Rvent = 7.98e-3
gA = 11.468
f_rad = 0.3

_prim = None
_prim_lock = threading.Lock()


def _primitives():
    """A minimal device context for the batched primitives (one per process)."""
    global _prim
    with _prim_lock:
        if _prim is None:
            from .engine import DeviceCommunityBatch
            _prim = DeviceCommunityBatch(1, 1, 0, 1, device=setup.device)
        return _prim


def temperature_simulation(t_out, t_in, t_bm, hp_power, hp_cop: float = 3.0,
                           solar_rad: float = 0) -> Tuple[np.ndarray, np.ndarray]:
    """heating.py:37-56 on the device, f32 with the reference's constant casts.  Only the
    reference's constants are compiled into the primitive: hp_cop must be 3.0 and solar_rad 0
    (the values every reference caller uses, community.py:226)."""
    if float(hp_cop) != 3.0 or float(solar_rad) != 0.0:
        raise NotImplementedError("temperature_simulation: only hp_cop=3.0, solar_rad=0 are supported")
    a, b = _primitives().rc_step(t_out, t_in, t_bm, hp_power)
    if np.ndim(a) == 0:
        return np.float32(a), np.float32(b)
    return a, b


class Heating(ElectricalAsset):

    @property
    @abstractmethod
    def lower_bound(self) -> float: ...

    @property
    @abstractmethod
    def upper_bound(self) -> float: ...

    @property
    @abstractmethod
    def temperature(self): ...

    @property
    @abstractmethod
    def normalized_temperature(self): ...

    @property
    @abstractmethod
    def power(self): ...

    @abstractmethod
    def has_heater(self) -> bool: ...

    @abstractmethod
    def set_power(self, power: float) -> None: ...


@dataclass
class HeatPump:
    cop: float
    max_power: float
    power: float


class HPHeating(Heating):
    """Heat pump + RC house.  The initial temperatures are drawn exactly as the reference draws
    them from the global np.random (heating.py:101-104: T_m first, then T_in; homogeneous
    communities start at the setpoint)."""

    TEMPERATURE_MARGIN = 1.

    def __init__(self, hp: HeatPump, temperature_setpoint: float, rng=None):
        from .rng import ReferenceRNG
        self.temperature_choice = (temperature_setpoint - self.TEMPERATURE_MARGIN,
                                   temperature_setpoint + self.TEMPERATURE_MARGIN)
        self.hp = hp
        self._time = 0
        self._history: List[float] = []
        self._power_history: List[float] = []
        self._temperature_setpoint = temperature_setpoint
        self._rng = rng if rng is not None else ReferenceRNG()
        t_in, t_m = self._rng.initial_temperature(temperature_setpoint, setup.homogeneous)
        self._t_indoor = np.array([t_in], np.float32)
        self._t_building_mass = np.array([t_m], np.float32)

    @property
    def lower_bound(self) -> float:
        return self.temperature_choice[0]

    @property
    def upper_bound(self) -> float:
        return self.temperature_choice[1]

    @property
    def temperature(self) -> np.ndarray:
        return self._t_indoor

    @property
    def building_mass_temperature(self) -> np.ndarray:
        return self._t_building_mass

    @property
    def normalized_temperature(self) -> np.ndarray:
        return ((self._t_indoor - np.float32(self._temperature_setpoint))
                / np.float32(self.TEMPERATURE_MARGIN)).astype(np.float32)

    @property
    def power(self) -> np.ndarray:
        return np.array([self.hp.power * self.hp.max_power], np.float32)

    def has_heater(self) -> bool:
        return True

    def set_power(self, power: float) -> None:
        self.hp.power = power

    def set_state(self, t_in: float, t_m: float) -> None:
        self._t_indoor = np.array([t_in], np.float32)
        self._t_building_mass = np.array([t_m], np.float32)

    def step(self) -> None:
        """One RC step on the device with the current heat-pump power (heating.py:138-143)."""
        from .environment import env
        self._history.append(float(self._t_indoor[0]))
        self._power_history.append(float(self.power[0]))
        a, b = temperature_simulation(np.float32(env.temperature), self._t_indoor, self._t_building_mass,
                                      self.power, self.hp.cop)
        self._t_indoor, self._t_building_mass = np.asarray(a, np.float32), np.asarray(b, np.float32)
        self._time += 1

    def reset(self) -> None:
        """heating.py:145-152: new T0, T_in drawn first, then T_m."""
        self._time = 0
        self._history = []
        self._power_history = []
        t_in, t_m = self._rng.reset_temperature(self._temperature_setpoint, setup.homogeneous)
        self._t_indoor = np.array([t_in], np.float32)
        self._t_building_mass = np.array([t_m], np.float32)

    def get_history(self) -> List[float]:
        """heating.py:154-155: T_in before each step of the last run."""
        return self._history
