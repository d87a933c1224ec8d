"""PV production (mirrors microgrid/production.py:23-64).

The profiles are parameter containers: ``CommunityMicrogrid`` uploads them to HBM as the
per-agent [T] PV series the episode kernel reads (a14 in SURVEY.md §8a).
"""
from __future__ import annotations

from abc import abstractmethod
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from .dataset import ProfileDataset
from .electrical_asset import ElectricalAsset


class Production(ElectricalAsset):

    @property
    @abstractmethod
    def production(self): ...

    @abstractmethod
    def reset(self) -> None: ...

    @abstractmethod
    def series(self, T: int) -> np.ndarray: ...


@dataclass
class PV:
    peak_power: float
    production: ProfileDataset


class Prosumer(Production):

    def __init__(self, pv: PV):
        self.pv = pv
        self._time = 0
        self._history: Optional[List[float]] = None

    @property
    def production(self):
        """(p_t, p_{t+1}) at the current step (production.py:30-32)."""
        d = self.pv.production
        return d.data[self._time % len(d)], d.rolled[self._time % len(d)]

    def series(self, T: int) -> np.ndarray:
        return np.asarray(self.pv.production.data, dtype=np.float32).reshape(-1)[:T]

    def step(self) -> None:
        self._time += 1

    def get_history(self) -> List[float]:
        return [float(p) for p in np.asarray(self.pv.production.data).reshape(-1)]

    def reset(self) -> None:
        self._time = 0


class Consumer(Production):
    """No PV (production.py:44-58)."""

    def __init__(self) -> None:
        self._production = (np.float32(0.), np.float32(0.))

    @property
    def production(self):
        return self._production

    def series(self, T: int) -> np.ndarray:
        return np.zeros(T, np.float32)

    def step(self) -> None: ...

    def get_history(self) -> List[float]:
        return []

    def reset(self) -> None: ...
