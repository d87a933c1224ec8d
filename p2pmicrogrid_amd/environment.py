"""Global environment clock (mirrors microgrid/environment.py:15-65).

``env.setup(dataset)`` takes the (x_t, x_{t+1}) table of [time, temperature] rows built by
``dataset.dataframe_to_dataset``; ``CommunityMicrogrid`` uploads it to the device once per
episode set-up.  ``env.data`` iterates the rows on the host (used by callers that inspect the
timeline; the hot path never iterates on the host).
"""
from __future__ import annotations

from typing import Generator, Optional

import numpy as np

from .dataset import ProfileDataset


class Singleton(type):
    _instances = {}

    def __call__(cls, *args, **kwargs):
        if cls not in cls._instances:
            cls._instances[cls] = super(Singleton, cls).__call__(*args, **kwargs)
        return cls._instances[cls]


class Environment(metaclass=Singleton):

    def __init__(self):
        self._initialized = False
        self._running = False
        self._length: int = 0
        self._time: float = 0.
        self._temperature: float = 0.
        self._dataset: Optional[ProfileDataset] = None
        self.version = 0  # bumped on every setup(): communities re-upload the environment

    def setup(self, data: ProfileDataset) -> None:
        self._dataset = data
        self._length = len(data)
        self._initialized = True
        self.version += 1

    @property
    def dataset(self) -> Optional[ProfileDataset]:
        return self._dataset

    @property
    def data(self) -> Generator:
        if not self._initialized:
            return None
        return self._iterate()

    def _iterate(self):
        self._running = True
        for d in self._dataset:
            self._time = d[0][0]
            self._temperature = d[0][1]
            yield d
        self._running = False

    @property
    def time(self) -> float:
        return self._time if self._running else 0.

    @property
    def temperature(self) -> float:
        return self._temperature if self._running else 0.

    def arrays(self):
        """(time [T] f32, t_out [T] f32) of the current dataset."""
        d = np.asarray(self._dataset.data, dtype=np.float32)
        return np.ascontiguousarray(d[:, 0]), np.ascontiguousarray(d[:, 1])

    def __len__(self) -> int:
        return self._length


env = Environment()
