"""Asset interface (mirrors microgrid/electrical_asset.py:6-15)."""
from abc import ABC, abstractmethod
from typing import List


class ElectricalAsset(ABC):

    @abstractmethod
    def step(self) -> None: ...

    @abstractmethod
    def reset(self) -> None: ...

    @abstractmethod
    def get_history(self) -> List[float]: ...
