"""p2pmicrogrid_amd — MI355X-native batched simulator/trainer for the P2PMicrogrid hot path.

The compute path is libp2pmg.so (hand-written HIP for gfx950, C ABI in include/p2pmg.h),
reached through ctypes.  The modules mirror the reference's package layout
(microgrid/{setup,environment,dataset,production,storage,heating,rl,agent,community}.py).
"""
from . import setup  # noqa: F401
from .engine import DeviceCommunityBatch, price_table  # noqa: F401

__all__ = ["setup", "DeviceCommunityBatch", "price_table"]
__version__ = "0.1.0"
