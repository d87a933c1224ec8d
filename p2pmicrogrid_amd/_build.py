"""Build libp2pmg.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo).

    python -m p2pmicrogrid_amd._build        # or __graft_entry__.build()

``-ffp-contract=off`` is part of the numerics contract: every f32/f64 op
rounds separately, matching TF eager / NumPy.  Correctly-rounded f32 division and f32
denormals are hipcc's defaults and are relied upon as well.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libp2pmg.so")
SOURCES = ["p2pmg_kernels.hip", "p2pmg_dqn.hip", "p2pmg_runtime.cpp"]
HEADERS = ["p2pmg_internal.h", "p2pmg_device.h", os.path.join(ROOT, "include", "p2pmg.h")]
ARCH = os.environ.get("P2PMG_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [h if os.path.isabs(h) else os.path.join(CSRC, h)
                                                         for h in HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """defines: extra -D flags (timing-only ablation builds go to a different ``out``)."""
    if out == LIB and not defines and not force and not needs_build():
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-Wno-pass-failed", f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}",
           *[f"-D{d}" for d in defines], *[os.path.join(CSRC, s) for s in SOURCES], "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
