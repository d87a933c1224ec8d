"""Build libp2pmg.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo).

    python -m p2pmicrogrid_amd._build        # or __graft_entry__.build()

``-ffp-contract=off`` is part of the numerics contract: every f32/f64 op
rounds separately, matching TF eager / NumPy.  Correctly-rounded f32 division and f32
denormals are hipcc's defaults and are relied upon as well.
"""
from __future__ import annotations

import fcntl
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


KERNEL_PARTS = 11  # p2pmg_kernels.hip is compiled once per part (-DP2PMG_PART=k), see its header
# Per-part compiler flags.  Part 5 (episode_sq16_kernel, VALU-issue-bound) without the SLP vectorizer:
# SLP packs adjacent f32 adds / muls into v_pk_add_f32 / v_pk_mul_f32, which issue at 6.6 SIMD cycles
# against 2 x 2.9 / 2 x 2.6 for the scalar pair at 4 waves per SIMD (profiles/r04_ubench_rate.jsonl);
# the kernel's explicit packed FMAs (v_pk_fma_f32, 6.8 against 2 x 3.8) stay.  configs[2] 3.18 ->
# 3.07 ms; the latency-bound fast kernel (other parts) measured slower without SLP
# (profiles/r04_sq16_slp_ab.txt).
PART_FLAGS = {5: ["-fno-slp-vectorize"]}


def build(force: bool = False, verbose: bool = True, out: str = LIB, defines=(), jobs: int = 0) -> str:
    """defines: extra -D flags, or raw compiler flags when they start with "-" (timing-only ablation
    builds go to a different ``out``).
    The translation units (11 parts of p2pmg_kernels.hip, p2pmg_dqn.hip, p2pmg_runtime.cpp) compile
    in parallel into build/obj/<tag>/, then link into one shared library.  An exclusive file lock
    per tag serialises concurrent builders (torchrun ranks, pytest-xdist workers that all find the
    sources newer): the later ones wait, see a fresh library and return without compiling."""
    if out == LIB and not defines and not force and not needs_build():
        return LIB
    tag = ARCH + ("_main" if not defines else "_" + "_".join(d.replace("=", "") for d in defines))
    obj_dir = os.path.join(ROOT, "build", "obj", tag)
    os.makedirs(obj_dir, exist_ok=True)
    with open(os.path.join(ROOT, "build", "obj", f"{tag}.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            if out == LIB and not defines and not force and not needs_build():
                return LIB  # another process built it while this one waited
            return _build_locked(obj_dir, out, defines, jobs, verbose, force)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)


def hipcc_identity() -> str:
    """The compiler's path and version line, part of every object's stamp."""
    try:
        v = subprocess.run([hipcc(), "--version"], capture_output=True, text=True, timeout=60).stdout
    except (OSError, subprocess.SubprocessError):
        v = ""
    return hipcc() + " | " + " ".join(v.split())


def _build_locked(obj_dir: str, out: str, defines, jobs: int, verbose: bool, force: bool = False) -> str:
    common = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
              "-Wall", "-Wno-unused-function", "-Wno-pass-failed", f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}",
              *[d if d.startswith("-") else f"-D{d}" for d in defines]]  # "-..." entries: raw flags
    units = [(os.path.join(CSRC, "p2pmg_kernels.hip"), [f"-DP2PMG_PART={k}", *PART_FLAGS.get(k, [])], f"kernels_{k}.o")
             for k in range(KERNEL_PARTS)]
    units += [(os.path.join(CSRC, s), [], os.path.splitext(s)[0] + ".o") for s in SOURCES if s != "p2pmg_kernels.hip"]
    jobs = jobs or min(len(units), max(1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    pending = list(units)
    running = []
    objs = []
    # an object is reused only when it is newer than its source, every header and this script AND
    # its stamp (the full compile command + the compiler's identity) matches; --force rebuilds all
    hdrs = [h if os.path.isabs(h) else os.path.join(CSRC, h) for h in HEADERS] + [os.path.abspath(__file__)]
    newest_hdr = max(os.path.getmtime(h) for h in hdrs if os.path.exists(h))
    ident = hipcc_identity()

    def stamp_of(cmd):
        return ident + "\n" + " ".join(cmd) + "\n"

    def fresh(src, obj, cmd):
        if force or not os.path.exists(obj) or os.path.getmtime(obj) <= max(os.path.getmtime(src), newest_hdr):
            return False
        try:
            return open(obj + ".cmd").read() == stamp_of(cmd)
        except OSError:
            return False

    stamps = []
    while pending or running:
        while pending and len(running) < jobs:
            src, extra, o = pending.pop(0)
            obj = os.path.join(obj_dir, o)
            cmd = [*common, *extra, "-c", src, "-o", obj]
            if fresh(src, obj, cmd):
                objs.append(obj)
                continue
            if os.path.exists(obj + ".cmd"):
                os.remove(obj + ".cmd")
            if verbose:
                print(" ".join(cmd), flush=True)
            running.append((subprocess.Popen(cmd), cmd))
            stamps.append((obj, cmd))
            objs.append(obj)
        if not running:
            break
        proc, cmd = running.pop(0)
        if proc.wait() != 0:
            for q, _ in running:
                q.wait()
            raise subprocess.CalledProcessError(proc.returncode, cmd)
    for obj, cmd in stamps:  # every compile succeeded: record what built each object
        with open(obj + ".cmd", "w") as f:
            f.write(stamp_of(cmd))
    tmp = f"{out}.{os.getpid()}.tmp"
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
