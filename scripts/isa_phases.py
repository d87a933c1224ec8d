#!/usr/bin/env python3
"""Per-phase instruction accounting of one kernel's ISA (static, from -gline-tables-only asm).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -gline-tables-only --cuda-device-only \
          -S -DP2PMG_PART=5 -I include -I p2pmicrogrid_amd/csrc p2pmicrogrid_amd/csrc/p2pmg_kernels.hip -o sq16.s
    python scripts/isa_phases.py sq16.s <symbol-substring> <phase-map.json>

Every instruction is attributed to the source line of the nearest preceding ``.loc``; a phase map
({"phase": [[file-suffix, first, last], ...]}) turns lines into phases.  Basic blocks are listed
with their instruction mix so rare paths (fallback divisions, probing loops) can be told apart
from the per-step path.  Output: JSON with per-block and per-phase VALU / SALU / VMEM / LDS counts."""
import collections
import json
import re
import sys


def classify(op):
    if op.startswith(("v_mfma", "v_smfmac")):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sleep")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main(path, sym, phase_map=None):
    lines = open(path).read().splitlines()
    files = {}
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2))
    start = next(k for k, ln in enumerate(lines) if re.match(r"^\S*" + re.escape(sym) + r"\S*:", ln))
    end = next(k for k in range(start + 1, len(lines)) if lines[k].strip().startswith(".Lfunc_end"))
    pm = json.load(open(phase_map)) if phase_map else {}

    def phase_of(f, line):
        for name, ranges in pm.items():
            for suf, a, b in ranges:
                if f.endswith(suf) and a <= line <= b:
                    return name
        return f"{f.split('/')[-1]}:{line}"

    blocks = []
    cur = {"label": "entry", "n": collections.Counter(), "phases": collections.Counter(), "branches": []}
    loc = ("?", 0)
    for ln in lines[start:end]:
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        if re.match(r"^\.LBB\S*:", s) or re.match(r"^; %bb\.\d+:", s):
            blocks.append(cur)
            cur = {"label": s.split(":")[0] if not s.startswith(";") else s.split()[1].rstrip(":"), "n": collections.Counter(), "phases": collections.Counter(),
                   "branches": []}
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c = classify(op)
        cur["n"][c] += 1
        if c in ("valu", "salu", "lds", "vmem", "smem", "mfma"):
            cur["phases"][(phase_of(*loc), c)] += 1
        if c == "branch":
            cur["branches"].append(s)
    blocks.append(cur)
    out = {"symbol": sym, "blocks": []}
    for b in blocks:
        ph = collections.defaultdict(dict)
        for (p, c), n in b["phases"].items():
            ph[p][c] = n
        out["blocks"].append({"label": b["label"], "counts": dict(b["n"]), "branches": b["branches"],
                              "phases": dict(ph)})
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
