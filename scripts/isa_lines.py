#!/usr/bin/env python3
"""Per-source-line VALU accounting of one kernel's loop at HEAD (static ISA, -gline-tables-only).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -gline-tables-only \
          --cuda-device-only -S -DP2PMG_PART=5 -I include -I p2pmicrogrid_amd/csrc \
          p2pmicrogrid_amd/csrc/p2pmg_kernels.hip -o sq16.s
    python scripts/isa_lines.py sq16.s <symbol-substring> <weights.json> [phase-map.json]

weights.json: {"loop": [first-block, last-block], "weights": {block: weight, ...}} -- every basic
block of the loop range counts with weight 1 unless listed (0 = a rare path: IEEE fallback
divisions, tot == 0 selects; 0.5 = every other step; 0.125 = the every-8th-step hash flush).
Every instruction is attributed to the nearest preceding .loc (file, line); the phase map
({"phase": [[file-suffix, first, last], ...]}) groups lines.  Prints JSON: per phase and per line
VALU / SALU / LDS / VMEM per wave-step."""
import collections
import json
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_phases import classify  # noqa: E402


def blocks_of(path, sym):
    lines = open(path).read().splitlines()
    files = {}
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2))
    start = next(k for k, ln in enumerate(lines) if re.match(r"^\S*" + re.escape(sym) + r"\S*:", ln))
    end = next(k for k in range(start + 1, len(lines)) if lines[k].strip().startswith(".Lfunc_end"))
    out = collections.OrderedDict()
    cur, loc = "entry", ("?", 0)
    out[cur] = []
    for ln in lines[start:end]:
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(int(m.group(1)), "?").split("/")[-1], int(m.group(2)))
            continue
        if re.match(r"^\.LBB\S*:", s) or re.match(r"^; %bb\.\d+:", s):
            cur = s.split(":")[0] if not s.startswith(";") else s.split()[1].rstrip(":")
            out[cur] = []
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        out[cur].append((loc, s.split()[0]))
    return out


def main(path, sym, weights_path, phase_map=None):
    blocks = blocks_of(path, sym)
    w = json.load(open(weights_path))
    names = list(blocks)
    a, b = names.index(w["loop"][0]), names.index(w["loop"][1])
    pm = json.load(open(phase_map)) if phase_map else {}

    def phase_of(f, line):
        for name, ranges in pm.items():
            for suf, lo, hi in ranges:
                if f.endswith(suf) and lo <= line <= hi:
                    return name
        return "unmapped"

    per_line = collections.defaultdict(collections.Counter)
    per_phase = collections.defaultdict(collections.Counter)
    for name in names[a:b + 1]:
        wt = float(w.get("weights", {}).get(name, 1.0))
        if wt == 0:
            continue
        for (f, line), op in blocks[name]:
            c = classify(op)
            if c in ("valu", "salu", "lds", "vmem", "smem", "mfma"):
                per_line[f"{f}:{line}"][c] += wt
                per_phase[phase_of(f, line)][c] += wt
    tot = sum(v["valu"] for v in per_line.values())
    out = {"symbol": sym, "loop": w["loop"], "weights": w.get("weights", {}),
           "valu_per_wave_step_static": tot,
           "salu_per_wave_step_static": sum(v["salu"] for v in per_line.values()),
           "phases": {k: dict(v, valu_share=round(v["valu"] / tot, 3)) for k, v in
                      sorted(per_phase.items(), key=lambda kv: -kv[1]["valu"])},
           "lines": {k: dict(v) for k, v in sorted(per_line.items(), key=lambda kv: -kv[1]["valu"])}}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
