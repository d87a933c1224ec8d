#!/usr/bin/env python3
"""Cycle-weighted VALU accounting of a kernel loop (static ISA x measured per-instruction costs).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --cuda-device-only -S \\
          -DP2PMG_PART=5 -I include -I p2pmicrogrid_amd/csrc p2pmicrogrid_amd/csrc/p2pmg_kernels.hip -o sq16.s
    python scripts/isa_cycles.py sq16.s <symbol-substring> <weights.json> > out.json

Every VALU instruction of the loop (from the weights file's loop header to its back-edge block) is
costed at the SIMD cycles one wave64 instruction of its kind occupies at 4 waves per SIMD, measured
on the MI355X by scripts/dev/ubench_rate.hip (profiles/r04_ubench_rate.jsonl, r05_ubench_rate.jsonl)
and scripts/ubench_select.hip (profiles/r06_ubench_select.jsonl: a v_cndmask among other VALU costs
2.3 cycles, a v_cmp + v_cndmask pair 7.7; only back-to-back VCC selects cost 23).  Blocks are
weighted by how often a step runs them (weights.json: 0 rare paths, 0.5 every other step, ...; a
block not listed runs once per step).  The sum is the VALU issue floor of one wave-step: the SIMD
time the step's VALU work occupies when the SIMD's waves always have an instruction ready."""
import collections
import json
import re
import sys

# SIMD cycles per wave64 instruction at 4 waves per SIMD (measured; see the docstring)
COST = [
    (r"^v_(add|sub|subrev)_f32", 2.8), (r"^v_mul_f32", 2.63), (r"^v_(fma|fmac|mac)_f32", 3.83),
    (r"^v_med3_f32", 4.28), (r"^v_(max|min)_f32", 4.34), (r"^v_cndmask_b32", 2.3),
    (r"^v_cmp", 5.4), (r"^v_(xor|and|or|not|lshl|lshr|ashr|add|sub|bfe|alignbit|lshl_add|add3|perm|bitop3)",
                       2.8),
    (r"^v_mov_b32", 2.8), (r"^v_mul_lo_u32", 5.06), (r"^v_mul_hi_u32_u24", 4.41), (r"^v_mul_hi_u32", 4.69),
    (r"^v_mad_u64_u32", 5.64), (r"^v_mul_u32_u24", 4.52), (r"^v_fma_f64|^v_fmac_f64", 4.54),
    (r"^v_add_f64", 4.42), (r"^v_mul_f64", 4.64), (r"^v_ldexp", 4.69), (r"^v_cvt_f64", 5.22),
    (r"^v_(max|min)_f64", 4.5), (r"^v_rcp_f32", 8.34), (r"^v_rcp_f64", 8.34), (r"^v_pk_fma_f32", 6.9),
    (r"^v_pk_add_f32", 6.74), (r"^v_pk_mul_f32", 6.71), (r"^v_cvt", 4.34), (r"^v_bfi", 4.46),
]
DEFAULT = 4.0  # nominal one instruction per quad-cycle for kinds not measured


def cost(op):
    for pat, c in COST:
        if re.match(pat, op):
            return c, pat
    return DEFAULT, "other"


def main(path, sym, weights_path):
    w = json.load(open(weights_path))
    head, tail = w["loop"]
    weights = w["weights"]
    lines = open(path).read().splitlines()
    start = next(k for k, ln in enumerate(lines) if re.match(r"^\S*" + re.escape(sym) + r"\S*:", ln))
    end = next(k for k in range(start + 1, len(lines)) if lines[k].strip().startswith(".Lfunc_end"))
    in_loop, label = False, None
    total, n_valu = 0.0, 0.0
    by_kind = collections.Counter()
    cyc_kind = collections.Counter()
    salu = lds = vmem = 0.0
    done = False
    for ln in lines[start:end]:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S*):", s) or re.match(r"^; (%bb\.\d+):", s)
        if m:
            if in_loop and label == tail:
                done = True
            label = m.group(1)
            if label == head:
                in_loop = True
            continue
        if done:
            break
        if not in_loop or not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        wt = float(weights.get(label, 1.0))
        if op.startswith("v_") and not op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            c, kind = cost(op)
            total += wt * c
            n_valu += wt
            by_kind[kind] += wt
            cyc_kind[kind] += wt * c
        elif op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            total += wt * DEFAULT
            n_valu += wt
            by_kind["lane moves"] += wt
            cyc_kind["lane moves"] += wt * DEFAULT
        elif op.startswith("s_") and not op.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch")):
            salu += wt
        elif op.startswith("ds_"):
            lds += wt
        elif op.startswith(("global_", "buffer_")):
            vmem += wt
    out = {"symbol": sym, "weights": weights_path, "valu_per_wave_step": n_valu,
           "valu_cycles_per_wave_step": total, "mean_cycles_per_valu": total / max(n_valu, 1e-9),
           "salu_per_wave_step": salu, "lds_per_wave_step": lds, "vmem_per_wave_step": vmem,
           "by_kind": {k: {"insts": by_kind[k], "cycles": cyc_kind[k]} for k in sorted(cyc_kind, key=lambda x: -cyc_kind[x])}}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
