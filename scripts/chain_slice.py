#!/usr/bin/env python3
"""Critical-chain listing of one step of episode_fast_kernel (configs[1]) from its ISA.

    hipcc ... -gline-tables-only --cuda-device-only -S -DP2PMG_PART=1 ... -o fast.s
    python scripts/chain_slice.py fast.s <kernel-symbol-substring> > profiles/r03_fast/chain_listing.txt

Takes the first unrolled step of the episode loop: from the step's first wait on the rows
(s_waitcnt vmcnt) to the last of the next step's row gathers (global_load with an SGPR base).
Walks the straight-line code backward from the gathers' address registers (a def-use slice over
VGPRs / SGPRs / VCC / EXEC), and prints every instruction of the window with a mark: '*' on the
slice (it feeds a next-step row address: forced between the rows' arrival and the gathers), ' '
off the slice (placed inside the window by the scheduler, not needed by the gathers).  Each line
carries the source line (.loc) and a latency class from the single-wave microbenchmark
(scripts/dev/ubench_issue.hip): dependent VALU ~8.4 cycles, f64 ~8.5, transcendental ~12.3, a DPP
move with its hazard nop ~16.3, a compare + 2 selects ~18."""
import re
import sys


def regs(tok):
    """Registers named by one operand token: v5, v[4:7], s[2:3], vcc, exec, ..."""
    tok = tok.strip().lstrip("-").replace("|", "")
    out = []
    m = re.match(r"^([vs])\[(\d+):(\d+)\]", tok)
    if m:
        return [f"{m.group(1)}{k}" for k in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = re.match(r"^([vs])(\d+)$", tok)
    if m:
        return [tok]
    if tok.startswith("vcc"):
        return ["vcc"]
    if tok.startswith("exec"):
        return ["exec"]
    if tok == "scc":
        return ["scc"]
    return out


def parse(line):
    s = line.split(";")[0].strip()
    if not s or s.startswith(".") or s.endswith(":"):
        return None
    parts = s.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    ops = [o.split()[0] if o else o for o in ops]
    dst, src = [], []
    if op.startswith(("global_load", "ds_read", "scratch_load", "buffer_load")):
        dst = regs(ops[0]) if ops else []
        for o in ops[1:]:
            src += regs(o)
    elif op.startswith(("global_store", "ds_write", "scratch_store", "buffer_store", "s_waitcnt", "s_nop",
                        "s_cbranch", "s_branch", "s_barrier", "s_setprio")):
        for o in ops:
            src += regs(o)
    elif op.startswith("v_cmp") and not op.startswith("v_cmpx"):
        dst = regs(ops[0]) if ops else ["vcc"]
        if op.endswith("_e32"):
            dst = ["vcc"]
            src = [r for o in ops for r in regs(o)]
        else:
            src = [r for o in ops[1:] for r in regs(o)]
    else:
        if ops:
            dst = regs(ops[0])
            src = [r for o in ops[1:] for r in regs(o)]
        if op.startswith("v_cndmask_b32_e32") or op.startswith(("v_addc", "v_subb")):
            src.append("vcc")
        if op.startswith("s_") and ("scc" in op or op.startswith(("s_cselect", "s_cmov", "s_addc", "s_subb"))):
            src.append("scc")
        if op.startswith(("s_add", "s_sub", "s_cmp", "s_and", "s_or", "s_xor", "s_lsl", "s_lshr", "s_andn2",
                          "s_orn2", "s_bfe", "s_min", "s_max", "s_not", "s_cselect")):
            dst = dst + ["scc"] if not op.startswith("s_cmp") else ["scc"]
        if "_dpp" in op or "dpp" in s:
            pass
    if op.startswith("v_") and "saveexec" not in op:
        src.append("exec")
    if "saveexec" in op:
        dst += ["exec"]
        src += ["exec"]
    return op, dst, src, s


def lat(op, s):
    if "_dpp" in op or "row_" in s or "quad_perm" in s:
        return "dpp~16"
    if op.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log")):
        return "trans~12"
    if "_f64" in op:
        return "f64~8.5"
    if op.startswith("v_cmp"):
        return "cmp"
    if op.startswith("v_"):
        return "valu~8.4"
    if op.startswith(("global_", "buffer_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "WAIT"
    if op.startswith("s_"):
        return "salu"
    return ""


def main(path, sym):
    lines = open(path).read().splitlines()
    files = {}
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
    start = next(k for k, ln in enumerate(lines) if re.match(r"^\S*" + re.escape(sym) + r"\S*:", ln))
    hdr = next(k for k in range(start, len(lines)) if "Inner Loop Header: Depth=1" in lines[k])
    body = []
    loc = ("?", 0)
    for ln in lines[hdr + 1:]:
        s = ln.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        p = parse(ln)
        if p:
            body.append((p, loc))
    # window: first vmcnt wait .. the 10th SGPR-based row gather after it
    w0 = next(k for k, (p, _) in enumerate(body) if p[0].startswith("s_waitcnt") and "vmcnt" in p[3])
    g = [k for k in range(w0, len(body)) if body[k][0][0].startswith("global_load") and re.search(r",\s*s\[\d+:\d+\]", body[k][0][3])]
    w1 = g[9] if len(g) >= 10 else g[-1]
    win = body[w0:w1 + 1]
    need = set()
    mark = [False] * len(win)
    for k in range(len(win) - 1, -1, -1):
        p, _ = win[k]
        if p[0].startswith("global_load") and re.search(r",\s*s\[\d+:\d+\]", p[3]):
            mark[k] = True
            need.update(r for r in p[2] if r != "exec")  # the gather's address (and exec mask source)
            continue
        if set(p[1]) & need:
            mark[k] = True
            need.difference_update(p[1])
            need.update(r for r in p[2] if r not in ("exec",))
    n_on = sum(1 for k, (p, _) in enumerate(win) if mark[k] and p[0].startswith("v_"))
    n_off = sum(1 for k, (p, _) in enumerate(win) if not mark[k] and p[0].startswith("v_"))
    print(f"# window: {len(win)} instructions from the rows' first wait to the 10th next-step row gather")
    print(f"# VALU on the address slice (*): {n_on}; VALU in the window off the slice: {n_off}")
    for k, (p, (f, l)) in enumerate(win):
        print(f"{'*' if mark[k] else ' '} {lat(p[0], p[3]):9s} {f}:{l:<5d} {p[3]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
