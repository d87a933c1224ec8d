"""Device fuzz of the kernels' fast division sequences against the IEEE operator, bit for bit.

The episode kernels divide through a hoisted / per-round reciprocal and two Newton steps
(p2pmg_kernels.hip fdiv_core, fdiv_core_pk, fdiv64, qcore64), relying on the argument that inside
their guarded domains these ARE the IEEE quotient.  The reference's divisions they replace:
agent.py:175 (balance / max_in), :193 (out * |f| / total), :203 (p2p / max_in), community.py:63
(/ 60), heating.py:120 (/ margin) and storage.py:58,61,64 (/ capacity, / sqrt(eff), / 900).
Here ~10^7 random f32 pairs (in range, near the range edges and outside it), every divisor with an
all-ones significand (the hardest case for the reciprocal refinement) and the f64 equivalents go
through p2pmg_fdiv_check / p2pmg_fdiv64_check and must equal a / b exactly (as bit patterns)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _f32_bits(sign, exp, mant):
    return ((sign.astype(np.uint32) << 31) | (exp.astype(np.uint32) << 23) | mant.astype(np.uint32)).view(np.float32)


def _f64_bits(sign, exp, mant):
    return ((sign.astype(np.uint64) << np.uint64(63)) | (exp.astype(np.uint64) << np.uint64(52))
            | mant.astype(np.uint64)).view(np.float64)


def _rand_f32(rs, n, emin, emax):
    return _f32_bits(rs.randint(0, 2, n), rs.randint(emin, emax + 1, n), rs.randint(0, 1 << 23, n))


def _rand_f64(rs, n, emin, emax):
    mant = (rs.randint(0, 1 << 26, n).astype(np.uint64) << np.uint64(26)) | rs.randint(0, 1 << 26, n).astype(np.uint64)
    return _f64_bits(rs.randint(0, 2, n), rs.randint(emin, emax + 1, n), mant)


def _same(x, y):
    return np.array_equal(x.view(np.uint32 if x.dtype == np.float32 else np.uint64),
                          y.view(np.uint32 if y.dtype == np.float32 else np.uint64))


def test_f32_fast_division_is_ieee():
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    eng = DeviceCommunityBatch(1, 1, 0, 1)
    rs = np.random.RandomState(2024)
    n = 2_500_000
    parts = []
    # in the fast domain [2^-40, 2^40] (biased exponents 87..167), a little beyond it, and wide
    for lo, hi in ((87, 167), (80, 175), (1, 254)):
        parts.append((_rand_f32(rs, n, lo, hi), _rand_f32(rs, n, lo, hi)))
    # every all-ones-significand divisor of the fast domain, against random numerators
    exps = np.arange(87, 168)
    d = _f32_bits(np.tile([0, 1], exps.size * 2000), np.repeat(exps, 4000), np.full(exps.size * 4000, (1 << 23) - 1))
    parts.append((_rand_f32(rs, d.size, 87, 167), d))
    # the workload's own magnitudes: powers in W over max_in / totals in W, costs over 60
    w = rs.uniform(-6000, 6000, n).astype(np.float32)
    parts.append((w, rs.uniform(300, 8000, n).astype(np.float32)))
    parts.append((w * rs.uniform(0, 6000, n).astype(np.float32), np.abs(rs.uniform(-12000, 12000, n)).astype(np.float32)))
    parts.append((np.concatenate([np.zeros(4, np.float32), -np.zeros(4, np.float32)]), np.float32([1, -1, 3, 1e-30] * 2)))
    # (form 2, the packed sq16 quotient, is only ever used with a positive divisor: tot = |sum|;
    # the check kernel falls back to form 1 for other divisors, see fdiv_core_pk)
    total = 0
    for a, b in parts:
        out = eng.fdiv_check(a, b)
        ieee = out[:, 3]
        with np.errstate(all="ignore"):
            assert _same(ieee[np.isfinite(ieee)], (a / b)[np.isfinite(ieee)])  # the device IEEE op is the host's
        for k in range(3):
            assert _same(out[:, k], ieee), f"form {k}: {np.flatnonzero(out[:, k].view(np.uint32) != ieee.view(np.uint32))[:5]}"
        total += a.size
    assert total > 10_000_000
    eng.close()


def test_f64_fast_division_is_ieee():
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    eng = DeviceCommunityBatch(1, 1, 0, 1)
    rs = np.random.RandomState(7)
    n = 1_000_000
    parts = []
    for lo, hi in ((723, 1322), (700, 1350), (1, 2046)):  # [2^-300, 2^300) and beyond
        parts.append((_rand_f64(rs, n, lo, hi), _rand_f64(rs, n, lo, hi)))
    exps = np.arange(723, 1323)
    d = _f64_bits(np.tile([0, 1], exps.size * 500), np.repeat(exps, 1000),
                  np.full(exps.size * 1000, (1 << 52) - 1, np.uint64))
    parts.append((_rand_f64(rs, d.size, 723, 1322), d))
    # the battery rule's operands: energies in J over capacities in J, sqrt(0.9), 900 s
    e = rs.uniform(-2e7, 2e7, n)
    parts.append((e, np.full(n, 10 * 3.6e6)))
    parts.append((e / 3.6e7, np.full(n, np.sqrt(0.9))))
    parts.append((e, np.full(n, 900.0)))
    for a, b in parts:
        out = eng.fdiv64_check(a, b)
        for k in range(2):
            assert _same(out[:, k], out[:, 2]), f"form {k}"
    eng.close()
