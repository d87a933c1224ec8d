"""The f32 throughput mode (q_dtype="f32": tables and TD arithmetic in f32)
held to north_star's 1e-5 against the reference's f64 tables (rl.py:73 np.zeros, rl.py:119-129).

The reference-driven loop fixtures (tests/golden/make_golden.py: the reference's own QActor and
temperature_simulation, exploration replayed from its np.random stream) are re-run with f32 tables.
Actions and state indices must equal the f64 fixture's; rewards, costs, flows and temperatures
(f32 in both modes) must be within 1e-5 relative (they are equal while the trajectories agree);
every Q entry the fixture's table holds must be within 1e-5 relative of its f64 value, and the
tables must hold the same non-zero entries.  A greedy tie flip (two actions whose Q values the f32
rounding reorders) would make the trajectories diverge; the test then reports the first divergent
(episode, step) and checks the tolerance up to it.  None occurs on these fixtures.
"""
import numpy as np
import pytest

from conftest import load_golden
from p2pmicrogrid_amd.engine import DeviceCommunityBatch, unpack_index

pytestmark = pytest.mark.gpu

REC = ["reward", "cost", "grid", "p2p", "t_in", "action", "index"]
RTOL = 1e-5  # north_star: "power flows, prices, rewards and Q-values within 1e-5 relative in fp32"


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    den = np.maximum(np.abs(b), np.finfo(np.float32).tiny)
    return float(np.max(np.abs(a - b) / den)) if a.size else 0.0


def _engine(d, q_dtype, prefix=""):
    N, R = int(d["N"]), int(d["R"])
    T = d[f"{prefix}env_time"].shape[-1]
    eng = DeviceCommunityBatch(1, N, R, T, q_dtype=q_dtype)
    eng.set_env(d[f"{prefix}env_time"], d[f"{prefix}env_tout"], d[f"{prefix}buy"], d[f"{prefix}inj"],
                d[f"{prefix}p2pp"])
    eng.set_profiles(d[f"{prefix}load_w"][None], d[f"{prefix}pv_w"][None])
    eng.set_max_in(d["max_in"][None])
    return eng


@pytest.mark.parametrize("name", ["loop_thesis_T96", "loop_thesis_T672", "loop_n5_r2_T96"])
def test_f32_tables_track_reference_f64_trajectory(name):
    d = load_golden(name)
    E = int(d["E"])
    eng = _engine(d, "f32")
    worst = {"flows": 0.0, "q": 0.0}
    for e in range(E):
        eng.set_temperatures(d["t_in0"][e][None], d["t_m0"][e][None])
        eng.set_replay_codes(d["codes"][e])
        eng.run_episode("train", "replay", episode=e, epsilon=float(d["eps"][e]), record=REC)
        rec = eng.get_records(REC)
        act, idx = rec["action"][:, :, 0], unpack_index(rec["index"][:, :, 0])
        same = np.all(act == d["train_action"][e], axis=(1, 2)) & np.all(idx == d["train_idx"][e], axis=(1, 2, 3))
        upto = len(same) if same.all() else int(np.argmin(same))
        for k in ("reward", "cost", "grid", "p2p", "t_in"):
            r = _rel(rec[k][:upto, 0], d[f"train_{k}"][e][:upto])
            worst["flows"] = max(worst["flows"], r)
            assert r <= RTOL, (name, e, k, r)
        assert same.all(), f"{name}: f32 tables diverge from the f64 trajectory at episode {e}, step {upto}"
        q = eng.get_q(dtype=np.float64)
        qi, qv = d[f"q_idx_{e}"], d[f"q_val_{e}"]
        assert np.count_nonzero(q) == len(qv), (name, e)
        r = _rel(q[tuple(qi.T)], qv)
        worst["q"] = max(worst["q"], r)
        assert r <= RTOL, (name, e, "q", r)
    # greedy evaluation day with the f32 tables: the same actions as the f64 fixture's
    ev = _engine(d, "f32", prefix="eval_")
    ev.set_q(eng.get_q(dtype=np.float32))
    ev.set_temperatures(d["eval_t_in0"][None], d["eval_t_m0"][None])
    ev.run_episode("greedy", record=REC)
    rec = ev.get_records(REC)
    assert np.array_equal(rec["action"][:, :, 0], d["eval_action"])
    assert np.array_equal(unpack_index(rec["index"][:, :, 0]), d["eval_idx"])
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert _rel(rec[k][:, 0], d[f"eval_{k}"]) <= RTOL, k
    print(f"{name}: max relative error flows {worst['flows']:.3g}, Q {worst['q']:.3g}")
    eng.close()
    ev.close()
