"""Configs 3-4 rows on the device vs the oracle: shared policy table with int64 fixed-point TD
deltas (build-defined), battery storage (storage.py / agent.py:138-153),
N = 16 agents, heterogeneous heat pumps and batteries, RCCL exchange of the deltas."""
import numpy as np
import pytest

from conftest import load_golden
from oracle.restatement import OracleBatch

pytestmark = pytest.mark.gpu
REC = ["reward", "cost", "grid", "p2p", "t_in", "action", "index"]


def test_battery_primitive_matches_reference_storage():
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    d = load_golden("battery")
    eng = DeviceCommunityBatch(1, 1, 0, 1)
    ob, sh, soc = eng.battery_seq(d["bal"][None], float(d["soc0"]), float(d["capacity"]), float(d["min_soc"]),
                                  float(d["max_soc"]), float(d["efficiency"]))
    assert np.array_equal(ob[0], d["out_bal"]) and np.array_equal(sh[0], d["soc"])


def _setup(S, N, R, T, q_dtype, shared, battery, hetero, seed=9):
    from p2pmicrogrid_amd.dataset import scenario_batch
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    inp = scenario_batch(S, N, T, seed=seed)
    rs = np.random.RandomState(seed)
    lv = np.broadcast_to(np.array([0.0, 1500.0, 3000.0], np.float32), (S, N, 3)).copy()
    cap = np.full((S, N), 10 * 3.6e6) if battery else None
    if hetero:  # config 4 mixes: some agents without heat pump, some without battery, other HP sizes
        lv[rs.rand(S, N) < 0.25] = 0.0
        big = rs.rand(S, N) < 0.3
        lv[big] = np.array([0.0, 2500.0, 5000.0], np.float32)
        if battery:
            cap[rs.rand(S, N) < 0.4] = 0.0
    ob = OracleBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in, env_time=inp.time[None],
                     env_tout=inp.t_out, q_dtype=q_dtype, shared_q=shared, hp_levels=lv, battery_capacity=cap)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype, shared_q=shared)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    eng.set_hp_levels(lv)
    if battery:
        eng.set_battery(cap, 0.1, 0.9, 0.9)
    return eng, ob


def _cmp(out, rec, tag):
    from p2pmicrogrid_amd.engine import unpack_index
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert np.array_equal(rec[k], out[k]), (tag, k)
    assert np.array_equal(rec["action"], out["action"].astype(np.uint8)), tag
    assert np.array_equal(unpack_index(rec["index"]), out["idx"]), tag


@pytest.mark.parametrize("N,R,T,q_dtype,shared,battery,hetero", [
    (16, 1, 24, "f32", True, True, False),     # config 3 shape
    (16, 1, 24, "f64", True, False, False),
    (2, 1, 96, "f64", True, True, False),
    (4, 2, 32, "f64", False, True, True),      # config 4 shape: per-agent tables, mixed assets
    (16, 1, 16, "f32", False, True, True),
    (2, 1, 96, "f64", False, False, True),
    (4, 1, 48, "f64", False, True, True),      # configs[3] shape on the fast kernel (battery variant)
    (2, 1, 96, "f64", False, True, True),      # N = 2 with a battery: no round-1 candidate rows
    (3, 0, 24, "f32", False, True, True),
    (8, 1, 24, "f32", False, True, False),
    # community sizes outside {1..8, 16}: the general kernel's LDS-tile form with the shared table's
    # delta hash (4 waves per workgroup; 2 at 64-agent capacity) and the battery rule
    (10, 1, 24, "f32", True, True, False),
    (24, 2, 16, "f64", True, False, True),
    (40, 1, 12, "f32", True, True, True),
    (12, 1, 24, "f64", False, True, True),
])
def test_shared_battery_hetero_match_oracle(N, R, T, q_dtype, shared, battery, hetero):
    S = 24
    eng, ob = _setup(S, N, R, T, q_dtype, shared, battery, hetero)
    for e in range(3):
        eng.run_episode("train", "philox", episode=e, epsilon=0.6, record=REC)
        out = ob.run_episode("train", rng="philox", episode=e, eps=0.6)
        _cmp(out, eng.get_records(REC), (N, shared, battery, hetero, e))
        if battery:
            assert np.array_equal(eng.get_soc(), ob.soc)
        if shared:
            assert np.array_equal(eng.get_q_delta().reshape(-1, 3), ob.q_delta)
            eng.apply_q_delta()
            ob.apply_q_delta()
            assert not eng.get_q_delta().any()
        dt = np.float64 if q_dtype == "f64" else np.float32
        assert np.array_equal(eng.get_q(dtype=dt).reshape(ob.q.shape), ob.q)
    eng.run_episode("greedy", record=REC)
    _cmp(ob.run_episode("greedy"), eng.get_records(REC), "greedy")


def test_sq16_small_epsilon_matches_oracle():
    """configs[2]'s kernel (shared table, N = 16, battery) at epsilon < 2^-8: the exploring lanes'
    actions come from the TAG_ACTION block (p2pmg_device.h::philox_block_codes), as in the oracle."""
    S, N, R, T = 64, 16, 1, 48
    eng, ob = _setup(S, N, R, T, "f32", True, True, False, seed=23)
    for e in range(2):
        eng.run_episode("train", "philox", episode=e, epsilon=0.0035, record=REC)
        assert eng.last_kernel().startswith("episode_sq16_kernel<")
        out = ob.run_episode("train", rng="philox", episode=e, eps=0.0035)
        _cmp(out, eng.get_records(REC), ("small-eps", e))
        assert np.array_equal(eng.get_q_delta().reshape(-1, 3), ob.q_delta)
        eng.apply_q_delta()
        ob.apply_q_delta()


@pytest.mark.parametrize("N", [2, 4])
def test_battery_fast_kernel_narrow_records_match_oracle(N):
    """configs[3] shape on the battery fast kernel: only {reward, cost} requested -> 8-B record rows
    (the bench's request); alternating with full records over back-to-back episodes, every record,
    the SoC and the tables still equal the oracle's."""
    S, R, T = 24, 1, 48
    eng, ob = _setup(S, N, R, T, "f64", False, True, True, seed=21)
    for e in range(4):
        narrow = e % 2 == 0
        rec = ("reward", "cost") if narrow else REC
        eng.run_episode("train", "philox", episode=e, epsilon=0.6, record=rec)
        assert eng.last_kernel().startswith("episode_fast_kernel<") and "battery" in eng.last_kernel()
        out = ob.run_episode("train", rng="philox", episode=e, eps=0.6)
        got = eng.get_records(rec)
        if narrow:
            assert np.array_equal(got["reward"], out["reward"]) and np.array_equal(got["cost"], out["cost"]), e
        else:
            _cmp(out, got, ("narrow-alt", N, e))
        assert np.array_equal(eng.get_soc(), ob.soc), e
        assert np.array_equal(eng.episode_reward(), out["episode_reward"]), e
    assert np.array_equal(eng.get_q().reshape(ob.q.shape), ob.q)


def test_rccl_allreduce_world1_is_identity():
    from p2pmicrogrid_amd.engine import comm_unique_id
    eng, ob = _setup(16, 16, 1, 12, "f32", True, True, False)
    eng.comm_init(comm_unique_id(), 0, 1)
    eng.run_episode("train", "philox", episode=0, epsilon=0.5)
    ob.run_episode("train", rng="philox", episode=0, eps=0.5)
    before = eng.get_q_delta()
    eng.allreduce_q_delta()
    assert np.array_equal(eng.get_q_delta(), before)
    assert np.array_equal(before.reshape(-1, 3), ob.q_delta)
    eng.apply_q_delta()
    ob.apply_q_delta()
    assert np.array_equal(eng.get_q(dtype=np.float32).reshape(ob.q.shape), ob.q)


@pytest.mark.parametrize("q_dtype,battery,R", [("f32", True, 1), ("f64", False, 1), ("f32", True, 0)])
def test_sq16_kernel_matches_general_kernel(q_dtype, battery, R):
    """configs[2] runs on episode_sq16_kernel; the general episode_kernel (checked against the
    oracle above) must give the same records, deltas, SoC and temperatures on a ragged batch."""
    S, T = 701, 40  # 701: a partial last wave and a partial last workgroup
    a, _ = _setup(S, 16, R, T, q_dtype, True, battery, False, seed=3)
    b, _ = _setup(S, 16, R, T, q_dtype, True, battery, False, seed=3)
    dt = np.float64 if q_dtype == "f64" else np.float32
    for e in range(3):
        philox = "prepass" if e == 1 else "auto"
        a.run_episode("train", "philox", episode=e, epsilon=0.5, record=REC, philox=philox, reset_sigma=0.3)
        b.run_episode("train", "philox", episode=e, epsilon=0.5, record=REC, philox=philox, reset_sigma=0.3,
                      kernel="general")
        assert "sq16" in a.last_kernel() and "sq16" not in b.last_kernel()
        ra, rb = a.get_records(REC), b.get_records(REC)
        for k in REC:
            assert np.array_equal(ra[k], rb[k]), (e, k)
        assert np.array_equal(a.get_q_delta(), b.get_q_delta()), e
        assert np.array_equal(a.episode_reward(), b.episode_reward()), e
        if battery:
            assert np.array_equal(a.get_soc(), b.get_soc()), e
        for x, y in zip(a.get_temperatures(), b.get_temperatures()):
            assert np.array_equal(x, y), e
        a.apply_q_delta()
        b.apply_q_delta()
        assert np.array_equal(a.get_q(dtype=dt), b.get_q(dtype=dt))
    a.run_episode("greedy", record=REC)
    b.run_episode("greedy", record=REC, kernel="general")
    ra, rb = a.get_records(REC), b.get_records(REC)
    for k in REC:
        assert np.array_equal(ra[k], rb[k]), ("greedy", k)
    # only reward + cost requested: sq16 writes the narrow float2 record rows
    a.run_episode("train", "philox", episode=5, epsilon=0.5, record=("reward", "cost"))
    b.run_episode("train", "philox", episode=5, epsilon=0.5, record=("reward", "cost"), kernel="general")
    for k in ("reward", "cost"):
        assert np.array_equal(a.get_record(k), b.get_record(k)), ("narrow", k)
    assert np.array_equal(a.get_q_delta(), b.get_q_delta())


@pytest.mark.parametrize("N,shared", [(4, False), (16, True)])
def test_battery_outside_verified_domain_takes_checked_rule(N, shared):
    """The fast / sq16 kernels drop the battery rule's per-lane range tests only inside the operand
    domain the runtime verifies (p2pmg_set_battery / set_profiles); one tiny battery (2^-30 J, below
    the verified capacities) selects the range-checked variant, which still equals the oracle."""
    S, R, T = 24, 1, 32
    q_dtype = "f32" if shared else "f64"
    eng, ob = _setup(S, N, R, T, q_dtype, shared, True, False, seed=5)
    for e in range(3):
        if e == 1:  # the same community from here on with one tiny battery
            cap = np.full((S, N), 10 * 3.6e6)
            cap[0, 0] = 2.0 ** -30
            eng.set_battery(cap, 0.1, 0.9, 0.9, soc0=eng.get_soc())
            ob.battery_capacity = cap.copy()
        eng.run_episode("train", "philox", episode=e, epsilon=0.6, record=REC)
        assert ("range-checked" in eng.last_kernel()) == (e >= 1), eng.last_kernel()
        out = ob.run_episode("train", rng="philox", episode=e, eps=0.6)
        _cmp(out, eng.get_records(REC), ("checked", N, e))
        assert np.array_equal(eng.get_soc(), ob.soc), e
        if shared:
            eng.apply_q_delta()
            ob.apply_q_delta()
