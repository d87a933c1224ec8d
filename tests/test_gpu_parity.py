"""GPU parity: the HIP path (libp2pmg.so via its C ABI) against the reference-generated golden
fixtures and the CPU restatement (oracle/).  Bit-exact for indices, actions and every f32/f64
value: the kernel and the oracle follow one op order (-ffp-contract=off).
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import philox
from oracle.restatement import OracleBatch, reference_replay_codes
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.engine import DeviceCommunityBatch, unpack_index

pytestmark = pytest.mark.gpu

LOOPS = ["loop_thesis_T96", "loop_thesis_T672", "loop_homo_T96", "loop_n5_r2_T96"]
REC = ["reward", "cost", "grid", "p2p", "t_in", "action", "index"]


def _engine_from_fixture(d, prefix=""):
    N, R = int(d["N"]), int(d["R"])
    T = d[f"{prefix}env_time"].shape[-1]
    eng = DeviceCommunityBatch(1, N, R, T)
    eng.set_env(d[f"{prefix}env_time"], d[f"{prefix}env_tout"], d[f"{prefix}buy"], d[f"{prefix}inj"],
                d[f"{prefix}p2pp"])
    eng.set_profiles(d[f"{prefix}load_w"][None], d[f"{prefix}pv_w"][None])
    eng.set_max_in(d["max_in"][None])
    return eng


def test_rc_step_matches_reference_temperature_simulation():
    d = load_golden("heating")
    eng = DeviceCommunityBatch(1, 1, 0, 1)
    a, b = eng.rc_step(d["tout"], d["tin"], d["tm"], d["hp"])
    assert np.array_equal(a, d["out_in"]) and np.array_equal(b, d["out_m"])
    for T in (96, 672):
        hist = d[f"roll{T}_hist"]
        ti, tm = hist[0, :1].copy(), hist[0, 1:2].copy()
        for t in range(T):
            ti, tm = eng.rc_step(d[f"roll{T}_tout"][t:t + 1], ti, tm, d[f"roll{T}_hp"][t:t + 1])
            assert ti[0] == hist[t + 1, 0] and tm[0] == hist[t + 1, 1], (T, t)


def test_state_indices_match_reference_qactor():
    d = load_golden("qactor")
    eng = DeviceCommunityBatch(1, 1, 0, 1)
    idx = eng.state_indices(d["obs"])
    assert np.array_equal(idx, d["idx"])


@pytest.mark.parametrize("name", LOOPS)
def test_training_replay_matches_reference_loop(name):
    """Replay mode: exploration replayed from the reference's own np.random consumption."""
    d = load_golden(name)
    N, R, E = int(d["N"]), int(d["R"]), int(d["E"])
    eng = _engine_from_fixture(d)
    for e in range(E):
        eng.set_temperatures(d["t_in0"][e][None], d["t_m0"][e][None])
        eng.set_replay_codes(d["codes"][e])
        eng.run_episode("train", "replay", episode=e, epsilon=float(d["eps"][e]), record=REC)
        rec = eng.get_records(REC)
        for k, g in (("reward", "reward"), ("cost", "cost"), ("grid", "grid"), ("p2p", "p2p"), ("t_in", "t_in")):
            assert np.array_equal(rec[k][:, 0], d[f"train_{g}"][e]), (name, e, k)
        assert np.array_equal(rec["action"][:, :, 0], d["train_action"][e]), (name, e)
        assert np.array_equal(unpack_index(rec["index"][:, :, 0]), d["train_idx"][e]), (name, e)
        q = eng.get_q()
        qi, qv = d[f"q_idx_{e}"], d[f"q_val_{e}"]
        assert np.count_nonzero(q) == len(qv)
        assert np.array_equal(q[tuple(qi.T)], qv), (name, e)
    # greedy evaluation (CommunityMicrogrid.run) with the trained tables
    q = eng.get_q()
    ev = _engine_from_fixture(d, prefix="eval_")
    ev.set_q(q)
    ev.set_temperatures(d["eval_t_in0"][None], d["eval_t_m0"][None])
    ev.run_episode("greedy", record=REC)
    rec = ev.get_records(REC)
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert np.array_equal(rec[k][:, 0], d[f"eval_{k}"]), (name, "eval", k)
    assert np.array_equal(rec["action"][:, :, 0], d["eval_action"])
    assert np.array_equal(unpack_index(rec["index"][:, :, 0]), d["eval_idx"])


def _oracle_for(inp, N, R, q_dtype="f64"):
    S = inp.load_w.shape[0]
    return OracleBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                       env_time=inp.time[None], env_tout=inp.t_out, q_dtype=q_dtype)


def _device_for(inp, N, R, q_dtype="f64", scenario_offset=0):
    S, T = inp.load_w.shape[0], inp.load_w.shape[-1]
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype, scenario_offset=scenario_offset)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    return eng


def _compare(out, rec, tag):
    for k in ("reward", "cost", "grid", "p2p"):
        assert np.array_equal(rec[k], out[k]), (tag, k)
    assert np.array_equal(rec["t_in"], out["t_in"]), tag
    assert np.array_equal(rec["action"], out["action"].astype(np.uint8)), tag
    assert np.array_equal(unpack_index(rec["index"]), out["idx"]), tag


CASES = [(2, 1, 96, "f64"), (3, 2, 48, "f64"), (5, 0, 40, "f64"), (8, 1, 24, "f64"), (16, 1, 12, "f64"),
         (1, 1, 30, "f64"), (2, 1, 96, "f32"), (4, 3, 20, "f32"), (2, 7, 10, "f64"), (6, 4, 10, "f32"),
         (7, 2, 16, "f64"), (3, 3, 12, "f32")]
# kernel choice x scenarios per wave: the fast kernel (auto), partially filled fast waves, the general
# kernel, the general kernel's LDS-tile form (the form every N outside {1..8, 16} runs) at these sizes
KERNELS = [("auto", 0), ("auto", 5), ("general", 0), ("tile", 0)]


@pytest.mark.parametrize("kernel,spw", KERNELS)
@pytest.mark.parametrize("N,R,T,q_dtype", CASES)
def test_replay_batch_matches_oracle(N, R, T, q_dtype, kernel, spw):
    """Many scenarios, each with its own RandomState(42 + s) replay stream, several episodes."""
    S = 64
    inp = scenario_batch(S, N, T, seed=7)
    ob = _oracle_for(inp, N, R, q_dtype)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R, q_dtype)
    rss = [np.random.RandomState(42 + s) for s in range(S)]
    for e, eps in enumerate((0.81, 0.729, 0.2)):
        codes = np.stack([reference_replay_codes(rs, T, R, N, eps) for rs in rss], axis=2)  # [T,R+1,S,N]
        eng.set_replay_codes(codes)
        eng.run_episode("train", "replay", episode=e, epsilon=eps, record=REC, kernel=kernel, scen_per_wave=spw)
        out = ob.run_episode("train", codes=codes, eps=eps)
        _compare(out, eng.get_records(REC), (N, R, T, q_dtype, e))
        assert np.array_equal(eng.episode_reward(), out["episode_reward"])
        a, b = eng.get_temperatures()
        assert np.array_equal(a, out["t_in_final"]) and np.array_equal(b, out["t_m_final"])
    q = eng.get_q(dtype=np.float64 if q_dtype == "f64" else np.float32)
    assert np.array_equal(q.reshape(S * N, -1, 3), ob.q)
    # greedy pass with the learned tables
    eng.run_episode("greedy", record=REC, kernel=kernel, scen_per_wave=spw)
    _compare(ob.run_episode("greedy"), eng.get_records(REC), "greedy")


@pytest.mark.parametrize("q_dtype", ["f64", "f32"])
@pytest.mark.parametrize("R", [0, 1, 2])
@pytest.mark.parametrize("N", [9, 12, 15, 17, 24, 32, 64])
def test_any_community_size_matches_oracle(N, R, q_dtype):
    """Community sizes outside the compiled-in {1..8, 16} (get_community takes any n_agents,
    community.py:198-204): the general kernel's LDS-tile form (P in two LDS tiles, sequential
    j = 0..N-1 sums) against the oracle, replayed reference streams, 3 episodes + a greedy day."""
    S, T = max(4, 256 // N), 12
    inp = scenario_batch(S, N, T, seed=7)
    ob = _oracle_for(inp, N, R, q_dtype)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R, q_dtype)
    rss = [np.random.RandomState(42 + s) for s in range(S)]
    for e, eps in enumerate((0.81, 0.729, 0.2)):
        codes = np.stack([reference_replay_codes(rs, T, R, N, eps) for rs in rss], axis=2)
        eng.set_replay_codes(codes)
        eng.run_episode("train", "replay", episode=e, epsilon=eps, record=REC)
        assert eng.last_kernel().startswith(f"episode_kernel<{N},tile"), eng.last_kernel()
        out = ob.run_episode("train", codes=codes, eps=eps)
        _compare(out, eng.get_records(REC), (N, R, q_dtype, e))
        assert np.array_equal(eng.episode_reward(), out["episode_reward"])
        a, b = eng.get_temperatures()
        assert np.array_equal(a, out["t_in_final"]) and np.array_equal(b, out["t_m_final"])
    q = eng.get_q(dtype=np.float64 if q_dtype == "f64" else np.float32)
    assert np.array_equal(q.reshape(S * N, -1, 3), ob.q)
    eng.run_episode("greedy", record=REC)
    _compare(ob.run_episode("greedy"), eng.get_records(REC), "greedy")
    eng.close()


@pytest.mark.parametrize("N,R,kernel,placement", [(3, 9, "general", "prepass"), (3, 9, "general", "inkernel"),
                                                  (2, 8, "auto", "prepass"), (12, 11, "auto", "inkernel"),
                                                  (5, 12, "tile", "prepass"),
                                                  # tens of rounds: replay words 0..10, Philox blocks 0..10
                                                  (4, 40, "auto", "inkernel"), (17, 33, "auto", "prepass"),
                                                  # the bound: R + 1 = 4096 (include/p2pmg.h)
                                                  (2, 4095, "auto", "inkernel")])
def test_more_than_eight_rounds_match_oracle(N, R, kernel, placement):
    """R + 1 > 8 negotiation rounds (community.py:75 runs any `rounds`): rounds 8 and up take their
    exploration codes one at a time (replay words 2.. and Philox words k = t (R + 1) + r), in the
    register and tile forms, Philox pre-pass and in-kernel draws, against the oracle."""
    S, T = (24, 10) if R < 1000 else (4, 4)  # the oracle's per-round loop bounds the 4096-round case
    inp = scenario_batch(S, N, T, seed=29)
    ob = _oracle_for(inp, N, R)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R)
    rss = [np.random.RandomState(42 + s) for s in range(S)]
    for e, eps in enumerate((0.81, 0.5)):
        eng.run_episode("train", "philox", episode=e, epsilon=eps, record=REC, philox=placement, kernel=kernel)
        _compare(ob.run_episode("train", rng="philox", seed=42, episode=e, eps=eps), eng.get_records(REC), (N, R, e))
    codes = np.stack([reference_replay_codes(rs, T, R, N, 0.6) for rs in rss], axis=2)
    eng.set_replay_codes(codes)
    eng.run_episode("train", "replay", episode=2, epsilon=0.6, record=REC, kernel=kernel)
    _compare(ob.run_episode("train", codes=codes, eps=0.6), eng.get_records(REC), (N, R, "replay"))
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)
    eng.close()


@pytest.mark.parametrize("placement", ["prepass", "inkernel"])
def test_philox_matches_oracle_and_t0(placement):
    S, N, R, T = 256, 2, 1, 96
    inp = scenario_batch(S, N, T, seed=3)
    ob = _oracle_for(inp, N, R)
    eng = _device_for(inp, N, R)
    for e in range(3):
        eng.reset_temperatures_philox(e, 0.3)
        t_in, t_m = philox.t0_draws(42, e, np.arange(S * N))
        a, b = eng.get_temperatures()
        assert np.array_equal(a.ravel(), t_in) and np.array_equal(b.ravel(), t_m)
        ob.t_in, ob.t_m = t_in.reshape(S, N), t_m.reshape(S, N)
        eps = 0.81 * 0.9 ** e
        eng.run_episode("train", "philox", episode=e, epsilon=eps, record=REC, philox=placement)
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=eps)
        _compare(out, eng.get_records(REC), e)
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)


@pytest.mark.parametrize("placement,kernel", [("prepass", "auto"), ("inkernel", "auto"), ("inkernel", "general")])
def test_small_epsilon_actions_from_their_own_block(placement, kernel):
    """epsilon below 2^-8 (threshold < 2^24): an exploring lane's action comes from the TAG_ACTION
    Philox block, independent of its explore test (w % 3 of a w below a small threshold
    is biased).  Fast (pre-pass and in-kernel draws) and general kernels against the oracle."""
    S, N, R, T = 512, 2, 1, 96
    inp = scenario_batch(S, N, T, seed=13)
    ob = _oracle_for(inp, N, R)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R)
    explored = 0
    for e, eps in enumerate((0.003, 0.0009)):
        eng.run_episode("train", "philox", episode=e, epsilon=eps, record=REC, philox=placement, kernel=kernel)
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=eps)
        _compare(out, eng.get_records(REC), (placement, kernel, e))
        for t in range(T):
            for r in range(R + 1):
                u, _ = philox.decision_draws(42, e, np.arange(S * N), t, r, R, eps=eps)
                explored += int((u < eps).sum())
    assert explored > 100  # the small-epsilon branch did draw actions
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)


def test_speculative_prepass_next_epsilon():
    """next_epsilon: the launch writes episode e+1's Philox codes at the caller's next epsilon
    (the decay schedule, community.py:279-286).  Right guesses (hits), wrong guesses (a recompute)
    and no guess must all give the oracle's trajectory."""
    S, N, R, T = 128, 2, 1, 48
    inp = scenario_batch(S, N, T, seed=9)
    ob = _oracle_for(inp, N, R)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R)
    eps = [0.81, 0.729, 0.729, 0.6561, 0.6561, 0.5, 0.0]
    # guess[e] is launch e's guess of eps[e + 1]: right (launch e + 1 hits) or wrong (it misses);
    # None = "the same epsilon"; 0.0 is a real guess (P2PMG_FLAG_NEXT_EPSILON), not "no guess"
    guess = [0.729, 0.729, 0.3, None, 0.6561, 0.0, None]
    expect_hit = [False, True, True, False, True, False, True]
    for e in range(len(eps)):
        h0, _ = eng.prepass_stats()
        eng.run_episode("train", "philox", episode=e, epsilon=eps[e], record=REC, next_epsilon=guess[e])
        h1, _ = eng.prepass_stats()
        assert (h1 - h0 == 1) == expect_hit[e], f"launch {e}: pre-pass hit {h1 - h0 == 1}, expected {expect_hit[e]}"
        _compare(ob.run_episode("train", rng="philox", seed=42, episode=e, eps=eps[e]), eng.get_records(REC), e)
    assert eng.prepass_stats() == (4, 3)
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)


def test_full_size_config2_sampled_against_oracle():
    """configs[1] at full size (4096 scenarios x thesis community): the whole batch runs on the
    device; 48 sampled scenarios are re-run by the oracle with the same global Philox ids, and
    size-independent properties are checked over all scenarios."""
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    eng = _device_for(inp, N, R)
    rng = np.random.RandomState(0)
    pick = np.sort(rng.choice(S, 48, replace=False))
    sub = scenario_batch(S, N, T)
    for k in ("load_w", "pv_w", "max_in", "t_in0", "t_m0", "t_out"):
        setattr(sub, k, getattr(sub, k)[pick])
    ob = _oracle_for(sub, N, R)
    ob.t_in, ob.t_m = sub.t_in0.copy(), sub.t_m0.copy()
    gids = (pick[:, None] * N + np.arange(N)[None, :])
    for e in range(2):
        eng.run_episode("train", "philox", episode=e, epsilon=0.81, record=REC)
        rec = eng.get_records(REC)
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=0.81, agent_ids=gids)
        sl = {k: (v[:, :, pick] if k in ("action", "index") else v[:, pick]) for k, v in rec.items()}
        _compare(out, sl, e)
        # properties over ALL scenarios: P2P exchange is antisymmetric (sum_i p2p_i == 0 for N = 2)
        assert np.all(rec["p2p"].sum(axis=-1) == 0)
        assert np.all(np.isfinite(rec["reward"])) and np.all(rec["action"] <= 2)
    q = eng.get_q(first=0, count=S * N)
    sel = q.reshape(S, N, -1)[pick].reshape(-1, q[0].size)
    assert np.array_equal(sel, ob.q.reshape(len(pick) * N, -1))


def test_edge_cases_eps_extremes_and_t1():
    for eps in (0.0, 1.0):
        S, N, R, T = 32, 2, 1, 24
        inp = scenario_batch(S, N, T, seed=11)
        ob = _oracle_for(inp, N, R)
        ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
        eng = _device_for(inp, N, R)
        eng.run_episode("train", "philox", episode=0, epsilon=eps, record=REC)
        _compare(ob.run_episode("train", rng="philox", eps=eps), eng.get_records(REC), eps)
    # T = 1: the next-step pair wraps onto itself (np.roll(-1) of a single row)
    inp = scenario_batch(8, 2, 1, seed=5)
    ob = _oracle_for(inp, 2, 1)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, 2, 1)
    for e in range(3):
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=REC)
        _compare(ob.run_episode("train", rng="philox", episode=e, eps=0.5), eng.get_records(REC), "T1")


def test_q_roundtrip_and_sharded_offsets():
    S, N, R, T = 40, 2, 1, 16
    inp = scenario_batch(S, N, T)
    eng = _device_for(inp, N, R)
    tab = np.random.RandomState(1).randn(S * N, 20, 20, 20, 20, 3)
    eng.set_q(tab)
    assert np.array_equal(eng.get_q(), tab)
    assert np.array_equal(eng.get_q(first=7, count=5), tab[7:12])
    # two shards with scenario offsets reproduce the unsharded batch (Philox ids are global)
    eng.zero_q()
    eng.run_episode("train", "philox", episode=0, epsilon=0.6, record=REC)
    full = eng.get_records(REC)
    parts = []
    for lo, hi in ((0, 17), (17, 40)):
        sub = scenario_batch(hi - lo, N, T, first_scenario=lo)
        e2 = _device_for(sub, N, R, scenario_offset=lo)
        e2.run_episode("train", "philox", episode=0, epsilon=0.6, record=REC)
        parts.append(e2.get_records(REC))
    for k in REC:
        ax = 2 if k in ("action", "index") else 1
        assert np.array_equal(np.concatenate([p[k] for p in parts], axis=ax), full[k]), k


@pytest.mark.parametrize("kernel", ["auto", "general"])
def test_unrecorded_episodes_match_oracle(kernel):
    """No records requested (the fast kernel's stores all go to its dummy slots except the TD
    updates): Q-tables, episode rewards and final temperatures still match the oracle."""
    S, N, R, T = 96, 3, 1, 48
    inp = scenario_batch(S, N, T, seed=21)
    ob = _oracle_for(inp, N, R)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R)
    for e in range(3):
        eng.run_episode("train", "philox", episode=e, epsilon=0.6, kernel=kernel)
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=0.6)
        assert np.array_equal(eng.episode_reward(), out["episode_reward"]), e
        a, b = eng.get_temperatures()
        assert np.array_equal(a, out["t_in_final"]) and np.array_equal(b, out["t_m_final"]), e
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)
    eng.run_episode("greedy", kernel=kernel)
    assert np.array_equal(eng.episode_reward(), ob.run_episode("greedy")["episode_reward"])


@pytest.mark.parametrize("kernel", ["auto", "general"])
def test_fused_t0_reset_equals_separate_reset(kernel):
    """reset_sigma fuses agent.reset() into the episode: same temperatures, rewards and tables as
    an episode followed by reset_temperatures_philox(episode + 1), over back-to-back episodes
    (which also exercises the double-buffered pre-pass of the fast path)."""
    S, N, R, T = 64, 2, 1, 40
    inp = scenario_batch(S, N, T, seed=13)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    for e in range(5):
        a.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward",), kernel=kernel, reset_sigma=0.3)
        b.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward",), kernel=kernel)
        b.reset_temperatures_philox(e + 1, 0.3)
    for x, y in zip(a.get_temperatures(), b.get_temperatures()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.get_record("reward"), b.get_record("reward"))
    assert np.array_equal(a.episode_reward(), b.episode_reward())
    assert np.array_equal(a.get_q(), b.get_q())


@pytest.mark.parametrize("N", [2, 4])
def test_narrow_reward_cost_records_match_oracle(N):
    """Only {reward, cost} requested: the fast kernel writes 8-B record rows instead of 32-B
    FastRec rows.  Alternating narrow and full requests over back-to-back episodes, every
    returned record still equals the oracle's."""
    S, R, T = 80, 1, 48
    inp = scenario_batch(S, N, T, seed=17)
    ob = _oracle_for(inp, N, R)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R)
    for e in range(4):
        narrow = e % 2 == 0
        rec = ("reward", "cost") if narrow else REC
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=rec)
        assert eng.last_kernel().startswith("episode_fast_kernel<")
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=0.5)
        got = eng.get_records(rec)
        if not narrow:
            _compare(out, got, e)
        else:
            assert np.array_equal(got["reward"], out["reward"]) and np.array_equal(got["cost"], out["cost"]), e
        assert np.array_equal(eng.episode_reward(), out["episode_reward"]), e
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)


@pytest.mark.parametrize("dims,fast", [((40, 40, 40, 40), False), ((30, 20, 20, 30), True)])
def test_non_default_state_dims_match_oracle(dims, fast):
    """Other Q-table sizes (agent.py:258-261's 20 x 20 x 20 x 20 as parameters).  The fast kernel
    addresses a wave's rows as 32-bit offsets from its first table, so it only takes tables whose
    64-lane span fits 4 GiB (40^4 states x 32 B x 64 does not: the general kernel runs); either way
    records and tables equal the oracle's."""
    from oracle.restatement import OracleParams
    S, N, R, T = 4, 2, 1, 24
    nt, nT, nb, npp = dims
    inp = scenario_batch(S, N, T, seed=23)
    ob = OracleBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in, env_time=inp.time[None],
                     env_tout=inp.t_out, params=OracleParams(n_time=nt, n_temp=nT, n_bal=nb, n_p2p=npp))
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = DeviceCommunityBatch(S, N, R, T, n_time_states=nt, n_temp_states=nT, n_balance_states=nb,
                               n_p2p_states=npp)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    for e in range(2):
        eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=REC)
        assert eng.last_kernel().startswith("episode_fast_kernel<") == fast, eng.last_kernel()
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=0.5)
        _compare(out, eng.get_records(REC), ("dims", dims, e))
        assert np.array_equal(eng.episode_reward(), out["episode_reward"]), e
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)
    eng.close()


def test_timing_period_samples_launches_only():
    """set_timing_period(k): only every k-th episode launch carries timing events; results are
    the same as with every launch timed."""
    S, N, R, T = 32, 2, 1, 24
    inp = scenario_batch(S, N, T, seed=5)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    a.set_timing_period(3)
    for e in range(7):
        for eng in (a, b):
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=("reward", "cost"), reset_sigma=0.3)
    assert len(a.kernel_times()) == 3 and len(b.kernel_times()) == 7
    assert all(t > 0 for t in a.kernel_times())
    assert np.array_equal(a.get_record("reward"), b.get_record("reward"))
    assert np.array_equal(a.get_q(), b.get_q())
