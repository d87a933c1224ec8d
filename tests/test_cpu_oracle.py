"""CPU tests: the oracle pinned against vectors produced by the reference's own code
(tests/golden/make_golden.py), plus the Philox known answers.  No GPU needed."""
import warnings

import numpy as np
import pytest

from conftest import load_golden
from oracle import philox
from oracle.restatement import (GREEDY, OracleBatch, OracleParams, assign_powers, divide_power,
                                reference_replay_codes, state_index, temperature_step)

LOOPS = ["loop_thesis_T96", "loop_thesis_T672", "loop_homo_T96", "loop_n5_r2_T96"]


def test_philox_random123_known_answers():
    kat = [((0, 0, 0, 0, 0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 6, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for args, want in kat:
        got = tuple(int(x) for x in philox.philox4x32_10(*args))
        assert got == want


def test_philox_draws_are_uniform_and_deterministic():
    u, a = philox.decision_draws(42, 3, np.arange(100000), 5, 1, 1)
    u2, a2 = philox.decision_draws(42, 3, np.arange(100000), 5, 1, 1)
    assert np.array_equal(u, u2) and np.array_equal(a, a2)
    assert 0.49 < u.mean() < 0.51 and set(np.unique(a)) == {0, 1, 2}
    assert abs((a == 0).mean() - 1 / 3) < 0.01
    # one word per round: the action of an exploring draw (u < eps) is w % 3 of the same word, uniform
    # over the three actions for any epsilon, and the four rounds of a block are distinct words
    for eps in (0.1, 0.5, 0.81):
        ex = u < eps
        for k in range(3):
            assert abs((a[ex] == k).mean() - 1 / 3) < 0.02
    w = [philox.decision_draws(42, 3, np.arange(1000), t, r, 1)[0] for t in (4, 5) for r in (0, 1)]
    assert len({tuple(x[:8]) for x in w}) == 4
    ti, tm = philox.t0_draws(42, 0, np.arange(20000))
    assert abs(ti.mean() - 21.0) < 0.01 and abs(ti.std() - 0.3) < 0.01 and abs(tm.std() - 0.3) < 0.01


def test_state_index_matches_reference_qactor():
    d = load_golden("qactor")
    obs = d["obs"]
    p = OracleParams()
    idx = np.stack([state_index(obs[:, 0], p.n_time, "time"), state_index(obs[:, 1], p.n_temp, "temp"),
                    state_index(obs[:, 2], p.n_bal, "plain"), state_index(obs[:, 3], p.n_p2p, "plain")], axis=1)
    assert np.array_equal(idx, d["idx"])


def test_temperature_step_matches_reference_simulation():
    d = load_golden("heating")
    a, b = temperature_step(d["tout"], d["tin"], d["tm"], d["hp"])
    assert np.array_equal(a, d["out_in"]) and np.array_equal(b, d["out_m"])
    for T in (96, 672):
        hist = d[f"roll{T}_hist"]
        ti, tm = hist[0, 0], hist[0, 1]
        for t in range(T):
            ti, tm = temperature_step(d[f"roll{T}_tout"][t], ti, tm, d[f"roll{T}_hp"][t])
            assert ti == hist[t + 1, 0] and tm == hist[t + 1, 1]


def test_qactor_sequence_matches_reference():
    """epsilon-greedy + TD (rl.py:100-132) under np.random.seed(42), restated with oracle pieces."""
    d = load_golden("qactor")
    p = OracleParams()
    q = np.zeros((20, 20, 20, 20, 3))
    rs = np.random.RandomState(42)

    def ix(o):
        return (int(state_index(o[0], 20, "time")), int(state_index(o[1], 20, "temp")),
                int(state_index(o[2], 20, "plain")), int(state_index(o[3], 20, "plain")))
    for k in range(len(d["acts"])):
        eps = d["eps"][k]
        s = ix(d["s_obs"][k])
        if rs.rand() < eps:
            a, qv = rs.choice(3), 0.0
        else:
            a = int(q[s].argmax())
            qv = q[s][a]
        assert a == d["acts"][k] and qv == d["qs"][k]
        ns = ix(d["n_obs"][k])
        qmax = q[ns].max()
        q[s + (a,)] = q[s + (a,)] + p.alpha * ((float(d["rew"][k]) + p.gamma * qmax) - q[s + (a,)])
    nz = np.argwhere(q != 0)
    assert np.array_equal(nz, d["q_nz_idx"])
    assert np.array_equal(q[tuple(nz.T)], d["q_nz_val"])


@pytest.mark.parametrize("name", LOOPS)
def test_oracle_reproduces_reference_driven_loop(name):
    """Full community loop: the hybrid harness drove the reference's QActor and
    temperature_simulation; the vectorised restatement must match it bit-for-bit."""
    d = load_golden(name)
    N, R, E = int(d["N"]), int(d["R"]), int(d["E"])
    ob = OracleBatch(S=1, N=N, R=R, load_w=d["load_w"][None], pv_w=d["pv_w"][None], max_in=d["max_in"][None],
                     env_time=d["env_time"][None], env_tout=d["env_tout"][None],
                     price_table=(d["buy"], d["inj"], d["p2pp"]))
    for e in range(E):
        ob.t_in, ob.t_m = d["t_in0"][e][None].copy(), d["t_m0"][e][None].copy()
        out = ob.run_episode("train", codes=d["codes"][e][:, :, None, :], eps=d["eps"][e])
        for k in ("grid", "p2p", "cost", "reward", "t_in", "t_m", "hp"):
            assert np.array_equal(out[k][:, 0], d[f"train_{k}"][e]), (name, e, k)
        assert np.array_equal(out["action"][:, :, 0], d["train_action"][e])
        assert np.array_equal(out["idx"][:, :, 0], d["train_idx"][e])
        qi, qv = d[f"q_idx_{e}"], d[f"q_val_{e}"]
        tabs = np.stack([ob.q_table(i) for i in range(N)])
        assert np.count_nonzero(tabs) == len(qv) and np.array_equal(tabs[tuple(qi.T)], qv)
    ev = OracleBatch(S=1, N=N, R=R, load_w=d["eval_load_w"][None], pv_w=d["eval_pv_w"][None],
                     max_in=d["max_in"][None], env_time=d["eval_env_time"][None],
                     env_tout=d["eval_env_tout"][None], price_table=(d["eval_buy"], d["eval_inj"], d["eval_p2pp"]))
    ev.q = ob.q
    ev.t_in, ev.t_m = d["eval_t_in0"][None].copy(), d["eval_t_m0"][None].copy()
    out = ev.run_episode("greedy")
    for k in ("grid", "p2p", "cost", "reward", "t_in", "hp"):
        assert np.array_equal(out[k][:, 0], d[f"eval_{k}"]), (name, "eval", k)
    assert np.array_equal(out["action"][:, :, 0], d["eval_action"])


def test_reference_quirks_divide_power_and_market():
    """opposite-sign agents split evenly incl. the diagonal; same-sign
    agents send everything to each other and nothing clears."""
    F = np.float32
    # round 1 of N=2 after round 0 produced P = [[500, 500], [-1000, -1000]] (even split)
    P0 = np.array([[500, 500], [-1000, -1000]], F)
    P0[[0, 1], [0, 1]] = 0
    rows = np.stack([divide_power(F(1000), -P0[:, 0], 2), divide_power(F(-2000), -P0[:, 1], 2)])
    assert np.array_equal(rows, np.array([[500, 500], [-1000, -1000]], F))
    g, pp = assign_powers(rows)
    assert np.array_equal(pp, np.array([500, -500], F)) and np.array_equal(g, np.array([500, -1500], F))
    rows = np.stack([divide_power(F(1000), np.array([0, -500], F), 2),
                     divide_power(F(500), np.array([-1000, 0], F), 2)])
    assert np.array_equal(rows, np.array([[0, 1000], [500, 0]], F))
    g, pp = assign_powers(rows)
    assert np.array_equal(pp, np.zeros(2, F)) and np.array_equal(g, np.array([1000, 500], F))


def test_reference_replay_codes_consumption_order():
    rs = np.random.RandomState(42)
    codes = reference_replay_codes(rs, 3, 1, 2, 0.5)
    rs2 = np.random.RandomState(42)
    want = []
    for _ in range(3 * 2 * 2):
        want.append(rs2.choice(3) if rs2.rand() < 0.5 else GREEDY)
    assert np.array_equal(codes.ravel(), np.array(want, np.uint8))


def test_battery_rule_matches_reference_storage():
    """oracle.battery_rule vs the reference's BatteryStorage driven by the agent.py:138-153 rule."""
    from oracle.restatement import battery_rule
    d = load_golden("battery")
    soc = np.array(float(d["soc0"]))
    for k, b in enumerate(d["bal"]):
        ob, soc = battery_rule(np.array(b), soc, float(d["capacity"]), float(d["min_soc"]), float(d["max_soc"]),
                               np.sqrt(float(d["efficiency"])))
        assert ob == d["out_bal"][k] and soc == d["soc"][k], k
    assert np.all(d["soc"] >= 0.1 - 1e-12) and np.all(d["soc"] <= 0.9 + 1e-12)


def test_rule_community_market_broadcast_quirk():
    """RuleAgent's (1,) outputs stack to an (N, 1) P; community.py:45-54 broadcasts it against its
    transpose (worked by hand from TF's broadcasting rules): p_grid_i = sum_j (P_i - ex_ij)."""
    from oracle.restatement import rule_assign_powers
    g, pp = rule_assign_powers(np.array([1000.0, -2000.0], np.float32))
    assert np.array_equal(pp, np.array([1000.0, -1000.0], np.float32))
    assert np.array_equal(g, np.array([1000.0, -3000.0], np.float32))  # (1000-0)+(1000-1000); (-2000+1000)+(-2000-0)
    g, pp = rule_assign_powers(np.array([[500.0], [-200.0]], np.float32).T)  # one scenario, N = 2
    assert np.array_equal(pp, np.array([[200.0, -200.0]], np.float32))
    g1, pp1 = rule_assign_powers(np.array([700.0], np.float32))  # N = 1: grid = P
    assert g1[0] == np.float32(700.0) and pp1[0] == 0


def test_rule_oracle_hysteresis():
    from oracle.restatement import OracleBatch
    from p2pmicrogrid_amd.dataset import scenario_batch
    S, N, T = 3, 2, 96
    inp = scenario_batch(S, N, T)
    ob = OracleBatch(S=S, N=N, R=0, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                     env_time=inp.time[None], env_tout=inp.t_out)
    ob.t_in = np.full((S, N), np.float32(19.5))
    ob.t_m = np.full((S, N), np.float32(19.5))
    out = ob.run_rule_episode(np.zeros((S, N), np.int64))
    assert out["on"][0].all() and out["hp"][0].max() == np.float32(3000.0)  # cold start: on
    on, tin = out["on"], out["t_in"]
    for t in range(1, T):  # hysteresis: switches only at the band edges
        sw_on = (on[t] == 1) & (on[t - 1] == 0)
        sw_off = (on[t] == 0) & (on[t - 1] == 1)
        assert (tin[t][sw_on] <= np.float32(20.0)).all() and (tin[t][sw_off] >= np.float32(22.0)).all()


def test_rule_community_api_only_runs():
    import pytest
    from p2pmicrogrid_amd.community import get_rule_based_community
    np.random.seed(42)
    com = get_rule_based_community(2, homogeneous=False)
    assert com._rounds == 0 and {type(a).__name__ for a in com.agents} == {"RuleAgent"}
    with pytest.raises(AttributeError):
        com.train_episode()


def test_small_epsilon_action_words_are_independent_and_uniform():
    """Below epsilon 2^-8 the explore actions come from the TAG_ACTION block: uniform
    and unrelated to the explore word; at larger epsilon the action is w % 3 of the explore word."""
    agents = np.arange(300000)
    u, a_big = philox.decision_draws(42, 3, agents, 5, 1, 1, eps=0.5)
    w = np.round(u * 4294967296.0).astype(np.uint64)
    assert np.array_equal(a_big, (w % np.uint64(3)).astype(np.int64))
    u2, a_small = philox.decision_draws(42, 3, agents, 5, 1, 1, eps=1e-9)
    assert np.array_equal(u, u2)  # the explore test itself does not change
    shares = np.bincount(a_small, minlength=3) / len(agents)
    assert np.all(np.abs(shares - 1 / 3) < 0.005), shares
    assert np.mean(a_small == a_big) < 0.36  # independent of the explore word (1/3 by chance)
    thr, all_ = philox.eps_threshold(2.0 ** -8)
    assert thr == 1 << 24 and not all_
