"""The reference-shaped object API end to end on the GPU: a community built through the public
constructors with the global np.random seeded as community.py:30 does reproduces the
reference-driven fixture (exploration stream, T0 resets, rewards, Q-tables, greedy run)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle.restatement import OracleBatch

pytestmark = pytest.mark.gpu


def _community_from_fixture(d):
    from p2pmicrogrid_amd import setup
    from p2pmicrogrid_amd.agent import Agent, QAgent
    from p2pmicrogrid_amd.community import CommunityMicrogrid
    from p2pmicrogrid_amd.dataset import ProfileDataset
    from p2pmicrogrid_amd.environment import env
    from p2pmicrogrid_amd.heating import HeatPump, HPHeating
    from p2pmicrogrid_amd.production import PV, Prosumer
    from p2pmicrogrid_amd.rng import ReferenceRNG
    from p2pmicrogrid_amd.storage import NoStorage
    N, R, T = int(d["N"]), int(d["R"]), int(d["T"])
    setup.homogeneous = bool(d["homogeneous"])
    np.random.seed(42)
    rng = ReferenceRNG()
    lr, pr = rng.community_ratings(N, setup.homogeneous)
    assert np.array_equal(lr, d["load_ratings"]) and np.array_equal(pr, d["pv_ratings"])
    ds = lambda x: ProfileDataset(np.asarray(x, np.float32), np.roll(np.asarray(x, np.float32), -1, 0))  # noqa: E731
    Agent.reset_ids()
    agents = [QAgent(ds(d["load_w"][i]), Prosumer(PV(pr[i] * 1e3, ds(d["pv_w"][i]))), NoStorage(),
                     HPHeating(HeatPump(3.0, 3e3, 0.0), 21.0), max_in=max(lr[i], pr[i]) * 1.1 * 1e3,
                     max_out=-(max(lr[i], pr[i]) + 1.1e3)) for i in range(N)]
    env.setup(ds(np.stack([d["env_time"], d["env_tout"]], axis=1)))
    return CommunityMicrogrid(list(range(T)), agents, R), env


@pytest.mark.parametrize("name", ["loop_thesis_T96", "loop_n5_r2_T96", "loop_homo_T96"])
def test_object_api_reproduces_reference_driven_training(name):
    from p2pmicrogrid_amd import setup
    from p2pmicrogrid_amd.dataset import ProfileDataset
    from p2pmicrogrid_amd.engine import price_table
    d = load_golden(name)
    N, E = int(d["N"]), int(d["E"])
    try:
        com, env = _community_from_fixture(d)
        same_prices = all(np.array_equal(a, b) for a, b in zip(price_table(d["env_time"]),
                                                               (d["buy"], d["inj"], d["p2pp"])))
        if not same_prices:
            pytest.skip("this host's numpy f32 sin differs from the fixture host's (price table input)")
        for e in range(E):
            assert np.array_equal([a.heating.temperature[0] for a in com.agents], d["t_in0"][e])
            assert np.array_equal([a.heating.building_mass_temperature[0] for a in com.agents], d["t_m0"][e])
            reward, loss = com.train_episode()
            assert loss == 0.0
            assert np.array_equal(com.last_rewards, d["train_reward"][e])
            tabs = np.stack([a.actor.q_table for a in com.agents])
            qi, qv = d[f"q_idx_{e}"], d[f"q_val_{e}"]
            assert np.count_nonzero(tabs) == len(qv) and np.array_equal(tabs[tuple(qi.T)], qv)
            want = (d["train_hp"][e] / 3e3)
            assert np.array_equal(com.decisions[:, -1, :] / 3e3, want)
            if e % 50 == 0:
                for a in com.agents:
                    a.actor.decay_exploration()
        # greedy evaluation on the next day (CommunityMicrogrid.run), fresh start from the fixture's T0
        ds = lambda x: ProfileDataset(np.asarray(x, np.float32), np.roll(np.asarray(x, np.float32), -1, 0))  # noqa: E731
        env.setup(ds(np.stack([d["eval_env_time"], d["eval_env_tout"]], axis=1)))
        for i, a in enumerate(com.agents):
            a._load = ds(d["eval_load_w"][i])
            a.pv.pv.production = ds(d["eval_pv_w"][i])
            a.heating.set_state(d["eval_t_in0"][i], d["eval_t_m0"][i])
        power, cost = com.run()
        assert np.array_equal(cost, d["eval_cost"])
        assert np.array_equal(power, (d["eval_grid"] + d["eval_p2p"]).astype(np.float32))
    finally:
        setup.homogeneous = False


@pytest.mark.parametrize("n", [10, 24])
def test_get_community_any_size_trains_like_oracle(n):
    """get_community(QAgent, n, homogeneous=True) for community sizes outside {1..8, 16}
    (community.py:198-204 replicates agent_dfs[0] n times): train_episode replays the reference's
    np.random stream through the device (the general kernel's tile form) and equals the oracle fed
    the community's own inputs and the same stream: rewards, decisions, episode reward, tables."""
    from p2pmicrogrid_amd import community, setup
    from p2pmicrogrid_amd.agent import QAgent
    from p2pmicrogrid_amd.environment import env
    from oracle.restatement import reference_replay_codes
    setup.homogeneous = True  # HPHeating reads the module flag (heating.py:101,149)
    try:
        np.random.seed(42)
        com = community.get_community(QAgent, n, homogeneous=True)
        T, R = len(env), setup.rounds
        time_f, t_out = env.arrays()
        load = np.stack([a.load_series(T) for a in com.agents]).astype(np.float32)
        pv = np.stack([a.pv.series(T) for a in com.agents]).astype(np.float32)
        max_in = np.array([np.float32(a.max_in) for a in com.agents], np.float32)
        ob = OracleBatch(S=1, N=n, R=R, load_w=load[None], pv_w=pv[None], max_in=max_in[None],
                         env_time=np.asarray(time_f, np.float32)[None], env_tout=np.asarray(t_out, np.float32)[None])
        rs = np.random.RandomState(42)  # homogeneous: nothing drawn before the first episode
        for e in range(2):
            ob.t_in = np.array([[a.heating.temperature[0] for a in com.agents]], np.float32)
            ob.t_m = np.array([[a.heating.building_mass_temperature[0] for a in com.agents]], np.float32)
            eps = com.agents[0].actor._epsilon
            reward, loss = com.train_episode()
            assert com._engine.last_kernel().startswith(f"episode_kernel<{n},tile"), com._engine.last_kernel()
            out = ob.run_episode("train", codes=reference_replay_codes(rs, T, R, n, eps)[:, :, None, :], eps=eps)
            assert loss == 0.0 and reward == float(out["episode_reward"][0]), e
            assert np.array_equal(com.last_rewards, out["reward"][:, 0, :]), e
            assert np.array_equal(com.decisions, np.array([0.0, 0.5, 1.0])[out["action"][:, :, 0, :]] * 3e3), e
            tabs = np.stack([a.actor.q_table for a in com.agents])
            assert np.array_equal(tabs.reshape(n, -1, 3), ob.q), e
            assert np.count_nonzero(tabs) > 0
        power, cost = com.run()  # greedy day with the learned tables
        assert power.shape == (T, n) and np.all(np.isfinite(cost))
    finally:
        setup.homogeneous = False


def test_standalone_qactor_matches_reference_sequence():
    """rl.QActor per-call API (select_action/train) on the device vs the reference's QActor."""
    from p2pmicrogrid_amd.rl import QActor
    d = load_golden("qactor")
    a = QActor(20, 20, 20, 20, epsilon=0.81, decay=0.9)
    np.random.seed(42)
    for k in range(len(d["acts"])):
        assert a._epsilon == d["eps"][k]
        act, q = a.select_action(d["s_obs"][k:k + 1])
        assert act == d["acts"][k] and q == d["qs"][k], k
        a.train(d["s_obs"][k:k + 1], act, d["rew"][k:k + 1], d["n_obs"][k:k + 1])
        if k % 500 == 499:
            a.decay_exploration()
    q = a.q_table
    nz = np.argwhere(q != 0)
    assert np.array_equal(nz, d["q_nz_idx"]) and np.array_equal(q[tuple(nz.T)], d["q_nz_val"])
    assert a._get_state_indices(d["obs"][:1]) == tuple(d["idx"][0])


def test_main_loop_and_npy_checkpoints(tmp_path, monkeypatch):
    from p2pmicrogrid_amd import community, rl, setup
    monkeypatch.setattr(rl, "MODELS_DIR", str(tmp_path))
    np.random.seed(42)
    res = community.main(episodes=3, verbose=False)
    com = res["community"]
    assert len(res["rewards"]) == 3 and all(np.isfinite(res["rewards"]))
    setting = community.setting_name().replace("-", "_")
    for a in com.agents:
        saved = np.load(tmp_path / "models_tabular" / f"{setting}_{a.id}.npy")
        assert saved.shape == (20, 20, 20, 20, 3) and saved.dtype == np.float64
        assert np.array_equal(saved, a.actor.q_table) and np.count_nonzero(saved) > 0
    out = community.load_and_run(is_testing=True)
    assert len(out) == 5 and all(v["power"].shape == (96, setup.nr_agents) for v in out.values())


def test_db_sinks_from_training_and_evaluation(tmp_path, monkeypatch):
    """main(con) logs training_progress; load_and_run(con) writes test_results rows and the
    per-round decisions (community.py:333-353) that data_analysis.py reads back."""
    from p2pmicrogrid_amd import community, database as db, rl, setup
    monkeypatch.setattr(rl, "MODELS_DIR", str(tmp_path))
    con = db.get_connection(str(tmp_path / "results.db"))
    db.create_tables(con.cursor())
    np.random.seed(42)
    community.main(episodes=2, verbose=False, con=con)
    prog = db.get_training_progress(con)
    assert len(prog) == 2 and prog["episode"].tolist() == [0, 1]
    out = community.load_and_run(is_testing=True, con=con)
    res = db.get_test_results(con)
    N, days = setup.nr_agents, sorted(out)
    assert len(res) == 96 * N * len(days)
    for d in days:
        for i in range(N):
            rows = res[(res["day"] == d) & (res["agent"] == i)].sort_values("time")
            assert np.allclose(rows["cost"].values, out[d]["cost"][:, i].astype(np.float64))
            assert np.allclose(rows["heatpump"].values, out[d]["decisions"][:, -1, i])
    rd = db.get_rounds_decisions(con)
    assert len(rd) == 96 * N * len(days) * (setup.rounds + 1)


def test_reference_entry_point_calls(tmp_path, monkeypatch):
    """The reference's own call forms (community.py:436-437), positionally, against a temp
    SQLite DB: main(db_connection, load_agents=True, analyse=True) resumes from the saved tables,
    trains, logs and runs the greedy validation rollout; load_and_run(db_connection,
    is_testing=True, analyse=False) writes test_results and rounds_comparison rows."""
    from p2pmicrogrid_amd import agent as agent_mod, community, database as db, rl, setup
    monkeypatch.setattr(rl, "MODELS_DIR", str(tmp_path))
    monkeypatch.setattr(setup, "max_episodes", 101)  # decays after 0, 50, 100; checkpoints at 50, 100
    db_connection = db.get_connection(str(tmp_path / "results.db"))
    db.create_tables(db_connection.cursor())
    np.random.seed(42)
    first = community.main(db_connection)  # fresh training, saves the tables
    saved = [a.actor.q_table.copy() for a in first["community"].agents]
    loaded = []
    orig = agent_mod.QAgent.load_from_file

    def spy(self, setting, implementation):
        orig(self, setting, implementation)
        loaded.append(self.actor.q_table.copy())
    monkeypatch.setattr(agent_mod.QAgent, "load_from_file", spy)
    res = community.main(db_connection, load_agents=True, analyse=True)
    assert len(loaded) == setup.nr_agents and all(np.array_equal(a, b) for a, b in zip(loaded, saved))
    assert len(res["rewards"]) == 101 and np.all(np.isfinite(res["rewards"]))
    val_env, _ = community.ds.get_validation_data()
    T_val, N = len(val_env), setup.nr_agents
    assert res["power"].shape == (T_val, N) and res["cost"].shape == (T_val, N)
    assert np.all(np.isfinite(res["cost"])) and res["decisions"].shape == (T_val, setup.rounds + 1, N)
    prog = db.get_training_progress(db_connection)
    assert len(prog) == 2 * 4  # episodes 0, 50, 100 + the final row, per main() call
    community.load_and_run(db_connection, is_testing=True, analyse=False)
    res_rows = db.get_test_results(db_connection)
    test_env, _ = community.ds.get_test_data()
    n_days = len(np.unique(test_env["day"]))
    assert len(res_rows) == 96 * N * n_days
    rd = db.get_rounds_decisions(db_connection)
    assert len(rd) == 96 * N * n_days * (setup.rounds + 1)
    assert set(np.unique(rd["decision"])) <= {0.0, 1500.0, 3000.0}


def test_battery_is_inert_by_default_and_opt_in_rule(monkeypatch):
    """The reference never runs a battery rule for RL agents (agent.py:200-213): a community whose
    agents carry BatteryStorage trains and runs exactly like the NoStorage one, the SoC stays at
    its reset value and BatteryStorage.step fills the history.  battery_rule=True (the extension)
    changes the flows and moves the SoC."""
    from p2pmicrogrid_amd.community import CommunityMicrogrid
    from p2pmicrogrid_amd.storage import Battery, BatteryStorage
    d = load_golden("loop_thesis_T96")
    T = int(d["T"])
    outs = []
    for variant in ("none", "inert", "rule"):
        com, env = _community_from_fixture(d)
        if variant != "none":
            for a in com.agents:
                a.storage = BatteryStorage(Battery(10 * 3.6e6, 5e3, 0.1, 0.9, 0.9, 0.5))
            if variant == "rule":
                com = CommunityMicrogrid(com.timeline, com.agents, com._rounds, battery_rule=True)
        r1, _ = com.train_episode()
        rew = com.last_rewards.copy()
        for a in com.agents:
            a.heating.set_state(21.0, 21.0)
        power, cost = com.run()
        socs = [a.storage.soc for a in com.agents] if variant != "none" else None
        hist = [len(a.storage.get_history()) for a in com.agents] if variant != "none" else None
        outs.append((rew, power, cost, socs, hist))
    base, inert, rule = outs
    assert all(np.array_equal(x, y) for x, y in zip(base[:3], inert[:3]))
    assert inert[3] == [0.5, 0.5] and inert[4] == [T, T]
    assert not np.array_equal(rule[2], base[2]) and any(s != 0.5 for s in rule[3])
