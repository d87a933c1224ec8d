"""The per-agent step API (agent.py:111-136, 200-298; community.py:45-93,149-188) driven one
agent call at a time, in the reference's own loop shape, against the reference-driven fixtures.

Every decision goes through ``QAgent.__call__`` (exploration from the global np.random in the
reference's consumption order, the greedy action on the device table), every reward through
``get_reward``, every TD update through ``QAgent.train`` (p2pmg_q_calls) and every RC update through
``HPHeating.step`` (p2pmg_rc_step); the market and costs are ``CommunityMicrogrid._run`` /
``_compute_costs``.  Results must equal the fixtures bit for bit."""
import numpy as np
import pytest

from conftest import load_golden
from test_gpu_api import _community_from_fixture

pytestmark = pytest.mark.gpu
F32 = np.float32


def _episode_stepped(com, env, N):
    """community.py:149-182 with the agents stepped by hand; returns the per-step records."""
    rec = {k: [] for k in ("reward", "cost", "grid", "p2p", "t_in")}
    for t, (state, next_state) in enumerate(env.data):
        rec["t_in"].append([float(a.heating.temperature[0]) for a in com.agents])
        p_grid, p_p2p, buy, inj, p2pp = com._run(t, state, training=True)
        costs = com._compute_costs(p_grid, p_p2p, np.expand_dims(buy, 0), inj, p2pp).reshape(-1)
        rw = []
        for i, agent in enumerate(com.agents):
            r = agent.get_reward(costs[i])
            assert agent.train(r, np.expand_dims(next_state, 0), np.zeros(N, F32)) == 0.0
            rw.append(float(r[0]))
        rec["reward"].append(rw)
        rec["cost"].append(costs.tolist())
        rec["grid"].append(p_grid.tolist())
        rec["p2p"].append(p_p2p.tolist())
        com._step()
    for agent in com.agents:
        agent.reset()
    return {k: np.asarray(v, F32) for k, v in rec.items()}


@pytest.mark.parametrize("name", ["loop_thesis_T96", "loop_n5_r2_T96"])
def test_per_agent_stepping_reproduces_reference_driven_training(name):
    from p2pmicrogrid_amd import setup
    from p2pmicrogrid_amd.engine import price_table
    d = load_golden(name)
    N, E = int(d["N"]), min(int(d["E"]), 2)
    try:
        com, env = _community_from_fixture(d)
        if not all(np.array_equal(a, b) for a, b in zip(price_table(d["env_time"]), (d["buy"], d["inj"], d["p2pp"]))):
            pytest.skip("this host's numpy f32 sin differs from the fixture host's (price table input)")
        for e in range(E):
            assert np.array_equal([a.heating.temperature[0] for a in com.agents], d["t_in0"][e])
            rec = _episode_stepped(com, env, N)
            for k in ("reward", "cost", "grid", "p2p", "t_in"):
                assert np.array_equal(rec[k], d[f"train_{k}"][e]), (e, k)
            act = np.rint(com.decisions / 3e3 * 2).astype(np.int64)  # heat-pump power -> action index
            assert np.array_equal(act, d["train_action"][e]), e
            tabs = np.stack([a.actor.q_table for a in com.agents])
            qi, qv = d[f"q_idx_{e}"], d[f"q_val_{e}"]
            assert np.count_nonzero(tabs) == len(qv) and np.array_equal(tabs[tuple(qi.T)], qv), e
            if e % 50 == 0:
                for a in com.agents:
                    a.actor.decay_exploration()
    finally:
        setup.homogeneous = False


def test_greedy_take_decision_and_rule_agent():
    """QAgent.take_decision (agent.py:277-289) per agent == the device greedy run of the same
    community, and RuleAgent.take_decision (agent.py:116-128) == its hysteresis rule."""
    from p2pmicrogrid_amd import setup
    from p2pmicrogrid_amd.agent import RuleAgent, divide_power
    from p2pmicrogrid_amd.dataset import ProfileDataset
    from p2pmicrogrid_amd.heating import HeatPump, HPHeating
    from p2pmicrogrid_amd.production import PV, Prosumer
    from p2pmicrogrid_amd.storage import NoStorage
    d = load_golden("loop_thesis_T96")
    try:
        com, env = _community_from_fixture(d)
        q = np.random.RandomState(3).uniform(-1, 1, (2, 20, 20, 20, 20, 3))
        for i, a in enumerate(com.agents):
            a.actor.set_qtable(q[i])
        t_in0 = [a.heating.temperature[0] for a in com.agents]
        t_m0 = [a.heating.building_mass_temperature[0] for a in com.agents]
        power, cost = com.run()  # the fused device path
        dev_decisions = com.decisions.copy()
        for a, x, y in zip(com.agents, t_in0, t_m0):
            a.reset()
            a.heating.set_state(x, y)
        grid, p2p = [], []
        for t, (state, _) in enumerate(env.data):
            g, pp, buy, inj, p2pp = com._run(t, state, training=False)
            grid.append(g)
            p2p.append(pp)
            com._step()
        assert np.array_equal(com.decisions, dev_decisions)
        assert np.array_equal(np.asarray(grid, F32) + np.asarray(p2p, F32), power)
        # divide_power quirks: even split incl. the diagonal, opposite-sign keep
        assert np.array_equal(divide_power([1000.0], [-0.0, -0.0]), np.array([500.0, 500.0], F32))
        assert np.array_equal(divide_power([-1000.0], [-0.0, 500.0]), np.array([-0.0, -1000.0], F32))
        # RuleAgent: on at T_in <= 20, off at >= 22, net power (load - pv) + hp
        ds = lambda x: ProfileDataset(np.asarray(x, F32), np.roll(np.asarray(x, F32), -1, 0))  # noqa: E731
        h = HPHeating(HeatPump(3.0, 3e3, 0.0), 21.0)
        ra = RuleAgent(ds(d["load_w"][0]), Prosumer(PV(4e3, ds(d["pv_w"][0]))), NoStorage(), h, max_in=4.4e3,
                       max_out=0.0)
        h.set_state(19.5, 20.0)
        p, z = ra.take_decision()
        assert h.hp.power == 1 and np.array_equal(p, np.array([F32(d["load_w"][0][0] - d["pv_w"][0][0]) + F32(3e3)], F32))
        assert np.array_equal(z, np.array([0.0], F32))
    finally:
        setup.homogeneous = False


def test_battery_storage_rule_on_device_matches_reference_storage():
    """BatteryStorage.apply_rule / RuleAgent._update_storage (agent.py:138-153 on storage.py:36-76,
    run by p2pmg_battery_seq) vs the reference's own BatteryStorage sequence (battery.npz)."""
    from p2pmicrogrid_amd.agent import RuleAgent
    from p2pmicrogrid_amd.dataset import ProfileDataset
    from p2pmicrogrid_amd.heating import HeatPump, HPHeating
    from p2pmicrogrid_amd.production import PV, Prosumer
    from p2pmicrogrid_amd.storage import Battery, BatteryStorage
    g = load_golden("battery")
    mk = lambda: BatteryStorage(Battery(float(g["capacity"]), 5e3, float(g["min_soc"]), float(g["max_soc"]),  # noqa: E731
                                        float(g["efficiency"]), float(g["soc0"])))
    st = mk()
    out = st.apply_rule(g["bal"])
    assert np.array_equal(out, g["out_bal"]) and st.soc == g["soc"][-1]
    ds = lambda x: ProfileDataset(np.asarray(x, F32), np.roll(np.asarray(x, F32), -1, 0))  # noqa: E731
    ra = RuleAgent(ds(np.zeros(4)), Prosumer(PV(1e3, ds(np.zeros(4)))), mk(), HPHeating(HeatPump(3.0, 3e3, 0.0), 21.0),
                   max_in=1e3, max_out=0.0)
    for k in range(5):
        assert ra._update_storage(float(g["bal"][k])) == g["out_bal"][k] and ra.storage.soc == g["soc"][k]
    ra.storage.step()
    ra.storage.reset()
    assert ra.storage.soc == 0.5 and ra.storage.get_history() == []
