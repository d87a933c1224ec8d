"""The DQN object API (rl.ActorModel/Trainer/QNetwork/ReplayBuffer, agent.DQNAgent,
CommunityMicrogrid with DQN agents) on the device, checked against the oracle driven by the
same Python-random / np.random streams in the reference's consumption order."""
import random

import numpy as np
import pytest

from conftest import load_golden
from oracle import dqn as odqn

pytestmark = pytest.mark.gpu


def _dqn_community(d):
    from p2pmicrogrid_amd import setup
    from p2pmicrogrid_amd.agent import Agent, DQNAgent
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
    random.seed(42)
    rng = ReferenceRNG()
    lr, pr = rng.community_ratings(N, setup.homogeneous)
    ds = lambda x: ProfileDataset(np.asarray(x, np.float32), np.roll(np.asarray(x, np.float32), -1, 0))  # noqa: E731
    Agent.reset_ids()
    agents = [DQNAgent(ds(d["load_w"][i]), Prosumer(PV(pr[i] * 1e3, ds(d["pv_w"][i]))), NoStorage(),
                       HPHeating(HeatPump(3.0, 3e3, 0.0), 21.0), max_in=max(lr[i], pr[i]) * 1.1 * 1e3,
                       max_out=-(max(lr[i], pr[i]) + 1.1e3)) for i in range(N)]
    env.setup(ds(np.stack([d["env_time"], d["env_tout"]], axis=1)))
    return CommunityMicrogrid(list(range(T)), agents, R)


def _oracle_from(com, d):
    eng = com._engine
    ob = odqn.OracleDQNBatch(S=1, N=eng.N, R=eng.R, load_w=d["load_w"][None], pv_w=d["pv_w"][None],
                             max_in=np.array([a.max_in for a in com.agents], np.float32)[None],
                             env_time=d["env_time"][None], env_tout=d["env_tout"][None],
                             theta0=eng.get_weights("online"))
    ob.target = eng.get_weights("target")
    ob.m, ob.v = eng.get_weights("adam_m"), eng.get_weights("adam_v")
    ob.step = eng.step
    buf, added = eng.get_buffer()
    ob.buf = buf.reshape(1, eng.N, -1, 10).copy()
    ob.added = added.reshape(1, eng.N).astype(np.int64)
    ob.t_in = np.array([[a.heating.temperature[0] for a in com.agents]], np.float32)
    ob.t_m = np.array([[a.heating.building_mass_temperature[0] for a in com.agents]], np.float32)
    return ob


def test_dqn_community_train_matches_oracle(tmp_path, monkeypatch):
    from p2pmicrogrid_amd import rl
    d = load_golden("loop_thesis_T96")
    N, R, T = int(d["N"]), int(d["R"]), int(d["T"])
    com = _dqn_community(d)
    # init_buffers: 5 exploring episodes (epsilon 1: every action is a replayed random action)
    py_snap, np_snap = random.getstate(), np.random.get_state()
    com.init_buffers()
    eng = com._engine
    _, added = eng.get_buffer()
    assert (added == 5 * T).all()
    assert np.array_equal(eng.get_weights("online"), eng.get_weights("target"))  # initialize_target
    py, rs = random.Random(), np.random.RandomState()
    py.setstate(py_snap)
    rs.set_state(np_snap)
    codes, _ = odqn.reference_dqn_replay(py, rs, T, R, N, 1.0)
    buf, _ = eng.get_buffer()
    assert np.array_equal(buf[:, :T, 4], odqn.ACTION_VALUES[codes[:, R, :].T])  # first episode's stored actions

    for e in range(2):
        ob = _oracle_from(com, d)
        th0 = ob.theta.copy()
        eps = com.agents[0].actor._epsilon
        py.setstate(random.getstate())
        rs.set_state(np.random.get_state())
        codes, samples = odqn.reference_dqn_replay(py, rs, T, R, N, eps, counts=ob.count().ravel())
        reward, loss = com.train_episode()
        out = ob.run_episode("train", codes=codes[:, :, None, :], samples=samples[:, None], rng="replay")
        assert np.array_equal(com.last_rewards, out["reward"][:, 0, :])
        assert reward == float(out["episode_reward"][0])
        np.testing.assert_allclose(com.last_losses, out["loss"][:, 0, :], rtol=1e-4, atol=1e-7)
        th = eng.get_weights("online")
        upd, want = th - th0, ob.theta - th0
        assert np.abs(upd - want).max() <= 1e-2 * np.abs(want).max()
        for a in com.agents:
            a.actor.decay_exploration()

    ob.t_in = np.array([[a.heating.temperature[0] for a in com.agents]], np.float32)  # after agent.reset()
    ob.t_m = np.array([[a.heating.building_mass_temperature[0] for a in com.agents]], np.float32)
    power, cost = com.run()
    out = ob.run_episode("greedy")
    assert np.array_equal(com.decisions / 3e3, odqn.ACTION_VALUES[out["action"][:, :, 0, :]])

    monkeypatch.setattr(rl, "MODELS_DIR", str(tmp_path))
    for a in com.agents:
        a.save_to_file("setting-x", "dqn")
    th_saved = eng.get_weights("online")
    com2 = _dqn_community(d)
    for a in com2.agents:
        a.load_from_file("setting-x", "dqn")
    assert np.array_equal(np.stack([a.actor.q_network.flat_weights() for a in com2.agents]), th_saved)
    assert np.array_equal(np.stack([a.trainer.target_network.flat_weights() for a in com2.agents]),
                          eng.get_weights("target"))


def test_standalone_actor_and_trainer():
    from p2pmicrogrid_amd import rl
    actor = rl.ActorModel(epsilon=0.0)
    th = actor.q_network.flat_weights()
    s = np.array([[0.25, -0.3, 0.1, 0.0]], np.float32)
    act, q = actor.greedy_action(s)
    qo = odqn.q_values(th, s[None])[0, 0]
    assert act[0] == odqn.ACTION_VALUES[int(np.argmax(qo))]
    np.testing.assert_allclose(q[:, 0], qo, rtol=1e-5, atol=1e-6)
    tr = rl.Trainer(actor, buffer_size=100, batch_size=32, gamma=0.95, tau=0.005, optimizer=rl.Adam(1e-5))
    rs = np.random.RandomState(1)
    for _ in range(40):
        tr.buffer.add(rs.uniform(-1, 1, 4).astype(np.float32), np.float32(0.5), np.float32(-1.0),
                      rs.uniform(-1, 1, 4).astype(np.float32))
    tr._soft_update(actor.q_network, tr.target_network, tau=1.0)
    s_, a_, r_, ns_ = tr.buffer.sample_batch()
    th0, tg0 = actor.q_network.flat_weights(), tr.target_network.flat_weights()
    loss = tr._train(s_, a_, r_, ns_)
    g, lo = odqn.gradients(th0[None], s_[None], a_.reshape(1, -1), r_.reshape(1, -1), ns_[None], tg0[None], 0.95)
    m, v, tho = np.zeros_like(th0[None]), np.zeros_like(th0[None]), th0[None].copy()
    odqn.adam_step(tho, m, v, g, 1)
    assert abs(loss - lo[0]) <= 1e-5 * abs(lo[0])
    upd = actor.q_network.flat_weights() - th0
    assert np.abs(upd - (tho[0] - th0)).max() <= 1e-2 * np.abs(tho[0] - th0).max()
