"""CPU checks of the DQN oracle (config 5): gradients against torch autograd, sampler and
replay-order properties, mode equivalences.  TF is absent, so the reference's own numbers
are unavailable (parity with TF unpinned, see oracle/dqn.py)."""
import random

import numpy as np
import pytest
import torch

from oracle import dqn, philox
from oracle.restatement import GREEDY


def _torch_loss(theta, s, a, r, ns, target, gamma):
    def fwd(th, x):
        W1, b1 = th[0:320].reshape(5, 64), th[320:384]
        W2, b2 = th[384:4480].reshape(64, 64), th[4480:4544]
        W3, b3 = th[4544:4608].reshape(64, 1), th[4608:4609]
        h1 = torch.relu(x @ W1 + b1)
        h2 = torch.relu(h1 @ W2 + b2)
        return (h2 @ W3 + b3)[:, 0]
    B = s.shape[0]
    with torch.no_grad():
        qn = torch.stack([fwd(target, torch.cat([ns, torch.full((B, 1), v, dtype=ns.dtype)], 1))
                          for v in (0.0, 0.5, 1.0)]).max(0).values
    y = r + gamma * qn
    q = fwd(theta, torch.cat([s, a[:, None]], 1))
    return ((y - q) ** 2).mean()


def test_gradients_match_torch_autograd():
    rs = np.random.RandomState(1)
    th = dqn.glorot_init(3, seed=5)
    tg = dqn.glorot_init(3, seed=6)
    s = rs.uniform(-1, 1, (3, 32, 4)).astype(np.float32)
    ns = rs.uniform(-1, 1, (3, 32, 4)).astype(np.float32)
    a = dqn.ACTION_VALUES[rs.randint(0, 3, (3, 32))]
    r = rs.uniform(-3, 0, (3, 32)).astype(np.float32)
    g, loss = dqn.gradients(th, s, a, r, ns, tg, 0.95)
    for n in range(3):
        t = torch.tensor(th[n], dtype=torch.float64, requires_grad=True)
        L = _torch_loss(t, *(torch.tensor(x[n], dtype=torch.float64) for x in (s, a, r, ns)),
                        torch.tensor(tg[n], dtype=torch.float64), 0.95)
        L.backward()
        want = t.grad.numpy()
        assert abs(loss[n] - L.item()) <= 1e-5 * abs(L.item())
        np.testing.assert_allclose(g[n], want, rtol=1e-4, atol=1e-6 * np.abs(want).max())


def test_adam_and_soft_update_formulas():
    th = dqn.glorot_init(1, seed=2)
    m, v = np.zeros_like(th), np.zeros_like(th)
    g = np.random.RandomState(3).normal(size=th.shape).astype(np.float32) * 3
    t0 = th.copy()
    dqn.adam_step(th, m, v, g, 1)
    gc = g.copy()
    gc[:, :320] = np.clip(gc[:, :320], -1, 1)
    g64 = gc.astype(np.float64)
    m64, v64 = 0.1 * g64, 0.001 * g64 * g64
    lr_t = 1e-5 * np.sqrt(1 - 0.999) / (1 - 0.9)
    want = t0.astype(np.float64) - lr_t * m64 / (np.sqrt(v64) + 1e-7)
    np.testing.assert_allclose(th, want, rtol=0, atol=2e-7 * np.abs(t0).max() + 1e-9)
    assert np.abs(want - t0).max() > 5e-6  # the step is visible above the tolerance
    tg = t0.copy()
    dqn.soft_update(tg, th, 0.005)
    np.testing.assert_allclose(tg, 0.995 * t0 + 0.005 * th, rtol=1e-6, atol=1e-9)


def test_philox_sampler_distinct_and_in_range():
    for count in (32, 33, 480, 5000):
        idx = philox.sample_draws(42, 3, np.arange(500), 7, count)
        assert idx.shape == (500, 32) and idx.min() >= 0 and idx.max() < count
        assert all(len(set(row)) == 32 for row in idx)
    idx = philox.sample_draws(42, 3, np.arange(20000), 7, 480)
    hist = np.bincount(idx.ravel(), minlength=480) / idx.size
    assert np.abs(hist * 480 - 1).max() < 0.15


def test_reference_replay_consumption_order():
    py, npr = random.Random(42), np.random.RandomState(42)
    codes, samples = dqn.reference_dqn_replay(py, npr, 2, 1, 2, 0.5, counts=[480, 480])
    py2, np2 = random.Random(42), np.random.RandomState(42)
    for t in range(2):
        for r in range(2):
            for i in range(2):
                want = np2.choice([0, 1, 2]) if py2.random() < 0.5 else GREEDY
                assert codes[t, r, i] == want
        for i in range(2):
            assert list(samples[t, i]) == py2.sample(range(481 + t), 32)


def _batch(S, N, R, T, shared, theta=None):
    from p2pmicrogrid_amd.dataset import scenario_batch
    inp = scenario_batch(S, N, T)
    th = dqn.glorot_init(1 if shared else S * N, seed=11) if theta is None else theta
    ob = dqn.OracleDQNBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                            env_time=inp.time[None], env_tout=inp.t_out, theta0=th, shared=shared)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    return ob


def test_shared_equals_per_agent_for_a_single_agent():
    a = _batch(1, 1, 1, 24, shared=False)
    b = _batch(1, 1, 1, 24, shared=True, theta=a.theta.copy())
    for ob in (a, b):
        ob.run_episode("fill", rng="philox", episode=0, eps=1.0)
        ob.run_episode("fill", rng="philox", episode=1, eps=1.0)
    oa = a.run_episode("train", rng="philox", episode=2, eps=0.5)
    ob_ = b.run_episode("train", rng="philox", episode=2, eps=0.5)
    assert np.array_equal(oa["action"], ob_["action"])
    np.testing.assert_allclose(a.theta, b.theta, rtol=1e-6, atol=1e-9)


def test_episode_modes_run_and_learn_something():
    ob = _batch(4, 2, 1, 96, shared=False)
    ob.run_episode("fill", rng="philox", episode=0, eps=1.0)
    assert ob.count().min() == 96
    th0 = ob.theta.copy()
    out = ob.run_episode("train", rng="philox", episode=1, eps=1.0)
    assert np.isfinite(out["episode_reward"]).all() and (out["loss"] > 0).all()
    assert ob.step == 96 and not np.array_equal(th0, ob.theta)
    g = ob.run_episode("greedy")
    assert np.array_equal(g["action"], np.argmax(g["q"], axis=-1))


def _replay_fixture_draws(draw_fn, d):
    """Re-draw the fixture's episode sequence with ``draw_fn(py, npr, T, R, N, eps, counts)``:
    5 fill episodes, Trainer.initialize_target's sample per agent, then training episodes."""
    import random
    T, R, N = int(d["T"]), int(d["R"]), int(d["N"])
    F, E = int(d["fill_episodes"]), int(d["train_episodes"])
    py, npr = random.Random(42), np.random.RandomState(42)
    added = np.zeros(N, np.int64)
    codes, tags, init = [], {}, None
    for e in range(F + E):
        training = e >= F
        counts = np.minimum(added, 5000) if training else None
        c, smp = draw_fn(py, npr, T, R, N, float(d["eps"][e]), counts)
        codes.append(np.asarray(c))
        if training:
            # deque index j of the step's sample -> tag = added-before-step + 1 - count + j
            step_added = added[None, :] + np.arange(1, T + 1)[:, None]             # [T, N]
            first = step_added - np.minimum(step_added, 5000)
            tags[e - F] = np.asarray(smp, np.int64) + first[..., None]
        added += T
        if e == F - 1:
            init = np.array([py.sample(range(int(min(a, 5000))), 32) for a in added])
    return np.stack(codes), tags, init


@pytest.mark.parametrize("which", ["oracle", "package"])
def test_dqn_draws_match_reference_actor_and_replay_buffer(which):
    """Pins a20's exploration + replay stream on the reference's own code: ActorModel.select_action
    (rl.py:173-184) and ReplayBuffer.add/sample_batch (rl.py:209-244), driven in the DQN community's
    order with tagged experiences (tests/golden/dqn_draws.npz, make_golden.make_dqn_draws), across
    the 5000-entry deque eviction.  Both the oracle's reference_dqn_replay and the package's
    rng.dqn_episode_draws (what CommunityMicrogrid uploads as replay codes / samples) reproduce it."""
    from conftest import load_golden
    from p2pmicrogrid_amd import rng
    d = load_golden("dqn_draws")
    if which == "oracle":
        from oracle import dqn as odqn
        fn = lambda py, npr, T, R, N, eps, counts: odqn.reference_dqn_replay(py, npr, T, R, N, eps, counts=counts)  # noqa: E731
    else:
        fn = lambda py, npr, T, R, N, eps, counts: rng.dqn_episode_draws(py, npr, T, R, N, [eps] * N, counts=counts)  # noqa: E731
    codes, tags, init = _replay_fixture_draws(fn, d)
    assert np.array_equal(codes, d["codes"])
    assert np.array_equal(init, d["init_tags"])
    for e in d["keep"]:
        assert np.array_equal(tags[int(e)], d[f"sample_tags_{int(e)}"]), e
    assert tags[int(d["keep"][-1])].max() > 5000  # the kept tail episodes sample past the eviction


def test_host_replay_buffer_short_batches_match_reference():
    """rl.ReplayBuffer standalone (host deque): sampling after each of 40 adds (count < 32 first,
    rl.py:234-235) returns the reference's items in the reference's order."""
    import random
    from conftest import load_golden
    from p2pmicrogrid_amd.rl import ReplayBuffer
    d = load_golden("dqn_draws")
    random.seed(7)
    b = ReplayBuffer(5000, 32)
    got = []
    for k in range(40):
        b.add(np.float32(k), np.float32(0), np.float32(0), np.float32(0))
        s, _, _, _ = b.sample_batch()
        got.append(np.asarray(s).reshape(-1))
    assert np.array_equal([len(x) for x in got], d["short_len"])
    assert np.array_equal(np.concatenate(got).astype(np.uint16), d["short_tags"])
