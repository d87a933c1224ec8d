"""DQN variant (config 5) on the device vs the oracle (oracle/dqn.py).

The oracle's default order restates the kernels' summation order (fmaf chains in the MFMA k
order, the DPP / permlane trees, the block -> segment gradient structure), so Q values, losses,
weights, Adam state and every simulation quantity are compared BIT FOR BIT.  The NumPy-matmul
order (oracle.dqn.forward / gradients, order="matmul") is kept as an independent second check,
held to north_star's 1e-5 relative on Q values."""
import random

import numpy as np
import pytest

from oracle import dqn as odqn
from oracle import philox
from p2pmicrogrid_amd.dataset import scenario_batch
from p2pmicrogrid_amd.dqn import DeviceDQNBatch

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _rel_close(got, want, rtol=RTOL, floor=1e-3):
    """|got - want| <= rtol * max(|want|, floor * max|want|) elementwise."""
    want = np.asarray(want, np.float64)
    scale = np.maximum(np.abs(want), floor * np.abs(want).max())
    err = np.abs(np.asarray(got, np.float64) - want) / scale
    assert err.max() <= rtol, f"max rel err {err.max():.3g} at {np.unravel_index(err.argmax(), err.shape)}"


def _q_scale(theta, x):
    """fp32 yardstick of Q(x): magnitude of the summed terms sum_j |h2_j w3_j| + |b3| (a dot
    product's rounding error scales with it, not with the possibly cancelled result)."""
    _, (_, _, _, _, h2) = odqn.forward(theta, x)
    p = odqn.unpack(theta)
    return np.abs(h2) @ np.abs(p["W3"][..., 0]) + np.abs(p["b3"][0])


def _q_close(got, theta, x, rtol=RTOL):
    want, _ = odqn.forward(theta, x)
    err = np.abs(np.asarray(got, np.float64) - want) / _q_scale(theta, x)
    assert err.max() <= rtol, f"max scaled err {err.max():.3g}"


def _eq(got, want, what=""):
    got, want = np.asarray(got), np.asarray(want)
    if not np.array_equal(got, want):
        d = np.abs(got.astype(np.float64) - want)
        raise AssertionError(f"{what}: {np.count_nonzero(d)} of {d.size} differ, max |diff| {d.max():.3g}")


def test_forward_matches_oracle():
    eng = DeviceDQNBatch(1, 2, 1, 8, init_seed=3)
    th = eng.get_weights("online")
    x = np.random.RandomState(0).uniform(-1, 1, (500, 5)).astype(np.float32)
    for net in (0, 1):
        got = eng.forward(x, net)
        _eq(got, odqn.api_forward(th[net], x), "forward (device order)")
        _q_close(got, th[net], x)  # matmul order, north_star tolerance
    eng.close()


def test_train_batch_matches_oracle_step():
    eng = DeviceDQNBatch(1, 1, 1, 8, init_seed=4)
    th = eng.get_weights("online")
    tg = odqn.glorot_init(1, seed=9)
    eng.set_weights("target", tg)
    rs = np.random.RandomState(2)
    m, v = np.zeros_like(th), np.zeros_like(th)
    th_o, tg_o = th.copy(), tg.copy()
    th_m, tg_m, m_m, v_m = th.copy(), tg.copy(), m.copy(), v.copy()  # matmul-order second check
    for k in range(3):
        s = rs.uniform(-1, 1, (32, 4)).astype(np.float32)
        ns = rs.uniform(-1, 1, (32, 4)).astype(np.float32)
        a = odqn.ACTION_VALUES[rs.randint(0, 3, 32)]
        r = rs.uniform(-3, 0, 32).astype(np.float32)
        loss = eng.train_batch(s, a, r, ns)
        batch = np.concatenate([s, a[:, None], r[:, None], ns], 1)
        g, lo = odqn.train_block(th_o, tg_o, batch[None], 0.95)
        odqn.adam_step(th_o, m, v, g[None], k + 1)
        odqn.soft_update(tg_o, th_o, 0.005)
        assert np.float32(loss) == lo[0], (loss, lo[0])
        gm, lm = odqn.gradients(th_m, s[None], a[None], r[None], ns[None], tg_m, 0.95)
        if k == 0:
            # the first Adam step's m is (1 - beta1) * g: the device's gradient against the
            # matmul-order one at north_star's 1e-5 of each parameter group's scale
            # (tests/test_cpu_dqn_orders.py; the update itself amplifies near-zero components)
            b1c = np.float64(np.float32(1.0) - np.float32(0.9))
            g_dev = eng.get_weights("adam_m")[0].astype(np.float64) / b1c
            g_mm = gm[0].astype(np.float64)
            g_mm[:320] = np.clip(g_mm[:320], -1.0, 1.0)  # the first kernel's clip (rl.py:329, adam_step)
            for lo, hi in ((0, 320), (320, 384), (384, 4480), (4480, 4544), (4544, 4608), (4608, 4609)):
                scale = np.abs(g_mm[lo:hi]).max()
                assert np.abs(g_dev[lo:hi] - g_mm[lo:hi]).max() <= 1e-5 * scale, (lo, hi)
        odqn.adam_step(th_m, m_m, v_m, gm, k + 1)
        odqn.soft_update(tg_m, th_m, 0.005)
        assert abs(loss - lm[0]) <= 1e-5 * abs(lm[0])
    assert eng.step == 3
    _eq(eng.get_weights("online"), th_o, "online")
    _eq(eng.get_weights("adam_m"), m, "adam_m")
    _eq(eng.get_weights("adam_v"), v, "adam_v")
    _eq(eng.get_weights("target"), tg_o, "target")
    # the updates are ~1e-5 of the weights: the matmul order's update within 2e-3 of its size
    _rel_close(eng.get_weights("online") - th, th_m - th, rtol=2e-3)
    eng.close()


def test_train_batch_keeps_one_adam_count_per_network():
    """Each DQNAgent owns its Adam optimizer (agent.py:310), so training agent 0 then agent 1 of
    one context gives BOTH networks bias-correction step 1, then 2 (not 1, 2, 3, 4); an episode
    step afterwards advances each network's own count."""
    eng = DeviceDQNBatch(1, 2, 1, 8, init_seed=4)
    th = eng.get_weights("online")
    tg = eng.get_weights("target")
    rs = np.random.RandomState(5)
    state = {n: (th[n:n + 1].copy(), tg[n:n + 1].copy(), np.zeros_like(th[n:n + 1]), np.zeros_like(th[n:n + 1]))
             for n in (0, 1)}
    for k in range(2):
        for net in (0, 1):
            s = rs.uniform(-1, 1, (32, 4)).astype(np.float32)
            ns = rs.uniform(-1, 1, (32, 4)).astype(np.float32)
            a = odqn.ACTION_VALUES[rs.randint(0, 3, 32)]
            r = rs.uniform(-3, 0, 32).astype(np.float32)
            eng.train_batch(s, a, r, ns, net=net)
            th_o, tg_o, m, v = state[net]
            g, _ = odqn.train_block(th_o[0], tg_o[0], np.concatenate([s, a[:, None], r[:, None], ns], 1)[None], 0.95)
            odqn.adam_step(th_o, m, v, g[None], k + 1)  # this network's own iteration count
            odqn.soft_update(tg_o, th_o, 0.005)
    assert list(eng.net_steps()) == [2, 2]
    eng.train_batch(*[np.zeros(sh, np.float32) for sh in ((32, 4), 32, 32, (32, 4))], net=1)
    assert list(eng.net_steps()) == [2, 3]
    for net in (0, 1):
        th_o, tg_o, m, v = state[net]
        if net == 1:  # replay the extra zero batch on the oracle side too
            g, _ = odqn.train_block(th_o[0], tg_o[0], np.zeros((1, 32, 10), np.float32), 0.95)
            odqn.adam_step(th_o, m, v, g[None], 3)
            odqn.soft_update(tg_o, th_o, 0.005)
        _eq(eng.get_weights("online")[net:net + 1], th_o, f"online net {net}")
        _eq(eng.get_weights("adam_m")[net:net + 1], m, f"adam_m net {net}")
    eng.close()


def _pair(S, N, R, T, shared, init_seed=5, apb=2, segments=1):
    """Device batch + oracle with the same gradient layout (agents per train workgroup, segments)."""
    inp = scenario_batch(S, N, T)
    eng = DeviceDQNBatch(S, N, R, T, shared=shared, init_seed=init_seed, agents_per_block=apb if shared else 0,
                         grad_segments=segments if shared else 1)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    ob = odqn.OracleDQNBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                             env_time=inp.time[None], env_tout=inp.t_out, theta0=eng.get_weights("online"),
                             shared=shared, agents_per_block=apb, grad_segments=segments)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    return eng, ob


def _check_trained(eng, ob, th0):
    """The learned networks bit for bit (online, target, Adam moments), and the device network's
    Q values on probe observations: bitwise against the device-order forward, within 1e-5 of the
    matmul-order forward."""
    th, tg = eng.get_weights("online"), eng.get_weights("target")
    _eq(th, ob.theta, "online")
    _eq(tg, ob.target, "target")
    _eq(eng.get_weights("adam_m"), ob.m, "adam_m")
    _eq(eng.get_weights("adam_v"), ob.v, "adam_v")
    assert not np.array_equal(th, th0)
    probe = np.random.RandomState(7).uniform(-1, 1, (64, 4)).astype(np.float32)
    x = np.concatenate([np.repeat(probe, 3, 0), np.tile(odqn.ACTION_VALUES, 64)[:, None]], 1)
    for net in range(min(4, len(th))):
        got = eng.forward(x, net)
        _eq(got, odqn.api_forward(ob.theta[net], x), "probe Q")
        _q_close(got, ob.theta[net], x)


def _reset(eng, ob, episode):
    eng.reset_temperatures_philox(episode)
    ob.t_in, ob.t_m = (x.reshape(ob.S, ob.N) for x in philox.t0_draws(42, episode, np.arange(ob.S * ob.N)))


def _compare_episode(eng, out, mode, eps):
    rec = eng.get_records(["reward", "cost", "grid", "p2p", "t_in", "action"] + (["loss"] if mode == "train" else []))
    assert np.array_equal(rec["action"], out["action"].astype(np.uint8)), "actions differ"
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert np.array_equal(rec[k], out[k]), k
    if mode == "train":
        _eq(rec["loss"], out["loss"], "loss")
    assert np.array_equal(eng.episode_reward(), out["episode_reward"])


@pytest.mark.parametrize("S,N,R,shared,apb,segments", [(3, 2, 1, False, 0, 1), (3, 2, 1, True, 1, 1),
                                                       (2, 16, 1, False, 0, 1), (4, 3, 2, True, 5, 2),
                                                       (8, 2, 1, True, 3, 4),
                                                       # community sizes outside {1..8, 16} (the act
                                                       # kernel's 16-wave form) and R + 1 > 8 rounds
                                                       (2, 10, 1, False, 0, 1), (1, 20, 2, True, 4, 1),
                                                       (1, 33, 0, False, 0, 1), (2, 3, 8, True, 2, 1),
                                                       # 8 segments (the act kernel's fused Adam step at
                                                       # its limit) and 16 (the standalone Adam launch)
                                                       (8, 2, 1, True, 2, 8), (16, 1, 1, True, 1, 16)])
def test_episodes_match_oracle(S, N, R, shared, apb, segments):
    """Fill + two training episodes + a greedy day, bit for bit: records, replay rings, losses,
    weights, target and Adam state (shared network: blocks of apb agents, `segments` gradient
    segments on one context, summed in segment order)."""
    _episodes_vs_oracle(S, N, R, shared, apb, segments)


# The default form (fold with 4 runs per thread, standalone Adam launch) is test_episodes_match_oracle's
# segments > 1 cases; the oracle's per-agent training (tens of seconds per case) bounds the rest to one
# or two cases per form.  The fold's long runs are covered device-side (test_fold_forms_agree_on_long_runs).
@pytest.mark.parametrize("form,S,N,R,apb,segments",
                         [("act", 4, 3, 2, 5, 2), ("act", 8, 2, 1, 2, 8), ("fold1", 8, 2, 1, 3, 4),
                          ("fold16", 8, 2, 1, 3, 4), ("adam64", 8, 2, 1, 2, 8)])
def test_split_path_forms_match_oracle(monkeypatch, form, S, N, R, apb, segments):
    """The shared network's multi-segment path in each of its forms, bit for bit the oracle's step
    order (rl.py:307-359): the segment fold with 4 runs per thread (default), 1 (the reduce kernel's
    1024-thread form, P2PMG_FOLD_SPT=1), 2, 8 or 16; the post-exchange Adam step as its own launch per env
    step (default; 64-thread workgroups with P2PMG_ADAM_TPB=64) or inside env step t + 1's act launch (P2PMG_DQN_ADAM=act: double-buffered network
    state, the episode's last step settled into the primary arrays)."""
    monkeypatch.delenv("P2PMG_DQN_ADAM", raising=False)
    monkeypatch.delenv("P2PMG_FOLD_SPT", raising=False)
    monkeypatch.delenv("P2PMG_ADAM_TPB", raising=False)
    if form == "act":
        monkeypatch.setenv("P2PMG_DQN_ADAM", "act")
    elif form.startswith("fold"):
        monkeypatch.setenv("P2PMG_FOLD_SPT", form[4:])
    elif form.startswith("adam"):
        monkeypatch.setenv("P2PMG_ADAM_TPB", form[4:])
    _episodes_vs_oracle(S, N, R, True, apb, segments)


@pytest.mark.parametrize("prepass", ["1", "0"])
@pytest.mark.parametrize("S,N,R,shared,apb,segments", [(3, 2, 1, False, 0, 1), (8, 2, 1, True, 3, 4)])
def test_sample_draw_forms_match_oracle(monkeypatch, prepass, S, N, R, shared, apb, segments):
    """Philox training's replay draws (ReplayBuffer.sample_batch rl.py:226-241, Floyd's rule) from
    the per-episode pre-pass (dqn_sample_prepass_kernel, default) or drawn in each act launch's tail
    (P2PMG_DQN_SAMPLE_PREPASS=0): both bit for bit the oracle."""
    monkeypatch.setenv("P2PMG_DQN_SAMPLE_PREPASS", prepass)
    _episodes_vs_oracle(S, N, R, shared, apb, segments)


@pytest.mark.parametrize("spt", ["4", "2", "8", "16"])
def test_fold_forms_agree_on_long_runs(monkeypatch, spt):
    """Segments of 130 one-agent train workgroups (runs of 9 partials: the fold's 8-load batch and
    its remainder loop; the oracle's per-agent training is too slow at this size): every fold form
    trains the same network bit for bit as the reduce kernel's form (P2PMG_FOLD_SPT=1), which
    test_split_path_forms_match_oracle pins to the oracle."""
    S, N, T = 130, 2, 16
    nets = {}
    for form in ("1", spt):
        monkeypatch.setenv("P2PMG_FOLD_SPT", form)
        inp = scenario_batch(S, N, T)
        eng = DeviceDQNBatch(S, N, 1, T, shared=True, init_seed=5, agents_per_block=1, grad_segments=2)
        eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        eng.set_profiles(inp.load_w, inp.pv_w)
        eng.set_max_in(inp.max_in)
        eng.set_temperatures(inp.t_in0, inp.t_m0)
        for ep, (mode, eps) in enumerate((("fill", 1.0), ("fill", 1.0), ("train", 0.9), ("train", 0.5))):
            eng.run_episode(mode, "philox", episode=ep, epsilon=eps, record=("loss",) if mode == "train" else ())
        nets[form] = [eng.get_weights(k) for k in ("online", "target", "adam_m", "adam_v")] + [eng.get_record("loss")]
        eng.close()
    for a, b, k in zip(nets["1"], nets[spt], ("online", "target", "adam_m", "adam_v", "loss")):
        _eq(b, a, k)
    assert not np.array_equal(nets["1"][0], nets["1"][1])


def _episodes_vs_oracle(S, N, R, shared, apb, segments):
    # the oracle's per-agent Python loops bound the larger communities: T = 16 there, two fill episodes
    # (the 31 transitions training needs, rl.py:234-235) and one training episode
    big = N not in (1, 2, 3, 4, 5, 6, 7, 8, 16)
    T = 16 if big else 48
    eng, ob = _pair(S, N, R, T, shared, apb=apb, segments=segments)
    th0 = ob.theta.copy()
    ep = 0
    plan = (("fill", 1.0), ("fill", 1.0), ("train", 0.9)) if big else (("fill", 1.0), ("train", 0.9), ("train", 0.3))
    for mode, eps in plan:
        eng.run_episode(mode, "philox", episode=ep, epsilon=eps,
                        record=("reward", "cost", "grid", "p2p", "t_in", "action", "loss"))
        out = ob.run_episode(mode, rng="philox", episode=ep, eps=eps)
        _compare_episode(eng, out, mode, eps)
        buf, added = eng.get_buffer()
        assert np.array_equal(added, ob.added.ravel())
        assert np.array_equal(buf[:, :int(added.min())], ob.buf.reshape(S * N, -1, 10)[:, :int(added.min())])
        ep += 1
        _reset(eng, ob, ep)
    _check_trained(eng, ob, th0)
    eng.run_episode("greedy", record=("action", "reward"))
    out = ob.run_episode("greedy")
    assert np.array_equal(eng.get_record("action"), out["action"].astype(np.uint8))
    eng.close()


def test_reference_order_replay_thesis_community():
    """S=1, N=2, R=1: exploration from Python's random + np.random.choice and buffer samples from
    random.sample, generated in the reference's consumption order (oracle.dqn.reference_dqn_replay)."""
    S, N, R, T = 1, 2, 1, 96
    eng, ob = _pair(S, N, R, T, False)
    th0 = ob.theta.copy()
    py, npr = random.Random(42), np.random.RandomState(42)
    codes, _ = odqn.reference_dqn_replay(py, npr, T, R, N, 1.0)
    eng.set_replay_codes(codes[:, :, None, :])
    eng.run_episode("fill", "replay", epsilon=1.0, record=("action",))
    ob.run_episode("fill", codes=codes[:, :, None, :], rng="replay")
    codes, samples = odqn.reference_dqn_replay(py, npr, T, R, N, 0.9, counts=ob.count().ravel())
    eng.set_replay_codes(codes[:, :, None, :])
    eng.set_samples(samples[:, None])
    eng.run_episode("train", "replay", epsilon=0.9, record=("reward", "cost", "grid", "p2p", "t_in", "action", "loss"))
    out = ob.run_episode("train", codes=codes[:, :, None, :], samples=samples[:, None], rng="replay")
    _compare_episode(eng, out, "train", 0.9)
    _check_trained(eng, ob, th0)
    eng.close()


def test_episode_after_uneven_adam_counts():
    """p2pmg_dqn_train_batch on one network leaves the per-agent Adam counts uneven ([0, 1]);
    the next training episode then uses each network's own bias-corrected step size at every env
    step (one per-episode step-size table on the device) and matches the oracle run with the same
    per-network counts."""
    S, N, R, T = 1, 2, 1, 40
    eng, ob = _pair(S, N, R, T, False)
    th0 = ob.theta.copy()
    z = np.zeros((32, 4), np.float32)
    eng.train_batch(z, np.zeros(32, np.float32), np.zeros(32, np.float32), z, net=1)
    g, _ = odqn.gradients(ob.theta[1:2], z[None], np.zeros((1, 32), np.float32), np.zeros((1, 32), np.float32),
                          z[None], ob.target[1:2], 0.95)
    th1, tg1, m1, v1 = ob.theta[1:2].copy(), ob.target[1:2].copy(), ob.m[1:2].copy(), ob.v[1:2].copy()
    odqn.adam_step(th1, m1, v1, g, 1)
    odqn.soft_update(tg1, th1, 0.005)
    ob.theta[1], ob.target[1], ob.m[1], ob.v[1] = th1[0], tg1[0], m1[0], v1[0]
    ob.step = np.array([0, 1])
    assert list(eng.net_steps()) == [0, 1]
    for ep, (mode, eps) in enumerate((("fill", 1.0), ("train", 0.5), ("train", 0.2))):
        eng.run_episode(mode, "philox", episode=ep, epsilon=eps, record=("reward", "cost", "grid", "p2p", "t_in",
                                                                          "action", "loss"))
        out = ob.run_episode(mode, rng="philox", episode=ep, eps=eps)
        _compare_episode(eng, out, mode, eps)
        _reset(eng, ob, ep + 1)
    assert list(eng.net_steps()) == [2 * T, 2 * T + 1]
    _check_trained(eng, ob, th0)
    eng.close()


def test_replay_samples_past_eviction_match_reference_fixture():
    """The reference-pinned sample stream (tests/golden/dqn_draws.npz: ReplayBuffer.sample_batch
    past the 5000-entry deque eviction, rl.py:207,234-237) drives one replay-mode training episode
    on a full, wrapped ring: the device equals the oracle, and the host view of the device ring
    (rl.ReplayBuffer bound to it) returns exactly the reference's sampled experiences."""
    from conftest import load_golden
    from p2pmicrogrid_amd.rl import ReplayBuffer
    d = load_golden("dqn_draws")
    T, R, N = int(d["T"]), int(d["R"]), int(d["N"])
    F, e = int(d["fill_episodes"]), int(d["keep"][-1])
    added0 = (F + e) * T                      # adds before that training episode (> 5000)
    tags = d[f"sample_tags_{e}"].astype(np.int64)       # [T, N, 32]
    step_added = added0 + np.arange(1, T + 1)
    first = step_added - np.minimum(step_added, 5000)
    idx = (tags - first[:, None, None]).astype(np.uint16)  # deque indices
    eng, ob = _pair(1, N, R, T, False)
    th0 = ob.theta.copy()
    rs = np.random.RandomState(11)
    ring = np.zeros((N, 5000, 10), np.float32)
    ring[..., 0:4] = rs.uniform(-1, 1, (N, 5000, 4))
    ring[..., 4] = odqn.ACTION_VALUES[rs.randint(0, 3, (N, 5000))]
    ring[..., 5] = rs.uniform(-3, 0, (N, 5000))
    ring[..., 6:10] = rs.uniform(-1, 1, (N, 5000, 4))
    eng.set_buffer(ring, np.full(N, added0, np.int32))
    ob.buf[0] = ring
    ob.added[:] = added0
    hb = ReplayBuffer(5000, 32)
    hb.bind(eng, 0)
    codes = d["codes"][F + e][:, :, None, :]
    eng.set_replay_codes(codes)
    eng.set_samples(idx[:, None])
    eng.run_episode("train", "replay", epsilon=float(d["eps"][F + e]),
                    record=("reward", "cost", "grid", "p2p", "t_in", "action", "loss"))
    out = ob.run_episode("train", codes=codes, samples=idx[:, None], rng="replay")
    _compare_episode(eng, out, "train", float(d["eps"][F + e]))
    _check_trained(eng, ob, th0)
    # after the episode the device ring holds added0 + T entries; the deque view is the last 5000
    rows = hb._device_rows()
    buf, added = eng.get_buffer()
    n = int(added[0])
    assert n == added0 + T and len(rows) == 5000
    assert np.array_equal(rows, buf[0][(n - 5000 + np.arange(5000)) % 5000])
    eng.close()


@pytest.mark.parametrize("S,N,R,agw", [(37, 2, 1, 16), (11, 3, 2, 16), (5, 16, 1, 16), (20, 1, 0, 16), (9, 5, 1, 16),
                                      (6, 2, 7, 16), (37, 2, 1, 8), (11, 3, 7, 8), (9, 5, 1, 8)])
def test_shared_act_mfma_kernel_equals_wave_kernel(S, N, R, agw, monkeypatch):
    """A shared network's act launch on MFMA tiles (dqn_act_shared_kernel, 16 or 8 agent slots per
    workgroup (P2PMG_ACT_AGW), partial last workgroup when the slots / N do not divide S, up to the
    8-round maximum) gives bitwise the records, replay rings, sampled slots and trained weights of
    the one-wave-per-agent kernel (P2PMG_DQN_ACT=wave): same fmaf chain over k in layer 2, same
    pairwise tree over the 64 units in layer 3; Philox and replay-mode exploration and replay draws."""
    T = 24
    runs = []
    monkeypatch.setenv("P2PMG_ACT_AGW", str(agw))
    for kind in ("wave", "mfma"):
        if kind == "wave":
            monkeypatch.setenv("P2PMG_DQN_ACT", "wave")
        else:
            monkeypatch.delenv("P2PMG_DQN_ACT", raising=False)
        inp = scenario_batch(S, N, T)
        eng = DeviceDQNBatch(S, N, R, T, shared=True, init_seed=11)
        eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        eng.set_profiles(inp.load_w, inp.pv_w)
        eng.set_max_in(inp.max_in)
        eng.set_temperatures(inp.t_in0, inp.t_m0)
        recs = []
        keys = ("reward", "cost", "grid", "p2p", "t_in", "action")
        for ep, (mode, eps) in enumerate((("fill", 1.0), ("fill", 1.0), ("train", 0.6), ("train", 0.2))):
            eng.run_episode(mode, "philox", episode=ep, epsilon=eps, record=keys + (("loss",) if mode == "train" else ()))
            assert eng.last_kernel().startswith("dqn_act_kernel<" if kind == "wave" else "dqn_act_shared_kernel<")
            recs.append(eng.get_records(list(keys) + (["loss"] if mode == "train" else [])))
            recs.append({"episode_reward": eng.episode_reward()})
            eng.reset_temperatures_philox(ep + 1)
        # a replay-mode training episode: uploaded codes (prefetched as words) and deque samples
        rs = np.random.RandomState(S * 100 + N)
        codes = rs.choice(np.array([0, 1, 2, 255, 255, 255], np.uint8), size=(T, R + 1, S * N))
        samples = np.stack([np.stack([rs.choice(96, 32, replace=False) for _ in range(S * N)]) for _ in range(T)])
        eng.set_replay_codes(codes)
        eng.set_samples(samples)
        eng.run_episode("train", "replay", episode=9, epsilon=0.5, record=keys + ("loss",))
        recs.append(eng.get_records(list(keys) + ["loss"]))
        eng.run_episode("greedy", record=keys)
        recs.append(eng.get_records(list(keys)))
        buf, added = eng.get_buffer()
        runs.append((recs, buf, added, eng.get_weights("online"), eng.get_weights("target")))
        eng.close()
    (ra, ba, aa, tha, tga), (rb, bb, ab, thb, tgb) = runs
    for x, y in zip(ra, rb):
        for k in x:
            assert np.array_equal(np.asarray(x[k]), np.asarray(y[k]), equal_nan=True), k
    assert np.array_equal(aa, ab)
    assert np.array_equal(ba, bb)
    assert np.array_equal(tha, thb) and np.array_equal(tga, tgb)
