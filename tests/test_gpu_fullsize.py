"""The bench workloads at their FULL per-GPU size (BASELINE.json configs[2] and configs[4]), on the
kernels the bench runs, checked two ways: against another device path over EVERY scenario, and
against the oracle on sampled scenarios (by global scenario id: the Philox counters and the
scenario data depend only on the id, so a sampled subset is an independent problem).

  configs[2]: 125,000 scenarios x 16 agents, battery, ONE shared f32 table (episode_sq16_kernel)
              == the general episode_kernel on all 2M agents (records, int64 deltas, SoC, T),
              32 sampled scenarios == oracle (the shared table is frozen per episode, so a
              scenario's episode depends on the table and its own inputs only).
  configs[4]: 4096 scenarios x 2 DQN agents.  Per-agent networks: 8 sampled scenarios == oracle
              (actions and simulation exact, losses and weights within the f32 tolerance of
              tests/test_gpu_dqn.py).  One shared network: whole-batch properties and bit-identical
              results of two identical contexts (deterministic gradient reduction)."""
import numpy as np
import pytest

from oracle import dqn as odqn
from oracle.restatement import OracleBatch

pytestmark = pytest.mark.gpu
F32 = np.float32
BATTERY_J = 10.0 * 3.6e6


def _engine(inp, S, N, R, T, kernel_q, shared, battery):
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype=kernel_q, shared_q=shared)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    if battery:
        eng.set_battery(BATTERY_J)
    return eng


def test_full_size_config3_sq16_vs_general_and_sampled_oracle():
    from p2pmicrogrid_amd.dataset import scenario_batch
    from p2pmicrogrid_amd.engine import unpack_index
    S, N, R, T = 125000, 16, 1, 96
    inp = scenario_batch(S, N, T)
    a = _engine(inp, S, N, R, T, "f32", True, True)
    b = _engine(inp, S, N, R, T, "f32", True, True)
    pick = np.sort(np.random.RandomState(1).choice(S, 32, replace=False))
    ob = OracleBatch(S=len(pick), N=N, R=R, load_w=inp.load_w[pick], pv_w=inp.pv_w[pick], max_in=inp.max_in[pick],
                     env_time=inp.time[None], env_tout=inp.t_out[pick], q_dtype="f32", shared_q=True,
                     battery_capacity=np.full((len(pick), N), BATTERY_J))
    ob.t_in, ob.t_m = inp.t_in0[pick].copy(), inp.t_m0[pick].copy()
    gids = pick[:, None] * N + np.arange(N)[None, :]
    del inp
    rec = ("reward", "cost", "t_in", "action", "index")
    for e, eps in enumerate((0.81, 0.729)):
        a.run_episode("train", "philox", episode=e, epsilon=eps, record=rec)
        b.run_episode("train", "philox", episode=e, epsilon=eps, record=rec, kernel="general")
        assert "sq16" in a.last_kernel() and "sq16" not in b.last_kernel()
        for k in rec:  # every agent-step of both kernels
            x, y = a.get_record(k), b.get_record(k)
            assert np.array_equal(x, y), (e, k)
            if k != "index":
                del y
        assert np.array_equal(a.get_q_delta(), b.get_q_delta()), e
        assert np.array_equal(a.get_soc(), b.get_soc()), e
        assert np.array_equal(a.episode_reward(), b.episode_reward()), e
        for u, v in zip(a.get_temperatures(), b.get_temperatures()):
            assert np.array_equal(u, v), e
        # the sampled scenarios on the oracle, from the device's (frozen) table of this episode
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=eps, agent_ids=gids)
        rw, cost, tin = (a.get_record(k)[:, pick] for k in ("reward", "cost", "t_in"))
        assert np.array_equal(rw, out["reward"]) and np.array_equal(cost, out["cost"]), e
        assert np.array_equal(tin, out["t_in"]), e
        assert np.array_equal(a.get_record("action")[:, :, pick], out["action"].astype(np.uint8)), e
        assert np.array_equal(unpack_index(x[:, :, pick]), out["idx"]), e
        assert np.array_equal(a.get_soc()[pick], ob.soc), e
        a.apply_q_delta()
        b.apply_q_delta()
        qa = a.get_q(dtype=np.float32)
        assert np.array_equal(qa, b.get_q(dtype=np.float32))
        ob.q[0] = qa.reshape(ob.q[0].shape)  # the next episode reads the table all scenarios built
        ob.q_delta[:] = 0
    a.close()
    b.close()


def _dqn(inp, S, N, R, T, shared, init_seed=0):
    from p2pmicrogrid_amd.dqn import DeviceDQNBatch
    eng = DeviceDQNBatch(S, N, R, T, shared=shared, init_seed=init_seed)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    return eng


def _rel_close(got, want, rtol, floor=1e-3):
    want = np.asarray(want, np.float64)
    scale = np.maximum(np.abs(want), floor * np.abs(want).max())
    err = np.abs(np.asarray(got, np.float64) - want) / scale
    assert err.max() <= rtol, f"max rel err {err.max():.3g}"


def test_full_size_config5_dqn_per_agent_sampled_oracle():
    from p2pmicrogrid_amd.dataset import scenario_batch
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    eng = _dqn(inp, S, N, R, T, shared=False)
    pick = np.sort(np.random.RandomState(2).choice(S, 8, replace=False))
    agents = (pick[:, None] * N + np.arange(N)[None, :]).ravel()
    th0 = eng.get_weights("online")
    ob = odqn.OracleDQNBatch(S=len(pick), N=N, R=R, load_w=inp.load_w[pick], pv_w=inp.pv_w[pick],
                             max_in=inp.max_in[pick], env_time=inp.time[None], env_tout=inp.t_out[pick],
                             theta0=th0[agents], shared=False)
    ob.t_in, ob.t_m = inp.t_in0[pick].copy(), inp.t_m0[pick].copy()
    rec = ("reward", "cost", "grid", "p2p", "t_in", "action")
    for e, (mode, eps) in enumerate((("fill", 1.0), ("train", 0.9))):
        eng.run_episode(mode, "philox", episode=e, epsilon=eps, record=rec + (("loss",) if mode == "train" else ()))
        out = ob.run_episode(mode, rng="philox", episode=e, eps=eps, agent_ids=agents)
        got = eng.get_records(rec)
        assert np.array_equal(got["action"][:, :, pick], out["action"].astype(np.uint8)), e
        for k in ("reward", "cost", "grid", "p2p", "t_in"):
            assert np.array_equal(got[k][:, pick], out[k]), (e, k)
        if mode == "train":
            # the kernel-order oracle: losses bit for bit
            assert np.array_equal(eng.get_record("loss")[:, pick], out["loss"])
            # properties over every agent of the batch
            assert np.all(np.isfinite(eng.get_record("loss")))
        assert np.all(got["action"] <= 2) and np.all(got["p2p"].sum(axis=-1) == 0)
    th = eng.get_weights("online")[agents]
    assert np.array_equal(th, ob.theta) and np.array_equal(eng.get_weights("adam_v")[agents], ob.v)
    _rel_close(th - th0[agents], ob.theta - th0[agents], rtol=1e-2, floor=1e-2)
    eng.close()


def test_full_size_config5_shared_gradient_segments_against_oracle():
    """The benched configs[4] shape (4096 x 2 agents, ONE shared network, 16 agents per train
    workgroup) at its first training env step: the gradient segments the device hands to the exchange
    (p2pmg_dqn_set_exchange) are compared bit for bit with oracle/dqn.train_block + fold_segments over
    the same agents, batches rebuilt from the device's replay rings (get_buffer) with the Philox
    sample draws.  64 segments of 128 agents: the train workgroups are the bench layout's (blocks of
    16 agents never straddle a segment), two sampled segments are re-run by the oracle."""
    from p2pmicrogrid_amd.dataset import scenario_batch
    from p2pmicrogrid_amd.dqn import DeviceDQNBatch
    from oracle import philox
    S, N, R, T, G, APB = 4096, 2, 1, 96, 64, 16
    inp = scenario_batch(S, N, T)
    eng = DeviceDQNBatch(S, N, R, T, shared=True, init_seed=0, grad_segments=G, agents_per_block=APB)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    assert eng.grad_layout() == {"segments": G, "agents_per_block": APB, "blocks": S * N // APB}
    th0 = eng.get_weights("online")[0]
    eng.run_episode("fill", "philox", episode=0, epsilon=1.0)
    eng.reset_temperatures_philox(1, 0.3)
    captured = []

    def capture(rows):  # rows [2, G * stride]: this context's segments in row 0 (world 2: the split path)
        if not captured:
            captured.append(rows[0].copy())
        rows[1] = 0.0

    eng.set_grad_exchange(capture, 0, 2)
    eng.run_episode("train", "philox", episode=1, epsilon=0.9)
    eng.sync()
    assert captured, "the exchange was not called"
    stride = captured[0].size // G
    segs = captured[0].reshape(G, stride)[:, :odqn.N_PARAMS]
    assert np.all(np.isfinite(segs)) and np.any(segs != 0)
    seg_agents = S * N // G
    for g in (0, 37):
        first = g * seg_agents
        ring, added = eng.get_buffer(first, seg_agents)
        assert np.all(added == T + T)  # 96 fill + 96 train transitions, no eviction (capacity 5000)
        # step 0 of the training episode: 97 transitions (the fill + the step's own), deque = ring slots
        idx = philox.sample_draws(42, 1, np.arange(first, first + seg_agents), 0, np.full(seg_agents, T + 1), 32)
        b = ring[np.arange(seg_agents)[:, None], idx]  # [agents, 32, 10]
        _, _, bps, blocks = odqn.block_layout(seg_agents, 1, APB)
        partials, _ = odqn.train_block(th0, th0, b.reshape(bps, APB, 32, 10), 0.95)
        want = odqn.fold_segments(partials, bps)[0]
        assert np.array_equal(segs[g], want), f"segment {g}: max |diff| {np.abs(segs[g] - want).max()}"
        # independent: the sum of the same agents' matmul-order gradients (rl.py:307-333 as numpy
        # matmuls), within north_star's 1e-5 of each parameter group's scale (test_cpu_dqn_orders.py)
        th_n = np.repeat(th0[None], seg_agents, 0)
        gm, _ = odqn.gradients(th_n, b[..., 0:4], b[..., 4], b[..., 5], b[..., 6:10], th_n, 0.95)
        gsum = gm.astype(np.float64).sum(0)
        for lo, hi in ((0, 320), (320, 384), (384, 4480), (4480, 4544), (4544, 4608), (4608, 4609)):
            err = np.abs(segs[g][lo:hi] - gsum[lo:hi]).max()
            assert err <= 1e-5 * np.abs(gsum[lo:hi]).max(), (g, lo, hi, err)
    eng.close()


def test_full_size_config5_dqn_shared_network_properties(monkeypatch):
    """The benched configs[4] shape: engine a acts with the MFMA act kernel (16 agents per
    workgroup), engine b with the one-wave-per-agent kernel (P2PMG_DQN_ACT=wave, checked against the
    oracle at small S): every record, the replay draws behind the trained weights and the weights
    themselves agree bit for bit over all 8,192 agents (and the deterministic gradient reduction)."""
    from p2pmicrogrid_amd.dataset import scenario_batch
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    a = _dqn(inp, S, N, R, T, shared=True)
    b = _dqn(inp, S, N, R, T, shared=True)
    w0 = a.get_weights("online")
    for e, (mode, eps) in enumerate((("fill", 1.0), ("train", 0.9), ("train", 0.81))):
        for x in (a, b):
            if x is b:
                monkeypatch.setenv("P2PMG_DQN_ACT", "wave")
            x.run_episode(mode, "philox", episode=e, epsilon=eps, record=("reward", "p2p", "action"))
            monkeypatch.delenv("P2PMG_DQN_ACT", raising=False)
            x.reset_temperatures_philox(e + 1, 0.3)
        assert a.last_kernel() == "dqn_act_shared_kernel<2>" and b.last_kernel() == "dqn_act_kernel<2>"
        ra, rb = a.get_records(("reward", "p2p", "action")), b.get_records(("reward", "p2p", "action"))
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), (e, k)  # same Q values, draws and reduction: same bits
        assert np.all(np.isfinite(ra["reward"])) and np.all(ra["action"] <= 2)
        assert np.all(ra["p2p"].sum(axis=-1) == 0)  # N = 2: the P2P exchange is antisymmetric
    wa, wb = a.get_weights("online"), b.get_weights("online")
    assert np.array_equal(wa, wb) and np.all(np.isfinite(wa))
    assert not np.array_equal(wa, w0)  # 2 x 96 Adam steps moved the network
    assert a.step == 2 * T
    b.close()
    # 8 sampled scenarios of a greedy day of the full-size launch against the kernel-order oracle
    # (ActorModel.greedy_action's Q values, act_q), with the network the full batch trained
    pick = np.sort(np.random.RandomState(5).choice(S, 8, replace=False))
    t_in, t_m = (x.reshape(S, N) for x in a.get_temperatures())
    ob = odqn.OracleDQNBatch(S=len(pick), N=N, R=R, load_w=inp.load_w[pick], pv_w=inp.pv_w[pick],
                             max_in=inp.max_in[pick], env_time=inp.time[None], env_tout=inp.t_out[pick],
                             theta0=wa, shared=True)
    ob.t_in, ob.t_m = t_in[pick].copy(), t_m[pick].copy()
    keys = ("reward", "cost", "grid", "p2p", "t_in", "action")
    a.run_episode("greedy", record=keys)
    got = a.get_records(keys)
    out = ob.run_episode("greedy")
    assert np.array_equal(got["action"][:, :, pick], out["action"].astype(np.uint8))
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert np.array_equal(got[k][:, pick], out[k]), k
    a.close()
