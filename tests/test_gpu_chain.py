"""Chained launches (p2pmg_run_episodes): the training loop of community.py:279-286 with up to 64
episodes per launch, every wave running its episodes back to back.  A chain must equal the same
episodes launched one by one, bit for bit (Q-tables, final temperatures, every episode's reward),
and the oracle over the same epsilon schedule with the end-of-episode T0 reset (community.py:181).
"""
import numpy as np
import pytest

from oracle import philox
from p2pmicrogrid_amd.dataset import scenario_batch
from test_gpu_parity import _device_for, _oracle_for

pytestmark = pytest.mark.gpu


def _schedule(e0, n):
    return [max(0.1, 0.9 ** e) for e in range(e0, e0 + n)]  # bench.py epsilon_at: the decay to the 0.1 floor


def _singles(eng, e0, eps):
    rew = []
    for k, e in enumerate(range(e0, e0 + len(eps))):
        eng.run_episode("train", "philox", episode=e, epsilon=eps[k], reset_sigma=0.3,
                        next_epsilon=eps[k + 1] if k + 1 < len(eps) else None)
        rew.append(eng.episode_reward())
    return np.stack(rew)


def _same_state(a, b):
    for x, y in zip(a.get_temperatures(), b.get_temperatures()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.episode_reward(), b.episode_reward())
    assert np.array_equal(a.get_q(), b.get_q())


@pytest.mark.parametrize("S,N,R,T,q", [(64, 2, 1, 96, "f64"), (40, 3, 1, 24, "f64"), (33, 2, 1, 10, "f32"),
                                       (16, 4, 1, 12, "f64"), (20, 2, 0, 16, "f64"), (12, 5, 2, 8, "f64")])
def test_chain_equals_single_launches(S, N, R, T, q):
    inp = scenario_batch(S, N, T, seed=31)
    a, b = _device_for(inp, N, R, q), _device_for(inp, N, R, q)
    eps = _schedule(3, 7)
    rew = _singles(a, 3, eps)
    b.run_episodes(3, eps, reset_sigma=0.3)
    assert b.last_kernel().startswith("episode_fast_kernel<"), b.last_kernel()
    assert np.array_equal(b.episode_rewards(), rew)
    _same_state(a, b)


def test_chain_matches_oracle_with_t0_resets():
    S, N, R, T = 48, 2, 1, 48
    inp = scenario_batch(S, N, T, seed=37)
    ob = _oracle_for(inp, N, R)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    eng = _device_for(inp, N, R)
    eps = _schedule(0, 6)
    eng.run_episodes(0, eps, reset_sigma=0.3)
    got = eng.episode_rewards()
    for e in range(6):
        out = ob.run_episode("train", rng="philox", seed=42, episode=e, eps=eps[e])
        assert np.array_equal(got[e], out["episode_reward"]), e
        t_in, t_m = philox.t0_draws(42, e + 1, np.arange(S * N))
        ob.t_in, ob.t_m = t_in.reshape(S, N), t_m.reshape(S, N)
    a, b = eng.get_temperatures()
    assert np.array_equal(a, ob.t_in) and np.array_equal(b, ob.t_m)
    assert np.array_equal(eng.get_q().reshape(S * N, -1, 3), ob.q)


def test_long_chain_splits_and_speculates_the_next_call():
    """70 episodes: two launches (64 + 6); the next call's schedule guessed right (a pre-pass hit)
    and then wrong (a recompute): every result still equals the single launches."""
    S, N, R, T = 8, 2, 1, 6
    inp = scenario_batch(S, N, T, seed=41)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    eps1, eps2, eps3 = _schedule(0, 70), _schedule(70, 5), [0.37] * 4
    r1 = _singles(a, 0, eps1)
    r2 = _singles(a, 70, eps2)
    r3 = _singles(a, 75, eps3)
    b.run_episodes(0, eps1, reset_sigma=0.3, next_epsilons=eps2)
    assert np.array_equal(b.episode_rewards(), r1)
    h0, m0 = b.prepass_stats()
    b.run_episodes(70, eps2, reset_sigma=0.3, next_epsilons=[0.5] * 4)
    h1, m1 = b.prepass_stats()
    assert (h1 - h0, m1 - m0) == (1, 0)
    assert np.array_equal(b.episode_rewards(), r2)
    b.run_episodes(75, eps3, reset_sigma=0.3)
    h2, m2 = b.prepass_stats()
    assert (h2 - h1, m2 - m1) == (0, 1)
    assert np.array_equal(b.episode_rewards(), r3)
    _same_state(a, b)


def test_chain_without_reset_and_after_single_launches():
    """No T0 reset (temperatures carry over between episodes), interleaved with single launches;
    the per-episode rewards of a chain are only readable until the next single launch."""
    from p2pmicrogrid_amd._lib import P2PMGError
    S, N, R, T = 24, 2, 1, 20
    inp = scenario_batch(S, N, T, seed=43)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    for e in range(2):
        a.run_episode("train", "philox", episode=e, epsilon=0.6)
        b.run_episode("train", "philox", episode=e, epsilon=0.6)
    for e in range(2, 6):
        a.run_episode("train", "philox", episode=e, epsilon=0.4)
    b.run_episodes(2, [0.4] * 4)
    _same_state(a, b)
    assert b.episode_rewards().shape == (4, S)
    a.run_episode("train", "philox", episode=6, epsilon=0.4)
    b.run_episode("train", "philox", episode=6, epsilon=0.4)
    _same_state(a, b)
    with pytest.raises(P2PMGError):
        b.episode_rewards()


def test_fallback_where_the_fast_kernel_does_not_apply():
    """N = 16 per-agent tables run the general kernel: run_episodes launches episode by episode."""
    S, N, R, T = 4, 16, 1, 8
    inp = scenario_batch(S, N, T, seed=47)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    eps = _schedule(1, 3)
    rew = _singles(a, 1, eps)
    b.run_episodes(1, eps, reset_sigma=0.3)
    assert b.last_kernel().startswith("episode_kernel<"), b.last_kernel()
    assert np.array_equal(b.episode_rewards(), rew)
    _same_state(a, b)


@pytest.mark.parametrize("record", [("reward", "cost"), ("reward", "cost", "grid", "p2p", "t_in", "action", "index")])
def test_chain_leaves_the_last_episodes_records(record):
    S, N, R, T = 32, 2, 1, 24
    inp = scenario_batch(S, N, T, seed=53)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    eps = _schedule(4, 5)
    for k, e in enumerate(range(4, 9)):
        a.run_episode("train", "philox", episode=e, epsilon=eps[k], reset_sigma=0.3, record=record)
    b.run_episodes(4, eps, reset_sigma=0.3, record=record)
    ra, rb = a.get_records(record), b.get_records(record)
    for k in record:
        assert np.array_equal(ra[k], rb[k]), k
    _same_state(a, b)


def test_sharded_trainer_train_episodes_equals_episode_loop():
    """ShardedTrainer.train_episodes (chained launches) against its train_episode loop (one launch and
    a separate T0 reset per episode): the same global means, tables and temperatures."""
    from p2pmicrogrid_amd.distributed import ShardedTrainer
    a = ShardedTrainer(40, 2, 1, 24)
    b = ShardedTrainer(40, 2, 1, 24)
    eps = _schedule(0, 6)
    m1 = [a.train_episode(e) for e in eps]
    m2 = b.train_episodes(eps)
    assert np.array_equal(np.array(m1), m2)
    _same_state(a.eng, b.eng)
    assert a.episode == b.episode == 6


def test_low_epsilon_wave_split_keeps_results():
    """configs[1]'s batch (4096 scenarios: one wave per CU) below epsilon 0.5 runs half-filled waves
    (two per CU): the same tables, temperatures and rewards as one full wave per CU."""
    S, N, R, T = 4096, 2, 1, 12
    inp = scenario_batch(S, N, T, seed=59)
    eng = _device_for(inp, N, R)
    out = []
    for spw in (0, 16):
        eng.zero_q()
        eng.set_temperatures(inp.t_in0, inp.t_m0)
        eng.run_episodes(0, [0.3, 0.3, 0.3], reset_sigma=0.3, scen_per_wave=spw)
        out.append((eng.episode_rewards(), eng.get_temperatures(), eng.get_q(first=0, count=64),
                    eng.get_q(first=S * N - 64, count=64)))
    for x, y in zip(out[0], out[1]):
        if isinstance(x, tuple):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)
        else:
            assert np.array_equal(x, y)


def test_full_size_chain_equals_single_launches():
    """configs[1] at full size (4096 scenarios, T = 96) over the bench's schedule: a 50-episode chain
    (epsilon 0.729) and a 20-episode chain below epsilon 0.5 (half-filled waves) equal the same
    episodes launched one by one: every episode's rewards, temperatures, and the whole tables'
    fingerprints."""
    import bench
    S, N, R, T = 4096, 2, 1, 96
    inp = scenario_batch(S, N, T)
    a, b = _device_for(inp, N, R), _device_for(inp, N, R)
    for e0, n in ((1, 50), (251, 20)):
        eps = [bench.epsilon_at(e) for e in range(e0, e0 + n)]
        rew = _singles(a, e0, eps)
        b.run_episodes(e0, eps, reset_sigma=0.3)
        assert np.array_equal(b.episode_rewards(), rew), e0
        for x, y in zip(a.get_temperatures(), b.get_temperatures()):
            assert np.array_equal(x, y)
    assert np.array_equal(a.table_hash_allgather(), b.table_hash_allgather())
    a.close()
    b.close()
