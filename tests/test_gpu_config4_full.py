"""configs[3] at the benched shape itself: 8192 scenarios x 4 heterogeneous households, one-year
episodes (T = 35,040), per-agent f64 tables (32,768 tables, 168 GB) — exactly what
``bench.py --workload config4`` launches, here with full records.

- 8 sampled scenarios (addressed by global agent id) are re-run by the oracle over the WHOLE year
  (round 6; rounds 4-5 checked the first 1440 slots): every record of every slot, the final tables,
  SoC, temperatures and episode rewards of those 32 agents, bit for bit;
- the whole year is checked over all 32,768 agents through size-independent properties: finite
  flows, valid actions, SoC bounds, bilateral P2P clearing, and the episode reward recomputed from
  the recorded rewards in the kernel's summation order (community.py:179)."""
import gc
import os

import numpy as np
import pytest

from test_gpu_config4 import YEAR, _device, _oracle_prefix

pytestmark = pytest.mark.gpu


def _picked_inputs(pick, N, T):
    """The sampled scenarios' own inputs (scenario data depend only on (seed, scenario))."""
    from p2pmicrogrid_amd.dataset import apply_asset_mix, asset_mix, scenario_batch
    parts = [apply_asset_mix(scenario_batch(1, N, T, first_scenario=int(s)), asset_mix(1, N, first_scenario=int(s)))
             for s in pick]
    mixes = [asset_mix(1, N, first_scenario=int(s)) for s in pick]

    class _In:
        time = parts[0].time

    inp = _In()
    for k in ("load_w", "pv_w", "max_in", "t_in0", "t_m0", "t_out"):
        setattr(inp, k, np.concatenate([getattr(q, k) for q in parts]))

    class _Mix:
        hp_levels = np.concatenate([m.hp_levels for m in mixes])
        battery_capacity = np.concatenate([m.battery_capacity for m in mixes])

    return inp, _Mix()


@pytest.mark.timeout(1100)
def test_benched_config4_shape_full_year_sampled_and_properties():
    from p2pmicrogrid_amd.dataset import SharedScenarioInputs, asset_mix
    from p2pmicrogrid_amd.engine import unpack_index
    S, N, R, T = 8192, 4, 1, YEAR
    pick = np.sort(np.random.RandomState(3).choice(S, 8, replace=False))
    gids = pick[:, None] * N + np.arange(N)[None, :]
    # the oracle over the whole year for the 8 sampled scenarios (~1 min on one core)
    pin, pmix = _picked_inputs(pick, N, T)
    ob = _oracle_prefix(pin, pmix, np.arange(len(pick)), N, R, T)
    out = ob.run_episode("train", rng="philox", episode=0, eps=0.81, agent_ids=gids)
    # the bench's generator and seed (bench.py WORKLOADS["config4"]), built by a worker pool
    mix = asset_mix(S, N, battery_j=10.0 * 3.6e6)
    workers = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8") or 8)))
    with SharedScenarioInputs(S, N, T, workers, mix=mix) as gen:
        inp = gen.inputs
        for k in ("load_w", "pv_w", "max_in", "t_in0", "t_m0", "t_out"):
            assert np.array_equal(getattr(inp, k)[pick], getattr(pin, k)), k
        eng = _device(inp, mix, S, N, R, T)
        del inp
    gc.collect()
    eng.run_episode("train", "philox", episode=0, epsilon=0.81,
                    record=("reward", "cost", "grid", "p2p", "t_in", "action", "index"))
    assert eng.last_kernel() == "episode_fast_kernel<4,f64,R1=2,train,battery>"
    ep = eng.episode_reward()
    assert np.array_equal(ep[pick], out["episode_reward"])
    # per-step records, one at a time (each [T, S, N] f32 is 4.6 GB): the sampled scenarios over the
    # whole year bit for bit, every scenario through properties
    rew = eng.get_record("reward")
    assert np.array_equal(rew[:, pick], out["reward"])
    assert np.all(np.isfinite(rew))
    acc = np.zeros(S, np.float32)
    for t in range(T):  # avg_reward = sum_t mean_i r: agents in order, then / N, then into the sum
        m = rew[t, :, 0]
        for i in range(1, N):
            m = m + rew[t, :, i]
        acc = acc + m * np.float32(1.0 / N)
    assert np.array_equal(acc, ep)
    del rew
    for k in ("cost", "grid", "t_in"):
        r = eng.get_record(k)
        assert np.array_equal(r[:, pick], out[k]), k
        assert np.all(np.isfinite(r)), k
        del r
    p2p = eng.get_record("p2p")
    assert np.array_equal(p2p[:, pick], out["p2p"])
    tot = np.abs(p2p.sum(axis=-1, dtype=np.float64))
    assert np.all(tot <= 1e-3 * (1 + np.abs(p2p).sum(axis=-1, dtype=np.float64)))
    del p2p
    act = eng.get_record("action")
    assert np.array_equal(act[:, :, pick], out["action"].astype(np.uint8))
    assert act.max() <= 2
    del act
    idx = eng.get_record("index")
    assert np.array_equal(unpack_index(idx[:, :, pick]), out["idx"])
    del idx
    # the state the year leaves behind: temperatures, SoC and the 32 agents' learned tables
    t_in, t_m = eng.get_temperatures()
    assert np.array_equal(t_in[pick], out["t_in_final"]) and np.array_equal(t_m[pick], out["t_m_final"])
    soc = eng.get_soc()
    assert np.array_equal(soc[pick], ob.soc)
    has_bat = mix.battery_capacity > 0
    assert np.all((soc[has_bat] >= 0.1 - 1e-12) & (soc[has_bat] <= 0.9 + 1e-12))
    for k, g in enumerate(gids.ravel()):
        q = eng.get_q(first=int(g), count=1)
        assert np.array_equal(q.reshape(-1, 3), ob.q[k]), ("table", int(g))
    eng.close()
