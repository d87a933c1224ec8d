"""configs[3] on the device: heterogeneous households (Consumers without PV, no / 3 kW / 5 kW heat
pumps, battery or NoStorage; dataset.asset_mix) over ONE-YEAR episodes (T = 35,040 slots) with
per-agent f64 tables, the shape `bench.py --workload config4` measures.

The oracle cannot replay a whole year in test time (~1.5 ms of NumPy per step), so:
- the first PREFIX slots of the year are compared bit-for-bit with the oracle run on the same
  inputs cut to PREFIX slots (everything recorded at step t depends only on steps <= t; only the
  TD target of the oracle's last step reads its wrapped row 0, and that is never recorded), on
  sampled scenarios addressed by their global agent ids;
- the whole year is checked through size-independent properties over every scenario."""
import numpy as np
import pytest

from oracle.restatement import OracleBatch

pytestmark = pytest.mark.gpu
REC = ["reward", "cost", "grid", "p2p", "t_in", "action", "index"]
YEAR = 365 * 96
PREFIX = 1440  # 15 days


def _inputs(S, N, T, seed=42):
    from p2pmicrogrid_amd.dataset import apply_asset_mix, asset_mix, scenario_batch
    mix = asset_mix(S, N, seed=seed)
    return apply_asset_mix(scenario_batch(S, N, T, seed=seed), mix), mix


def _device(inp, mix, S, N, R, T):
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    eng = DeviceCommunityBatch(S, N, R, T, q_dtype="f64")
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    eng.set_temperatures(inp.t_in0, inp.t_m0)
    eng.set_hp_levels(mix.hp_levels)
    eng.set_battery(mix.battery_capacity, 0.1, 0.9, 0.9)
    return eng


def _oracle_prefix(inp, mix, pick, N, R, T):
    sl = lambda a: np.ascontiguousarray(a[pick])  # noqa: E731
    ob = OracleBatch(S=len(pick), N=N, R=R, load_w=sl(inp.load_w)[..., :T], pv_w=sl(inp.pv_w)[..., :T],
                     max_in=sl(inp.max_in), env_time=inp.time[None, :T], env_tout=sl(inp.t_out)[:, :T],
                     q_dtype="f64", hp_levels=sl(mix.hp_levels), battery_capacity=sl(mix.battery_capacity))
    ob.t_in, ob.t_m = sl(inp.t_in0).copy(), sl(inp.t_m0).copy()
    return ob


def test_mix_covers_every_asset_class():
    _, mix = _inputs(256, 4, 96)
    assert (~mix.has_pv).any() and mix.has_pv.any()
    hp = mix.hp_levels[..., 2]
    assert (hp == 0).any() and (hp == 3000).any() and (hp == 5000).any()
    assert (mix.battery_capacity == 0).any() and (mix.battery_capacity > 0).any()


def test_year_episode_prefix_bit_exact_and_properties():
    from p2pmicrogrid_amd.engine import unpack_index
    S, N, R, T = 128, 4, 1, YEAR
    inp, mix = _inputs(S, N, T)
    eng = _device(inp, mix, S, N, R, T)
    pick = np.sort(np.random.RandomState(1).choice(S, 12, replace=False))
    ob = _oracle_prefix(inp, mix, pick, N, R, PREFIX)
    gids = pick[:, None] * N + np.arange(N)[None, :]
    eng.run_episode("train", "philox", episode=0, epsilon=0.81, record=REC)
    rec = eng.get_records(REC)
    assert eng.last_kernel() == "episode_fast_kernel<4,f64,R1=2,train,battery>"
    out = ob.run_episode("train", rng="philox", episode=0, eps=0.81, agent_ids=gids)
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert np.array_equal(rec[k][:PREFIX, pick], out[k]), k
    assert np.array_equal(rec["action"][:PREFIX, :, pick], out["action"].astype(np.uint8))
    assert np.array_equal(unpack_index(rec["index"][:PREFIX, :, pick]), out["idx"])
    # whole year, every scenario
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        assert np.all(np.isfinite(rec[k])), k
    assert np.all(rec["action"] <= 2)
    no_hp = mix.hp_levels[..., 2] == 0
    assert np.all(rec["action"][:, :, no_hp] <= 2)
    soc = eng.get_soc()
    has_bat = mix.battery_capacity > 0
    assert np.all((soc[has_bat] >= 0.1 - 1e-12) & (soc[has_bat] <= 0.9 + 1e-12))
    # the P2P market clears bilaterally: what a scenario imports from peers, its peers export
    assert np.all(np.abs(rec["p2p"].sum(axis=-1)) <= 1e-3 * (1 + np.abs(rec["p2p"]).sum(axis=-1)))
    # a greedy year afterwards is deterministic: two runs agree bit-for-bit
    t0, soc0 = eng.get_temperatures(), eng.get_soc()
    eng.run_episode("greedy", record=("reward", "action"))
    g1 = eng.get_records(("reward", "action"))
    eng.set_temperatures(*t0)
    eng.set_battery(mix.battery_capacity, 0.1, 0.9, 0.9, soc0=soc0)
    eng.run_episode("greedy", record=("reward", "action"))
    g2 = eng.get_records(("reward", "action"))
    assert all(np.array_equal(g1[k], g2[k]) for k in g1)
    eng.close()


def test_year_fast_kernel_equals_general_kernel():
    """The whole year, every scenario: the fast kernel's battery variant and the general
    episode_kernel (in-kernel Philox draws) give the same records, SoC, temperatures and tables."""
    S, N, R, T = 64, 4, 1, YEAR
    inp, mix = _inputs(S, N, T, seed=7)
    res = []
    for kern, phil in (("auto", "auto"), ("general", "inkernel")):
        eng = _device(inp, mix, S, N, R, T)
        for e in range(2):
            eng.run_episode("train", "philox", episode=e, epsilon=0.5, record=REC, kernel=kern, philox=phil)
        res.append((eng.last_kernel(), eng.get_records(REC), eng.get_soc(), eng.get_temperatures(),
                    eng.get_q(first=0, count=8)))
        eng.close()
    (k0, r0, s0, t0, q0), (k1, r1, s1, t1, q1) = res
    assert k0.startswith("episode_fast_kernel") and k1.startswith("episode_kernel")
    for k in REC:
        assert np.array_equal(r0[k], r1[k]), k
    assert np.array_equal(s0, s1) and np.array_equal(q0, q1)
    assert all(np.array_equal(a, b) for a, b in zip(t0, t1))
