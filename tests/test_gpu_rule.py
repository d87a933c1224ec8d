"""RuleAgent communities on the device (rule_episode_kernel) vs the oracle, bit-exact.
Reference: get_rule_based_community community.py:237-238, RuleAgent agent.py:106-136, run()
community.py:95-123.  The TF market glue is restated (TF absent); the heating
model the oracle uses is pinned by the reference's own temperature_simulation fixtures."""
import numpy as np
import pytest

from oracle.restatement import OracleBatch

pytestmark = pytest.mark.gpu
REC = ("cost", "grid", "p2p", "t_in", "action")


@pytest.mark.parametrize("S,N,T", [(37, 1, 96), (37, 2, 96), (21, 5, 50), (9, 16, 96), (11, 8, 30), (5, 3, 96)])
def test_rule_episode_matches_oracle(S, N, T):
    from p2pmicrogrid_amd.dataset import scenario_batch
    from p2pmicrogrid_amd.engine import DeviceCommunityBatch
    inp = scenario_batch(S, N, T, seed=11)
    eng = DeviceCommunityBatch(S, N, 0, T)
    eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
    eng.set_profiles(inp.load_w, inp.pv_w)
    eng.set_max_in(inp.max_in)
    rs = np.random.RandomState(S + N)
    t0 = (20.0 + 2.0 * rs.rand(S, N)).astype(np.float32)  # straddle the comfort band
    eng.set_temperatures(t0, t0)
    ob = OracleBatch(S=S, N=N, R=0, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                     env_time=inp.time[None], env_tout=inp.t_out)
    ob.t_in, ob.t_m = t0.copy(), t0.copy()
    on = (rs.rand(S, N) < 0.5).astype(np.int64)
    eng.set_hp_state(on.astype(np.float32))
    for run in range(2):  # the heat-pump state carries over between runs
        eng.run_rule_episode(record=REC)
        assert eng.last_kernel().startswith("rule_episode_kernel")
        out = ob.run_rule_episode(on)
        on = out["hp_on"]
        r = eng.get_records(REC)
        for k in ("cost", "grid", "p2p", "t_in"):
            assert np.array_equal(r[k], out[k]), (run, k)
        assert np.array_equal(r["action"][:, 0], np.where(out["on"] == 1, 2, 0).astype(np.uint8)), run
        assert np.array_equal(eng.get_hp_state(), on.astype(np.float32))
        ti, tm = eng.get_temperatures()
        assert np.array_equal(ti, ob.t_in) and np.array_equal(tm, ob.t_m)
    eng.close()


def test_rule_based_community_run_matches_oracle():
    from p2pmicrogrid_amd.community import get_rule_based_community
    from p2pmicrogrid_amd.environment import env
    np.random.seed(42)
    com = get_rule_based_community(2, homogeneous=False)
    T = len(env)
    t_in0 = np.array([[a.heating.temperature[0] for a in com.agents]], np.float32)
    t_m0 = np.array([[a.heating.building_mass_temperature[0] for a in com.agents]], np.float32)
    load = np.stack([a.load_series(T) for a in com.agents])[None]
    pv = np.stack([a.pv.series(T) for a in com.agents])[None]
    time_f, t_out = env.arrays()
    from p2pmicrogrid_amd.engine import price_table
    ob = OracleBatch(S=1, N=2, R=0, load_w=load, pv_w=pv, max_in=np.array([[a.max_in for a in com.agents]]),
                     env_time=np.asarray(time_f).reshape(1, -1), env_tout=np.asarray(t_out).reshape(1, -1),
                     price_table=price_table(time_f))
    ob.t_in, ob.t_m = t_in0.copy(), t_m0.copy()
    power, cost = com.run()
    out = ob.run_rule_episode(np.zeros((1, 2), np.int64))
    assert np.array_equal(cost, out["cost"][:, 0]) and np.array_equal(power, (out["grid"] + out["p2p"])[:, 0])
    assert np.array_equal(com.decisions[:, 0], out["hp"][:, 0])
    assert [a.heating.hp.power for a in com.agents] == [float(x) for x in out["hp_on"][0]]
