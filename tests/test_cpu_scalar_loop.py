"""CPU tests: the per-object scalar loop (oracle/scalar_loop.py, the reference-shaped CPU baseline)
reproduces the reference-driven loop fixtures bit for bit, and agrees with the vectorised oracle
when it draws its own exploration in the reference's order."""
import numpy as np
import pytest

from conftest import load_golden
from oracle.restatement import OracleBatch, reference_replay_codes
from oracle.scalar_loop import ScalarCommunity, ScalarQAgent


def _community(d, prefix=""):
    N = int(d["N"])
    agents = [ScalarQAgent(d[f"{prefix}load_w"][i], d[f"{prefix}pv_w"][i], d["max_in"][i], 0.0, 0.0) for i in range(N)]
    return ScalarCommunity(agents, d[f"{prefix}env_time"], d[f"{prefix}env_tout"], int(d["R"]),
                           price_table=(d[f"{prefix}buy"], d[f"{prefix}inj"], d[f"{prefix}p2pp"]))


@pytest.mark.parametrize("name", ["loop_thesis_T96", "loop_n5_r2_T96", "loop_homo_T96"])
def test_scalar_loop_reproduces_reference_driven_loop(name):
    d = load_golden(name)
    N, E = int(d["N"]), int(d["E"])
    com = _community(d)
    for e in range(E):
        for i, ag in enumerate(com.agents):
            ag.t_in, ag.t_m = np.float32(d["t_in0"][e][i]), np.float32(d["t_m0"][e][i])
        out = com.train_episode(codes=d["codes"][e])
        for k in ("grid", "p2p", "cost", "reward", "t_in", "t_m", "hp"):
            assert np.array_equal(out[k], d[f"train_{k}"][e]), (name, e, k)
        assert np.array_equal(out["action"], d["train_action"][e])
        assert np.array_equal(out["idx"], d["train_idx"][e])
        qi, qv = d[f"q_idx_{e}"], d[f"q_val_{e}"]
        tabs = np.stack([ag.q for ag in com.agents])
        assert np.count_nonzero(tabs) == len(qv) and np.array_equal(tabs[tuple(qi.T)], qv)
    ev = _community(d, "eval_")
    for i, ag in enumerate(ev.agents):
        ag.q = com.agents[i].q
        ag.t_in, ag.t_m = np.float32(d["eval_t_in0"][i]), np.float32(d["eval_t_m0"][i])
    out = ev.train_episode(training=False)
    for k in ("grid", "p2p", "cost", "reward", "t_in", "hp"):
        assert np.array_equal(out[k], d[f"eval_{k}"]), (name, "eval", k)
    assert np.array_equal(out["action"], d["eval_action"])
    assert N == len(ev.agents)


def test_scalar_loop_own_draws_match_vectorised_oracle():
    """rs-drawn exploration (reference order) == the same draws replayed through OracleBatch."""
    from p2pmicrogrid_amd.dataset import scenario_batch
    N, R, T = 2, 1, 96
    inp = scenario_batch(1, N, T)
    agents = [ScalarQAgent(inp.load_w[0, i], inp.pv_w[0, i], inp.max_in[0, i], inp.t_in0[0, i], inp.t_m0[0, i])
              for i in range(N)]
    com = ScalarCommunity(agents, inp.time, inp.t_out[0], R)
    ob = OracleBatch(S=1, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                     env_time=inp.time[None], env_tout=inp.t_out)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    for e, eps in enumerate((0.81, 0.5)):
        out = com.train_episode(rs=np.random.RandomState(7 + e), eps=eps)
        codes = reference_replay_codes(np.random.RandomState(7 + e), T, R, N, eps)
        want = ob.run_episode("train", codes=codes[:, :, None, :], eps=eps)
        for k in ("grid", "p2p", "cost", "reward", "t_in", "hp"):
            assert np.array_equal(out[k], want[k][:, 0]), (e, k)
        assert out["episode_reward"] == want["episode_reward"][0]
        for i in range(N):
            assert np.array_equal(com.agents[i].q, ob.q_table(i))
        # both carry the end-of-episode temperatures into the next episode
        ob.t_in = np.array([[ag.t_in for ag in com.agents]], np.float32)
        ob.t_m = np.array([[ag.t_m for ag in com.agents]], np.float32)
