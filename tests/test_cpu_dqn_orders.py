"""The DQN gradient in the kernels' summation order against an independent formulation.

`oracle/dqn.train_block` + `fold_segments` restate the order `dqn_train_kernel` and the segment fold
sum in; the GPU tests pin the device to them bit for bit.  `oracle/dqn.gradients` is the independent
check: Trainer._train (rl.py:307-333) up to the optimizer as numpy matmuls, in numpy's own order.
The two must agree at north_star's 1e-5 (relative to each parameter group's largest gradient).
Weight updates are not compared this way: Adam's first steps move each weight by about lr * sign(g),
so a gradient component near zero turns a 1e-7 summation difference into an O(1) relative change
of its update (the GPU tests' 2e-3 / 1e-2 tolerances on updates); the gradients themselves are the
quantity the summation order touches."""
import numpy as np
import pytest

from oracle import dqn as odqn

# parameter groups of the Keras weight order (p2pmg_internal.h kOff*)
GROUPS = {"W1": (0, 320), "b1": (320, 384), "W2": (384, 4480), "b2": (4480, 4544), "W3": (4544, 4608),
          "b3": (4608, 4609)}
TOL = 1e-5


def _batches(rs, n, obs_scale=1.0):
    s = (rs.uniform(-1, 1, (n, 32, 4)) * obs_scale).astype(np.float32)
    ns = (rs.uniform(-1, 1, (n, 32, 4)) * obs_scale).astype(np.float32)
    a = odqn.ACTION_VALUES[rs.randint(0, 3, (n, 32))]
    r = rs.uniform(-3, 0, (n, 32)).astype(np.float32)
    return s, a, r, ns


def _check_groups(got, want, what):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    for name, (lo, hi) in GROUPS.items():
        scale = np.abs(want[..., lo:hi]).max()
        err = np.abs(got[..., lo:hi] - want[..., lo:hi]).max()
        assert err <= TOL * max(scale, 1e-30), f"{what} {name}: max |diff| {err:.3g} vs scale {scale:.3g}"


@pytest.mark.parametrize("seed,obs_scale", [(0, 1.0), (1, 1.0), (2, 3.0), (3, 0.2)])
def test_per_network_gradient_matches_matmul_order(seed, obs_scale):
    """One network per agent (the reference's DQNAgent): the kernel-order block gradient of 8
    networks vs the matmul-order gradient, each network's batch of 32 transitions."""
    rs = np.random.RandomState(seed)
    n = 8
    theta = odqn.glorot_init(n, seed=10 + seed)
    target = odqn.glorot_init(n, seed=20 + seed)
    s, a, r, ns = _batches(rs, n, obs_scale)
    batch = np.concatenate([s, a[..., None], r[..., None], ns], -1)  # [n, 32, 10]
    g, loss = odqn.train_block(theta, target, batch[:, None], 0.95)
    gm, lm = odqn.gradients(theta, s, a, r, ns, target, 0.95)
    _check_groups(g, gm, "per-network")
    assert np.allclose(loss[:, 0], lm, rtol=TOL, atol=0)


@pytest.mark.parametrize("agents,apb", [(128, 16), (96, 5)])
def test_shared_segment_matches_sum_of_matmul_gradients(agents, apb):
    """One shared network (configs[4]): a segment of `agents` agents in train workgroups of `apb`
    (kernel-order partials folded by fold_segments) vs the sum over the same agents of each agent's
    matmul-order gradient, summed in float64."""
    rs = np.random.RandomState(agents)
    th = odqn.glorot_init(1, seed=7)
    tg = odqn.glorot_init(1, seed=8)
    s, a, r, ns = _batches(rs, agents)
    batch = np.concatenate([s, a[..., None], r[..., None], ns], -1)
    _, _, bps, blocks = odqn.block_layout(agents, 1, apb)
    padded = np.zeros((bps * apb, 32, 10), np.float32)
    padded[:agents] = batch
    counts = [n for _, n in blocks]
    partials, _ = odqn.train_block(th[0], tg[0], padded.reshape(bps, apb, 32, 10), 0.95, counts=counts)
    seg = odqn.fold_segments(partials, bps)[0]
    gm, _ = odqn.gradients(np.repeat(th, agents, 0), s, a, r, ns, np.repeat(tg, agents, 0), 0.95)
    _check_groups(seg, gm.astype(np.float64).sum(0), "segment")
