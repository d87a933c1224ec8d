"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own code.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    python -B tests/golden/make_golden.py

What is executed from the reference (``/root/reference/microgrid``, imported read-only with
``sys.dont_write_bytecode``; TensorFlow is absent, so ``tensorflow`` is replaced by a
MagicMock that none of the functions below ever calls — SURVEY.md §8c):

  * ``heating.temperature_simulation``     (heating.py:37-56)   -> heating.npz
  * ``rl.QActor._get_state_indices``       (rl.py:89-95)        -> qactor_idx.npz
  * ``rl.QActor.select_action/train/...``  (rl.py:100-132)      -> qactor_seq.npz, loop_*.npz
  * ``storage.BatteryStorage``             (storage.py:36-76)   -> battery.npz
  * ``rl.ActorModel.select_action`` + ``rl.ReplayBuffer.add/sample_batch`` (rl.py:173-244) in the
    DQN community's call order                              -> dqn_draws.npz
  * ``dataset.get_*_data``/``dataframe_to_dataset`` (dataset.py:39-103, database.py:128-147) on a
    small SQLite file in the reference schema                -> dataset.npz
  * the legacy global ``np.random`` stream in the reference's consumption order (§3.5)

The community glue that calls TF ops (agent.py:172-232, community.py:45-93,149-188) is
restated here per-agent/per-scalar in reference shape (``HybridCommunity``); the vectorised
oracle (oracle/restatement.py) is a second, independent restatement checked against it.
Only data (inputs and outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import os
import sys
import types
import warnings
from unittest.mock import MagicMock

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/microgrid"
F32 = np.float32
GREEDY = 255


def import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("tensorflow", MagicMock())
    sys.modules.setdefault("tensorflow.keras", MagicMock())
    sys.modules.setdefault("config", types.SimpleNamespace(DB_FILE="none.db", DATA_PATH="/tmp",
                                                          FIGURES_PATH="/tmp"))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import heating, rl, storage, setup  # noqa: E401
    return heating, rl, storage, setup


class Wrap:
    """Stands in for an eager tensor handed to QActor: only ``.numpy()`` is used (rl.py:114,120,127)."""

    def __init__(self, x):
        self.x = np.asarray(x, dtype=F32)

    def numpy(self):
        return self.x


# ---------------------------------------------------------------- synthetic data (schema of dataset.py)
def synthetic_days(n_days: int, seed: int = 2021):
    """Normalised profiles with the reference schema: time = slot/96 (dataset.py:43-44),
    temperature in degC, pv and l0..l4 normalised by their max (dataset.py:46-50)."""
    rs = np.random.RandomState(seed)
    T = 96 * n_days
    slot = np.arange(T) % 96
    time = slot / 96.0
    hour = slot / 4.0
    day = np.arange(T) // 96
    temp = 10.0 + 5.0 * np.sin(2 * np.pi * (hour - 9.0) / 24.0) + rs.normal(0, 1.0, T) + 0.5 * day
    pv = np.clip(np.sin(np.pi * (hour - 7.0) / 10.0), 0, None) * (0.6 + 0.4 * rs.rand(n_days)[day])
    pv = pv / pv.max()
    loads = []
    for k in range(5):
        m = 0.25 + 0.35 * np.exp(-((hour - (7.5 + k * 0.3)) ** 2) / 2.0) \
            + 0.6 * np.exp(-((hour - (19.0 + 0.25 * k)) ** 2) / 3.0) + 0.15 * rs.rand(T)
        loads.append(m / m.max())
    return time, temp, pv, np.stack(loads)


def price_table(time_f32):
    """GridAgent.take_decision (agent.py:59-67) with f32 constants; numpy f32 sin."""
    freq = F32(2 * np.pi * 24 / 12)
    s = np.sin(time_f32 * freq - F32(3)).astype(F32)
    buy = ((F32(12.0) + F32(5.0) * s) / F32(100)).astype(F32)
    inj = np.full_like(buy, F32(0.07))
    p2p = ((buy + inj) / F32(2)).astype(F32)
    return buy, inj, p2p


# ---------------------------------------------------------------- hybrid reference-shaped loop
class HybridCommunity:
    """Reference-shaped per-agent loop: QActor and temperature_simulation are the reference's,
    the TF glue is restated scalar-by-scalar following agent.py / community.py."""

    def __init__(self, rl, heating, N, R, homogeneous, norm_load, norm_pv, time, tout):
        self.rl, self.heating, self.N, self.R = rl, heating, N, R
        self.homogeneous = homogeneous
        self.time = np.asarray(time, dtype=F32)
        self.tout = np.asarray(tout, dtype=F32)
        self.T = len(self.time)
        self.buy, self.inj, self.p2pp = price_table(self.time)
        # get_community (community.py:210-229) -- RNG order: ratings, then per agent T_m, T_in
        if homogeneous:
            lr = np.array([0.7] * N)
            pr = np.array([4] * N)
        else:
            lr = np.random.normal(0.7, 0.2, N)
            pr = np.random.normal(4, 0.2, N)
        self.load_ratings, self.pv_ratings = lr, pr
        self.load_w = np.stack([(norm_load[i] * lr[i] * 1e3).astype(F32) for i in range(N)])
        self.pv_w = np.stack([(norm_pv * pr[i] * 1e3).astype(F32) for i in range(N)])
        self.max_in = np.array([F32(max(lr[i], pr[i]) * 1.1 * 1e3) for i in range(N)], dtype=F32)
        self.t_in = np.zeros(N, F32)
        self.t_m = np.zeros(N, F32)
        for i in range(N):  # HPHeating.__init__ heating.py:101-104: T_m drawn first, then T_in
            if homogeneous:
                self.t_m[i] = F32(21.0)
                self.t_in[i] = F32(21.0)
            else:
                self.t_m[i] = F32(np.random.normal(21.0, 0.3, 1)[0])
                self.t_in[i] = F32(np.random.normal(21.0, 0.3, 1)[0])
        self.actors = [rl.QActor(20, 20, 20, 20, epsilon=0.81, decay=0.9) for _ in range(N)]
        self.explored = [False] * N
        for i, a in enumerate(self.actors):
            orig = a.random_action

            def rnd(orig=orig, i=i):
                self.explored[i] = True
                return orig()
            a.random_action = rnd
        self.levels = np.array([F32(x * 3e3) for x in (0.0, 0.5, 1.0)], dtype=F32)

    def _obs(self, t, i, p2p, balance):
        return np.array([[self.time[t], F32(F32(self.t_in[i] - F32(21.0)) / F32(1.0)), balance, p2p]],
                        dtype=F32)

    def _divide(self, out, powers):
        N = self.N
        sgn = lambda x: F32(int(x > 0) - int(x < 0))  # noqa: E731
        filt = [powers[j] if sgn(out) != sgn(powers[j]) else F32(0) for j in range(N)]
        tot = F32(0)
        for j in range(N):
            tot = F32(tot + filt[j])
        tot = F32(abs(tot))
        if tot == F32(0):
            return np.array([F32(F32(out * F32(1)) / F32(N))] * N, dtype=F32)
        return np.array([F32(F32(out * F32(abs(filt[j]))) / tot) for j in range(N)], dtype=F32)

    def step_t(self, t, training):
        N, R = self.N, self.R
        tn = (t + 1) % self.T
        P = np.zeros((N, N), F32)
        rec = {"code": np.zeros((R + 1, N), np.uint8), "action": np.zeros((R + 1, N), np.int64),
               "idx": np.zeros((R + 1, N, 4), np.int64)}
        last_obs = [None] * N
        last_act = [0] * N
        hp = np.zeros(N, F32)
        for r in range(R + 1):
            for i in range(N):
                P[i, i] = F32(0)
            rows = []
            for i in range(N):
                powers = np.array([-P[j, i] for j in range(N)], dtype=F32)
                acc = F32(0)
                for j in range(N):
                    acc = F32(acc + powers[j])
                mi = self.max_in[i]
                p2p = F32(F32(acc / F32(N)) / mi)
                bal = F32(F32(self.load_w[i, t] - self.pv_w[i, t]) / mi)
                obs = self._obs(t, i, p2p, bal)
                self.explored[i] = False
                if training:
                    a, _ = self.actors[i].select_action(Wrap(obs))
                else:
                    a, _ = self.actors[i].greedy_action(Wrap(obs))
                a = int(a)
                rec["code"][r, i] = a if (training and self.explored[i]) else GREEDY
                rec["action"][r, i] = a
                rec["idx"][r, i] = self.actors[i]._get_state_indices(obs)
                hp[i] = self.levels[a]
                out = F32(F32(bal * mi) + hp[i])
                rows.append(self._divide(out, powers))
                last_obs[i], last_act[i] = obs, a
            P = np.stack(rows).astype(F32)
        # _assign_powers on final P
        sgn = lambda x: F32(int(x > 0) - int(x < 0))  # noqa: E731
        g = np.zeros(N, F32)
        pp = np.zeros(N, F32)
        for i in range(N):
            ag, ap = F32(0), F32(0)
            for j in range(N):
                cond = sgn(P[i, j]) != sgn(P[j, i])
                e = F32(sgn(P[i, j]) * min(abs(P[i, j]), abs(P[j, i]))) if cond else F32(0)
                ag = F32(ag + F32(P[i, j] - e))
                ap = F32(ap + e)
            g[i], pp[i] = ag, ap
        cost = np.zeros(N, F32)
        rew = np.zeros(N, F32)
        for i in range(N):
            c = F32(g[i] * self.buy[t]) if g[i] >= 0 else F32(g[i] * self.inj[t])
            c = F32(c + F32(pp[i] * self.p2pp[t]))
            c = F32(F32(F32(c * F32(15)) / F32(60)) * F32(1e-3))
            cost[i] = c
            T_ = self.t_in[i]
            pen = max(max(F32(0), F32(F32(20.0) - T_)), max(F32(0), F32(T_ - F32(22.0))))
            pen = F32(pen + F32(1)) if pen > 0 else F32(0)
            rew[i] = F32(-F32(c + F32(F32(10) * pen)))
        if training:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", DeprecationWarning)
                for i in range(N):
                    mi = self.max_in[i]
                    baln = F32(F32(self.load_w[i, tn] - self.pv_w[i, tn]) / mi)
                    ns = np.array([[self.time[tn], F32(F32(self.t_in[i] - F32(21.0)) / F32(1.0)), baln,
                                    F32(F32(0) / mi)]], dtype=F32)
                    self.actors[i].train(Wrap(last_obs[i]), last_act[i], Wrap(np.array([rew[i]], F32)), Wrap(ns))
        rec.update(grid=g, p2p=pp, cost=cost, reward=rew, t_in=self.t_in.copy(), t_m=self.t_m.copy(), hp=hp.copy())
        # _step -> HPHeating.step -> temperature_simulation (reference)
        for i in range(N):
            a, b = self.heating.temperature_simulation(F32(self.tout[t]), F32(self.t_in[i]), F32(self.t_m[i]),
                                                       F32(hp[i]), 3.0)
            self.t_in[i], self.t_m[i] = F32(a), F32(b)
        return rec

    def episode(self, training=True):
        recs = [self.step_t(t, training) for t in range(self.T)]
        out = {k: np.stack([r[k] for r in recs]) for k in recs[0]}
        return out

    def reset(self):
        for i in range(self.N):  # HPHeating.reset heating.py:149-152: T_in drawn first, then T_m
            if self.homogeneous:
                self.t_in[i] = F32(21.0)
                self.t_m[i] = F32(21.0)
            else:
                self.t_in[i] = F32(np.random.normal(21.0, 0.3, 1)[0])
                self.t_m[i] = F32(np.random.normal(21.0, 0.3, 1)[0])

    def q_sparse(self):
        idx, val = [], []
        for i, a in enumerate(self.actors):
            nz = np.argwhere(a.q_table != 0)
            for k in nz:
                idx.append([i, *k])
                val.append(a.q_table[tuple(k)])
        return np.array(idx, dtype=np.int64).reshape(-1, 6), np.array(val, dtype=np.float64)


def make_loop(rl, heating, name, N, R, homogeneous, days, episodes, eval_days=1):
    time, temp, pv, loads = synthetic_days(days + eval_days)
    T = 96 * days
    np.random.seed(42)  # community.py:30 -- last module seed before main()
    com = HybridCommunity(rl, heating, N, R, homogeneous, loads[:N, :T], pv[:T], time[:T], temp[:T])
    data = dict(N=N, R=R, T=T, E=episodes, homogeneous=int(homogeneous),
                env_time=com.time, env_tout=com.tout, buy=com.buy, inj=com.inj, p2pp=com.p2pp,
                load_w=com.load_w, pv_w=com.pv_w, max_in=com.max_in,
                load_ratings=com.load_ratings, pv_ratings=com.pv_ratings)
    t_in0, t_m0, eps_sched, codes, outs = [], [], [], [], []
    for e in range(episodes):
        t_in0.append(com.t_in.copy())
        t_m0.append(com.t_m.copy())
        eps_sched.append(com.actors[0]._epsilon)
        o = com.episode(training=True)
        codes.append(o.pop("code"))
        outs.append(o)
        com.reset()
        if e % 50 == 0:  # community.py:279-286
            for a in com.actors:
                a.decay_exploration()
        qi, qv = com.q_sparse()
        data[f"q_idx_{e}"] = qi
        data[f"q_val_{e}"] = qv
    data["t_in0"] = np.stack(t_in0)
    data["t_m0"] = np.stack(t_m0)
    data["eps"] = np.array(eps_sched, dtype=np.float64)
    data["codes"] = np.stack(codes)  # [E, T, R+1, N]
    for k in outs[0]:
        data[f"train_{k}"] = np.stack([o[k] for o in outs])
    # greedy evaluation on the next day (CommunityMicrogrid.run, community.py:95-123), fresh start
    etime = time[T:T + 96].astype(F32)
    etemp = temp[T:T + 96].astype(F32)
    com.time, com.tout, com.T = etime, etemp, 96
    com.buy, com.inj, com.p2pp = price_table(etime)
    com.load_w = np.stack([(loads[i, T:T + 96] * com.load_ratings[i] * 1e3).astype(F32) for i in range(N)])
    com.pv_w = np.stack([(pv[T:T + 96] * com.pv_ratings[i] * 1e3).astype(F32) for i in range(N)])
    data.update(eval_env_time=etime, eval_env_tout=etemp, eval_buy=com.buy, eval_inj=com.inj,
                eval_p2pp=com.p2pp, eval_load_w=com.load_w, eval_pv_w=com.pv_w,
                eval_t_in0=com.t_in.copy(), eval_t_m0=com.t_m.copy())
    o = com.episode(training=False)
    o.pop("code")
    for k in o:
        data[f"eval_{k}"] = o[k]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **data)
    print(name, {k: v.shape for k, v in data.items() if hasattr(v, 'shape') and v.ndim > 1})


def make_heating(heating):
    rs = np.random.RandomState(7)
    n = 2000
    tout = rs.uniform(-10, 25, n).astype(F32)
    tin = rs.uniform(15, 27, n).astype(F32)
    tm = rs.uniform(15, 27, n).astype(F32)
    hp = np.array([0.0, 1500.0, 3000.0], F32)[rs.randint(0, 3, n)]
    out_in = np.zeros(n, F32)
    out_m = np.zeros(n, F32)
    for k in range(n):
        a, b = heating.temperature_simulation(tout[k], tin[k], tm[k], hp[k], 3.0)
        out_in[k], out_m[k] = a, b
    roll = {}
    for T in (96, 672):
        ti, tmm = F32(20.5), F32(20.8)
        to = (8 + 6 * np.sin(np.arange(T) * 2 * np.pi / 96)).astype(F32)
        hps = np.array([0.0, 1500.0, 3000.0], F32)[(np.arange(T) // 7) % 3]
        hist = np.zeros((T + 1, 2), F32)
        hist[0] = ti, tmm
        for t in range(T):
            ti, tmm = heating.temperature_simulation(to[t], ti, tmm, hps[t], 3.0)
            hist[t + 1] = ti, tmm
        roll[f"roll{T}_tout"] = to
        roll[f"roll{T}_hp"] = hps
        roll[f"roll{T}_hist"] = hist
    np.savez_compressed(os.path.join(HERE, "heating.npz"), tout=tout, tin=tin, tm=tm, hp=hp,
                        out_in=out_in, out_m=out_m, **roll)


def make_qactor(rl):
    a = rl.QActor(20, 20, 20, 20, epsilon=0.81, decay=0.9)
    rs = np.random.RandomState(11)
    n = 4000
    obs = np.stack([rs.uniform(0, 1, n), rs.uniform(-3, 3, n), rs.uniform(-3, 3, n),
                    rs.uniform(-3, 3, n)], axis=1).astype(F32)
    # bin boundaries: x with (x+1)/2*K == k exactly, and their f32 neighbours
    extra = []
    for k in range(-2, 23):
        for K, off in ((20, 0.0),):
            x = F32(2.0 * k / K - 1.0)
            for y in (np.nextafter(x, F32(-9)), x, np.nextafter(x, F32(9))):
                extra.append([F32(k / 20.0), y, y, y])
        xt = F32(2.0 * (k - 1) / 18 - 1.0)
        for y in (np.nextafter(xt, F32(-9)), xt, np.nextafter(xt, F32(9))):
            extra.append([F32(0.5), y, F32(0), F32(0)])
    extra += [[0.0, -1.0, -1.0, -1.0], [0.999, 1.0, 1.0, 1.0], [-0.0, -0.0, -0.0, -0.0],
              [1.0, 7.0, -7.0, 0.0]]
    obs = np.concatenate([obs, np.array(extra, dtype=F32)])
    idx = np.array([a._get_state_indices(obs[k:k + 1]) for k in range(len(obs))], dtype=np.int64)
    # epsilon-greedy + TD sequence under np.random.seed(42)
    np.random.seed(42)
    b = rl.QActor(20, 20, 20, 20, epsilon=0.81, decay=0.9)
    m = 3000
    s_obs = np.stack([rs.uniform(0, 1, m), rs.uniform(-0.3, 0.3, m), rs.uniform(-0.3, 0.3, m),
                      rs.uniform(-0.2, 0.2, m)], axis=1).astype(F32)
    n_obs = np.stack([rs.uniform(0, 1, m), s_obs[:, 1], rs.uniform(-0.3, 0.3, m),
                      np.zeros(m)], axis=1).astype(F32)
    rew = rs.uniform(-2, 0.5, m).astype(F32)
    acts = np.zeros(m, np.int64)
    qs = np.zeros(m, np.float64)
    eps = np.zeros(m, np.float64)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        for k in range(m):
            eps[k] = b._epsilon
            act, q = b.select_action(Wrap(s_obs[k:k + 1]))
            acts[k], qs[k] = act, q
            b.train(Wrap(s_obs[k:k + 1]), act, Wrap(rew[k:k + 1]), Wrap(n_obs[k:k + 1]))
            if k % 500 == 499:
                b.decay_exploration()
    nz = np.argwhere(b.q_table != 0)
    np.savez_compressed(os.path.join(HERE, "qactor.npz"), obs=obs, idx=idx, s_obs=s_obs, n_obs=n_obs,
                        rew=rew, acts=acts, qs=qs, eps=eps, q_nz_idx=nz,
                        q_nz_val=b.q_table[tuple(nz.T)])


def make_battery(storage):
    # Battery(capacity J, peak_power W, min_soc, max_soc, efficiency, soc) storage.py:108-116;
    # policy: RuleAgent._update_storage (agent.py:138-153) restated (it is never called in the reference)
    bat = storage.Battery(capacity=10 * 3.6e6, peak_power=5e3, min_soc=0.1, max_soc=0.9, efficiency=0.9, soc=0.5)
    st = storage.BatteryStorage(bat)
    st.reset()
    rs = np.random.RandomState(5)
    bal = rs.uniform(-6e3, 6e3, 400)
    out_bal = np.zeros_like(bal)
    soc = np.zeros_like(bal)
    for k, b in enumerate(bal):
        energy = b * 60 * 15
        if b > 0 and st.available_energy > 0:
            x = min(energy, st.available_energy)
            st.discharge(st.to_soc(x))
            b -= x / (60 * 15)
        elif b < 0 and not st.is_full:
            x = min(-energy, st.available_space)
            st.charge(st.to_soc(x))
            b += x / (60 * 15)
        out_bal[k] = b
        soc[k] = bat.soc
        st.step()
    np.savez_compressed(os.path.join(HERE, "battery.npz"), bal=bal, out_bal=out_bal, soc=soc,
                        capacity=bat.capacity, min_soc=0.1, max_soc=0.9, efficiency=0.9, soc0=0.5)


# ---------------------------------------------------------------- DQN draws (a20)
class _ActionsProbe:
    """Stands in for ActorModel.actions (a TF tensor): records the index each action read uses.
    random_action reads it with np.random.choice's int (rl.py:184), greedy_action with the (mocked)
    argmax tensor (rl.py:192), so the recorded key tells the branch and the explored action."""
    shape = (3,)

    def __init__(self):
        self.keys = []

    def __getitem__(self, k):
        self.keys.append(k)
        return MagicMock()


def _sample_tags(rl, buf):
    """ReplayBuffer.sample_batch (rl.py:225-244) on integer-tagged experiences: the tags of the
    sampled items, in batch order, as handed to the first tf.stack (rl.py:239)."""
    rl.tf.stack = MagicMock()
    buf.sample_batch()
    return [int(x) for x in rl.tf.stack.call_args_list[0].args[0]]


def make_dqn_draws(rl, T: int = 96, R: int = 1, N: int = 2, fill_episodes: int = 5, train_episodes: int = 50,
                   keep=(0, 1, 48, 49)):
    """The reference DQN community's draws (community.py:125-182, agent.py:301-342): per (t, round,
    agent) ActorModel.select_action (Python ``random.random()`` then ``np.random.choice`` when
    exploring, rl.py:173-184); per agent ReplayBuffer.add then, when training, sample_batch
    (Python ``random.sample``, rl.py:234-237); 5 fill episodes at epsilon 1, then
    Trainer.initialize_target's sample per agent (rl.py:272-276), then training episodes with
    main()'s decay (x0.9 after episodes 0, 50, ..., community.py:279-286).  Experiences are tagged
    with their add count, so a sampled tag t is deque index t - (added - count).  The buffer passes
    5000 entries (deque eviction, rl.py:207) in the last kept episodes.  Homogeneous (no T0 draws
    between episodes).  Plus a short-batch sequence (count < 32, rl.py:234-235)."""
    import random
    rl.QNetwork = MagicMock  # the Keras model (TF absent) draws nothing from random / np.random
    random.seed(42)
    np.random.seed(42)
    actors = [rl.ActorModel(1) for _ in range(N)]
    for a in actors:
        a.actions = _ActionsProbe()
    bufs = [rl.ReplayBuffer(5 * 1000, 32) for _ in range(N)]
    added = [0] * N
    E = fill_episodes + train_episodes
    codes = np.full((E, T, R + 1, N), GREEDY, np.uint8)
    eps_used = np.zeros(E)
    samples = {e: np.zeros((T, N, 32), np.uint16) for e in keep}
    init_tags = np.zeros((N, 32), np.uint16)
    for e in range(E):
        training = e >= fill_episodes
        eps_used[e] = actors[0]._epsilon
        for t in range(T):
            for r in range(R + 1):
                for i, a in enumerate(actors):
                    n0 = len(a.actions.keys)
                    a.select_action(MagicMock())
                    assert len(a.actions.keys) == n0 + 1
                    k = a.actions.keys[-1]
                    if isinstance(k, (int, np.integer)):
                        codes[e, t, r, i] = int(k)
            for i in range(N):
                bufs[i].add(added[i], 0, 0, 0)
                added[i] += 1
                if training:
                    tags = _sample_tags(rl, bufs[i])
                    if e - fill_episodes in samples:
                        samples[e - fill_episodes][t, i] = tags
        if e == fill_episodes - 1:
            for i in range(N):
                init_tags[i] = _sample_tags(rl, bufs[i])
        if training and (e - fill_episodes) % 50 == 0:
            for a in actors:
                a.decay_exploration()
    assert added[0] > 5000 and bufs[0].count == 5000
    # short batches: a fresh buffer sampled after every add from 1 to 40 (count < 32 first)
    random.seed(7)
    sb = rl.ReplayBuffer(5 * 1000, 32)
    short = []
    for k in range(40):
        sb.add(k, 0, 0, 0)
        short.append(_sample_tags(rl, sb))
    short_len = np.array([len(x) for x in short])
    np.savez_compressed(os.path.join(HERE, "dqn_draws.npz"), T=T, R=R, N=N, fill_episodes=fill_episodes,
                        train_episodes=train_episodes, keep=np.array(keep), codes=codes, eps=eps_used,
                        init_tags=init_tags, **{f"sample_tags_{e}": samples[e] for e in keep},
                        short_tags=np.concatenate(short).astype(np.uint16), short_len=short_len)


# ---------------------------------------------------------------- data pipeline (f2)
DATASET_DAYS = (7, 8, 9, 11, 12, 13, 18, 19, 20, 21)  # 7 and 21 fall outside [start, end) (dataset.py:22-25)


def dataset_raw(seed: int = 5):
    """Raw rows of the two tables dataset.get_data reads (database.py:28-47 + the l0..l4 load
    columns dataset.py:30 selects): a few October 2021 days; one load row is missing, so the
    inner merge of database.get_data (database.py:145) drops that slot."""
    rs = np.random.RandomState(seed)
    env, load = [], []
    for d in DATASET_DAYS:
        for slot in range(96):
            date, tm = f"2021-10-{d:02d}", f"{slot // 4:02d}:{15 * (slot % 4):02d}:00"
            pv = max(0.0, float(np.sin(np.pi * (slot / 4.0 - 7.0) / 10.0))) * float(rs.uniform(200, 900))
            env.append((date, tm, "+00:00", float(rs.normal(10, 3)), float(rs.rand()), float(rs.rand()), 0.0, pv))
            if not (d == 12 and slot == 50):
                load.append((date, tm, "+00:00", float(rs.uniform(100, 900)),
                             *[float(rs.uniform(50, 2000)) for _ in range(5)]))
    return env, load


def write_dataset_db(path: str, env, load):
    import sqlite3
    con = sqlite3.connect(path)
    cur = con.cursor()
    cur.execute("CREATE TABLE environment (date text NOT NULL, time text NOT NULL, utc text NOT NULL, "
                "temperature real, cloud_cover real, humidity real, irradiation real, pv real, "
                "PRIMARY KEY (date, time, utc))")
    cur.execute("CREATE TABLE load (date text NOT NULL, time text NOT NULL, utc text NOT NULL, load_0 real, "
                "l0 real, l1 real, l2 real, l3 real, l4 real, PRIMARY KEY (date, time, utc))")
    cur.executemany("INSERT INTO environment VALUES (?,?,?,?,?,?,?,?)", env)
    cur.executemany("INSERT INTO load VALUES (?,?,?,?,?,?,?,?,?)", load)
    con.commit()
    con.close()


def make_dataset():
    """The reference's own dataset.get_train_data / get_validation_data / get_test_data
    (dataset.py:61-95: database.get_data, day filter, process_dataframe) on a small database in
    its schema, and the (x, np.roll(x, -1)) pair dataframe_to_dataset hands to tf.data
    (dataset.py:98-103, captured from the TF mock)."""
    import tempfile
    env, load = dataset_raw()
    tmp = tempfile.mkdtemp(prefix="p2pmg_golden_")
    write_dataset_db(os.path.join(tmp, "ref.db"), env, load)
    cfg = sys.modules["config"]
    cfg.DB_FILE, cfg.DATA_PATH = "ref.db", tmp  # database.get_connection's defaults (database.py:16)
    sys.modules.pop("database", None)
    sys.modules.pop("dataset", None)
    import dataset  # noqa: E402  (imports the reference's database with the config above)
    out = {"env_rows": np.array([r[:3] for r in env]), "env_vals": np.array([r[3:] for r in env]),
           "load_rows": np.array([r[:3] for r in load]), "load_vals": np.array([r[3:] for r in load])}
    for split, fn in (("train", dataset.get_train_data), ("validation", dataset.get_validation_data),
                      ("test", dataset.get_test_data)):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            env_df, agent_dfs = fn()
        out[f"{split}_env_cols"] = np.array(list(env_df.columns))
        out[f"{split}_env"] = env_df.to_numpy(dtype=np.float64)
        out[f"{split}_index"] = env_df.index.to_numpy()
        out[f"{split}_agents"] = np.stack([a.to_numpy(dtype=np.float64) for a in agent_dfs])
        out[f"{split}_agent_cols"] = np.array(list(agent_dfs[0].columns))
        if split == "train":
            tfmock = sys.modules["tensorflow"]
            tfmock.data.Dataset.from_tensor_slices.reset_mock()
            dataset.dataframe_to_dataset(env_df)
            x, xr = tfmock.data.Dataset.from_tensor_slices.call_args[0][0]
            out["train_ds_x"], out["train_ds_rolled"] = np.asarray(x), np.asarray(xr)
    np.savez_compressed(os.path.join(HERE, "dataset.npz"), **out)


def main():
    heating, rl, storage, setup = import_reference()
    if sys.argv[1:] == ["dqn_draws"]:  # regenerate only this fixture
        return make_dqn_draws(rl)
    make_dataset()
    assert setup.nr_agents == 2 and setup.rounds == 1 and setup.homogeneous is False
    make_heating(heating)
    make_qactor(rl)
    make_battery(storage)
    make_dqn_draws(rl)
    # thesis community (setup.py:33-35): N=2, rounds=1, heterogeneous
    make_loop(rl, heating, "loop_thesis_T96", N=2, R=1, homogeneous=False, days=1, episodes=3)
    make_loop(rl, heating, "loop_thesis_T672", N=2, R=1, homogeneous=False, days=7, episodes=2)
    make_loop(rl, heating, "loop_homo_T96", N=2, R=1, homogeneous=True, days=1, episodes=2)
    make_loop(rl, heating, "loop_n5_r2_T96", N=5, R=2, homogeneous=False, days=1, episodes=2)


if __name__ == "__main__":
    main()
