"""CPU restatement of the P2PMicrogrid hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline.  The product
(``p2pmicrogrid_amd``) never imports anything under ``oracle/``.

What it restates (every function cites the reference line it follows, paths relative to
``/root/reference/microgrid``), vectorised over S independent scenarios x N agents:

    GridAgent.take_decision            agent.py:59-67, community.py:69-70   -> prices()
    CommunityMicrogrid._run            community.py:67-93                   -> OracleBatch._step
    RLAgent.__call__/_get_balance/...  agent.py:172-213
    RLAgent._divide_power              agent.py:186-195                     -> divide_power()
    QActor._get_state_indices          rl.py:89-95                          -> state_index()
    QActor.select_action/greedy_action rl.py:100-117
    CommunityMicrogrid._assign_powers  community.py:45-54                   -> assign_powers()
    CommunityMicrogrid._compute_costs  community.py:56-65                   -> compute_costs()
    RLAgent.get_reward                 agent.py:225-232                     -> reward()
    QAgent.train -> QActor.train       agent.py:293-298, rl.py:119-129
    HPHeating.step/temperature_simulation heating.py:37-56,126-143          -> temperature_step()
    CommunityMicrogrid.train_episode   community.py:149-182                 -> OracleBatch.run_episode
    CommunityMicrogrid.run             community.py:95-123                  (mode="greedy")

Numerics contract: every simulation quantity is float32, each op rounded
separately (no FMA), Python constants cast to f32 before the op; the Q-table and the TD
update are float64 (NumPy 2 promotion of ``reward.numpy() + gamma * q_max``); the index
arithmetic is f32 (NumPy 2 / NEP 50).  Reductions over agents use ONE canonical order,
sequential j = 0..N-1 starting from +0.0, shared with the HIP kernel.

Parity pinning: ``state_index``/``QActor`` logic and ``temperature_step`` are checked
against vectors produced by the reference's own ``rl.QActor`` and
``heating.temperature_simulation`` (tests/golden/make_golden.py); the full-loop glue is
checked against the hybrid harness in that script which drives the reference's own QActor
and temperature_simulation.  The TF-op glue itself (agent.py/community.py) cannot be run
(TensorFlow absent), so its ulp-level parity with TF is unpinned.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

from . import philox

F32 = np.float32
GREEDY = 255  # replay code meaning "no exploration: take the greedy action"


# ----------------------------------------------------------------------------- constants
@dataclass
class OracleParams:
    """Constants of the reference, with the f32 casts TF applies."""
    # rl.py:58-60 / agent.py:258-264
    n_time: int = 20
    n_temp: int = 20
    n_bal: int = 20
    n_p2p: int = 20
    n_actions: int = 3
    alpha: float = 1e-5
    gamma: float = 0.9
    # agent.py:268 actions, heating.py:122-124 power = level * max_power; community.py:226
    action_levels: tuple = (0.0, 0.5, 1.0)
    hp_max_power: float = 3e3
    hp_cop: float = 3.0
    setpoint: float = 21.0
    margin: float = 1.0  # HPHeating.TEMPERATURE_MARGIN heating.py:90
    # heating.py:23-29
    Ci: float = 2.44e6 * 2
    Cm: float = 9.4e7
    Ri: float = 8.64e-4
    Re: float = 1.05e-2
    Rvent: float = 7.98e-3
    gA: float = 11.468
    f_rad: float = 0.3
    solar_rad: float = 0.0
    # setup.py:8-25
    seconds_per_minute: int = 60
    minutes_per_hour: int = 60
    time_slot: int = 15
    grid_cost_avg: float = 12.0
    grid_cost_amplitude: float = 5.0
    grid_cost_period: float = 12
    grid_cost_phase: float = 3
    hours_per_day: int = 24
    cents_per_euro: int = 100
    injection_price: float = 0.07
    penalty_weight: float = 10.0  # agent.py:230

    @property
    def hp_levels(self):
        # heating.power = tf.convert_to_tensor([hp.power * hp.max_power], f32)  heating.py:124
        return np.array([F32(l * self.hp_max_power) for l in self.action_levels], dtype=F32)

    @property
    def lower(self):
        return self.setpoint - self.margin  # heating.py:93-94

    @property
    def upper(self):
        return self.setpoint + self.margin


# ----------------------------------------------------------------------------- primitives
def prices(time_f32, p: OracleParams = OracleParams()):
    """Per-timestep price table (agent.py:59-67, community.py:69-70).

    buy = (f(12) + f(5) * sin(time * f(4pi) - f(3))) / f(100); inj = f(0.07);
    p2p = (buy + inj) / f(2).  TF's Eigen sin is not reproducible here, so the table is an
    input shared by the oracle and the device.
    """
    t = np.asarray(time_f32, dtype=F32)
    freq = F32(2 * np.pi * p.hours_per_day / p.grid_cost_period)
    arg = (t * freq) - F32(p.grid_cost_phase)
    s = np.sin(arg).astype(F32)
    buy = (F32(p.grid_cost_avg) + F32(p.grid_cost_amplitude) * s) / F32(p.cents_per_euro)
    inj = np.full_like(buy, F32(p.injection_price))
    p2p = (buy + inj) / F32(2)
    return buy.astype(F32), inj.astype(F32), p2p.astype(F32)


def state_index(x, K: int, kind: str):
    """rl.py:89-95 under NumPy 2 (f32 arithmetic, int() truncation, clamp to [0, K-1]).

    kind = 'time':  int(x * K)
           'temp':  int((x + 1) / 2 * (K - 2) + 1)
           'plain': int((x + 1) / 2 * K)           (balance and p2p)
    """
    x = np.asarray(x, dtype=F32)
    if kind == "time":
        v = x * F32(K)
    elif kind == "temp":
        v = ((x + F32(1)) / F32(2)) * F32(K - 2) + F32(1)
    else:
        v = ((x + F32(1)) / F32(2)) * F32(K)
    v = np.trunc(v)
    v = np.clip(v, 0, K - 1)
    return v.astype(np.int64)


def sign(x):
    """tf.math.sign for f32: +1/-1/0 (sign of +-0 is 0)."""
    x = np.asarray(x, dtype=F32)
    return (x > 0).astype(F32) - (x < 0).astype(F32)


def seq_sum(x, axis=-1):
    """Canonical reduction: sequential j = 0..N-1 from +0.0 in f32."""
    x = np.moveaxis(np.asarray(x, dtype=F32), axis, -1)
    acc = np.zeros(x.shape[:-1], dtype=F32)
    for j in range(x.shape[-1]):
        acc = acc + x[..., j]
    return acc


def divide_power(out, powers, N: int):
    """RLAgent._divide_power (agent.py:186-195), batched.

    out: (...,) f32; powers: (..., N) f32.  Returns (..., N) f32 row of P.
    """
    out = np.asarray(out, dtype=F32)
    powers = np.asarray(powers, dtype=F32)
    keep = sign(out)[..., None] != sign(powers)
    filtered = np.where(keep, powers, F32(0)).astype(F32)
    tot = np.abs(seq_sum(filtered))
    even = (out * F32(1)) / F32(N)
    prop = (out[..., None] * np.abs(filtered)) / np.where(tot == 0, F32(1), tot)[..., None]
    return np.where((tot == 0)[..., None], even[..., None], prop).astype(F32)


def assign_powers(P):
    """CommunityMicrogrid._assign_powers (community.py:45-54) on the final-round P.

    P: (..., N, N) f32 with the diagonal NOT zeroed.
    """
    P = np.asarray(P, dtype=F32)
    PT = np.swapaxes(P, -1, -2)
    cond = sign(P) != sign(PT)
    pm = np.where(cond, P, F32(0)).astype(F32)
    apm = np.abs(pm)
    ex = (sign(pm) * np.minimum(apm, np.swapaxes(apm, -1, -2))).astype(F32)
    p_grid = seq_sum(P - ex)
    p_p2p = seq_sum(ex)
    return p_grid, p_p2p


def rule_assign_powers(Pv):
    """CommunityMicrogrid._assign_powers (community.py:45-54) on a RuleAgent community's stack.

    RuleAgent.take_decision returns its net power as a (1,) tensor (agent.py:111-128), so the
    stacked P is (N, 1): TF broadcasts P (N,1) against P^T (1,N) inside ``tf.where`` and the
    subtraction, giving ex[i,j] = sign(P_i) min(|P_i|, |P_j|) on differing signs and
    p_grid[i] = sum_j (P_i - ex[i,j]) over all N columns (a reference quirk: N copies of P_i).
    Pv: (..., N) f32.
    """
    Pv = np.asarray(Pv, dtype=F32)
    P = Pv[..., :, None]
    PT = Pv[..., None, :]
    cond = sign(P) != sign(PT)
    pm = np.where(cond, P, F32(0)).astype(F32)
    apm = np.abs(pm)
    ex = (sign(pm) * np.minimum(apm, np.swapaxes(apm, -1, -2))).astype(F32)
    p_grid = seq_sum((P - ex).astype(F32))
    p_p2p = seq_sum(ex)
    return p_grid, p_p2p


def compute_costs(g, pp, buy, inj, p2p, p: OracleParams = OracleParams()):
    """CommunityMicrogrid._compute_costs (community.py:56-65)."""
    g = np.asarray(g, dtype=F32)
    pp = np.asarray(pp, dtype=F32)
    c = np.where(g >= 0, g * F32(buy), g * F32(inj)).astype(F32) + pp * F32(p2p)
    c = (c * F32(p.time_slot)) / F32(p.minutes_per_hour)
    return (c * F32(1e-3)).astype(F32)


def reward(cost, t_in, p: OracleParams = OracleParams()):
    """RLAgent.get_reward (agent.py:225-232), pre-update indoor temperature."""
    t = np.asarray(t_in, dtype=F32)
    pen = np.maximum(np.maximum(F32(0), F32(p.lower) - t), np.maximum(F32(0), t - F32(p.upper)))
    pen = np.where(pen > 0, pen + F32(1), F32(0)).astype(F32)
    return (-(np.asarray(cost, dtype=F32) + F32(p.penalty_weight) * pen)).astype(F32)


def temperature_step(t_out, t_in, t_m, hp, p: OracleParams = OracleParams()):
    """heating.temperature_simulation (heating.py:37-56) with TF's f32 casting."""
    t_out = np.asarray(t_out, dtype=F32)
    t_in = np.asarray(t_in, dtype=F32)
    t_m = np.asarray(t_m, dtype=F32)
    hp = np.asarray(hp, dtype=F32)
    cop = F32(p.hp_cop)
    d_in = F32(1 / p.Ci) * (
        (F32(1 / p.Ri) * (t_m - t_in) + F32(1 / p.Rvent) * (t_out - t_in))
        + (F32(1 - p.f_rad) * hp) * cop)
    d_m = F32(1 / p.Cm) * (
        ((F32(1 / p.Ri) * (t_in - t_m) + F32(1 / p.Re) * (t_out - t_m)) + F32(p.gA * p.solar_rad))
        + (F32(p.f_rad) * hp) * cop)
    spm, slot = F32(p.seconds_per_minute), F32(p.time_slot)
    return (t_in + (d_in * spm) * slot).astype(F32), (t_m + (d_m * spm) * slot).astype(F32)


DELTA_SCALE = 2.0 ** 40  # shared-table TD deltas in int64 fixed point (build-defined)


def battery_rule(balance, soc, cap, smin=0.1, smax=0.9, sqrt_eff=np.sqrt(0.9)):
    """RuleAgent._update_storage (agent.py:138-153) with BatteryStorage (storage.py:79-100), f64,
    vectorised; agents with cap == 0 are untouched.  Returns (balance', soc')."""
    b = np.asarray(balance, np.float64)
    soc = np.asarray(soc, np.float64)
    cap = np.broadcast_to(np.asarray(cap, np.float64), b.shape)
    with np.errstate(divide="ignore", invalid="ignore"):
        energy = (b * 60.0) * 15.0
        avail_e = (np.maximum(0.0, soc - smin) * cap) * sqrt_eff
        avail_s = (np.maximum(0.0, smax - soc) * cap) / sqrt_eff
        dis = (b > 0) & (avail_e > 0) & (cap > 0)
        chg = ~dis & (b < 0) & ~(soc >= smax) & (cap > 0)
        xd = np.where(energy <= avail_e, energy, avail_e)
        xc = np.where(-energy <= avail_s, -energy, avail_s)
        soc2 = np.where(dis, soc - (xd / cap) / sqrt_eff, np.where(chg, soc + sqrt_eff * (xc / cap), soc))
        b2 = np.where(dis, b - xd / 900.0, np.where(chg, b + xc / 900.0, b))
    return b2, soc2


# ----------------------------------------------------------------------------- RNG replay
def reference_replay_codes(rs: np.random.RandomState, T: int, R: int, N: int, eps) -> np.ndarray:
    """Exploration draws in the reference's exact consumption order:
    per (t, round r, agent i): rs.rand(); if < eps: rs.choice(3) (rl.py:101-111).
    Returns uint8 codes [T, R+1, N] (GREEDY = 255)."""
    eps = np.broadcast_to(np.asarray(eps, dtype=np.float64), (N,))
    codes = np.full((T, R + 1, N), GREEDY, dtype=np.uint8)
    for t in range(T):
        for r in range(R + 1):
            for i in range(N):
                if rs.rand() < eps[i]:
                    codes[t, r, i] = rs.choice(3)
    return codes


# ----------------------------------------------------------------------------- the batch
@dataclass
class OracleBatch:
    """S independent communities x N agents, per-agent tabular Q (f64 or f32).

    Inputs (all f32 unless noted):
      load_w, pv_w : [S, N, T] agent power profiles in W (community.py:219-220)
      max_in       : [S, N]     (community.py:216-227)
      env_time     : [S_env, T] normalised time slot (dataset.py:43-44), S_env in {1, S}
      env_tout     : [S_env, T] outdoor temperature in degC
    """
    S: int
    N: int
    R: int
    load_w: np.ndarray
    pv_w: np.ndarray
    max_in: np.ndarray
    env_time: np.ndarray
    env_tout: np.ndarray
    q_dtype: str = "f64"
    params: OracleParams = field(default_factory=OracleParams)
    price_table: Optional[tuple] = None  # (buy, inj, p2p) [S_env, T] f32; default: prices()
    shared_q: bool = False               # one frozen policy table, int64 fixed-point deltas
    hp_levels: Optional[np.ndarray] = None  # [S, N, 3] f32 per-agent heat-pump power per action
    battery_capacity: Optional[np.ndarray] = None  # [S, N] J (0 = none); None = no storage
    battery_bounds: tuple = (0.1, 0.9, 0.9)        # (min_soc, max_soc, efficiency)

    def __post_init__(self):
        p = self.params
        self.T = self.load_w.shape[-1]
        self.load_w = np.asarray(self.load_w, dtype=F32).reshape(self.S, self.N, self.T)
        self.pv_w = np.asarray(self.pv_w, dtype=F32).reshape(self.S, self.N, self.T)
        self.max_in = np.asarray(self.max_in, dtype=F32).reshape(self.S, self.N)
        self.env_time = np.asarray(self.env_time, dtype=F32).reshape(-1, self.T)
        self.env_tout = np.asarray(self.env_tout, dtype=F32).reshape(-1, self.T)
        self.n_states = p.n_time * p.n_temp * p.n_bal * p.n_p2p
        qt = np.float64 if self.q_dtype == "f64" else np.float32
        self.q = np.zeros((1 if self.shared_q else self.S * self.N, self.n_states, p.n_actions), dtype=qt)
        self.q_delta = np.zeros((self.n_states, p.n_actions), np.int64)
        if self.hp_levels is None:
            self.hp_levels = np.broadcast_to(p.hp_levels, (self.S, self.N, 3)).astype(F32)
        self.hp_levels = np.asarray(self.hp_levels, F32).reshape(self.S, self.N, 3)
        self.soc = np.full((self.S, self.N), 0.5)
        self.t_in = np.full((self.S, self.N), F32(p.setpoint), dtype=F32)
        self.t_m = np.full((self.S, self.N), F32(p.setpoint), dtype=F32)
        if self.price_table is None:
            buy, inj, p2p = prices(self.env_time, p)
        else:
            buy, inj, p2p = (np.asarray(x, dtype=F32).reshape(-1, self.T) for x in self.price_table)
        self.buy, self.inj, self.p2p = buy, inj, p2p

    # -- Q table in the reference layout (20, 20, 20, 20, 3) per agent (rl.py:73-74)
    def q_table(self, agent: int) -> np.ndarray:
        p = self.params
        return self.q[agent].reshape(p.n_time, p.n_temp, p.n_bal, p.n_p2p, p.n_actions)

    def set_q_table(self, agent: int, table: np.ndarray):
        self.q[agent] = np.asarray(table).reshape(self.n_states, -1).astype(self.q.dtype)

    def apply_q_delta(self):
        """Shared table: Q += delta * 2^-40 (f64) where delta != 0; delta = 0."""
        nz = self.q_delta != 0
        q0 = self.q[0]
        q0[nz] = (q0[nz].astype(np.float64) + self.q_delta[nz].astype(np.float64) * (1.0 / DELTA_SCALE)).astype(q0.dtype)
        self.q_delta[:] = 0

    def run_rule_episode(self, hp_on: np.ndarray) -> Dict:
        """CommunityMicrogrid.run (community.py:95-123) of a RuleAgent community
        (get_rule_based_community, community.py:237-238; RuleAgent agent.py:106-136), R = 0.

        Per step: the hysteresis heating rule on the pre-update T_in (agent.py:130-136: on at
        T_in <= setpoint - 1, off at T_in >= setpoint + 1, else unchanged), net power
        (load - pv) + hp (agent.py:119-128), the (N, 1)-broadcast market, costs, then the RC step
        with hp (HPHeating.step heating.py:138-143).  hp_on: [S, N] 0/1 state of HeatPump.power,
        updated in place (it persists across runs: HPHeating.reset does not touch it)."""
        p = self.params
        S, N, T = self.S, self.N, self.T
        hpmax = self.hp_levels[:, :, 2]
        tr = {k: [] for k in ("grid", "p2p", "cost", "t_in", "hp", "on")}
        for t in range(T):
            tout = self._env(self.env_tout, t)
            hp_on = np.where(self.t_in <= F32(p.lower), 1, np.where(self.t_in >= F32(p.upper), 0, hp_on))
            hp = (hp_on.astype(F32) * hpmax).astype(F32)  # HPHeating.power: hp.power * max_power
            Pv = ((self.load_w[:, :, t] - self.pv_w[:, :, t]) + hp).astype(F32)
            g, pp = rule_assign_powers(Pv)
            cost = compute_costs(g, pp, self._env(self.buy, t)[:, None], self._env(self.inj, t)[:, None],
                                 self._env(self.p2p, t)[:, None], p)
            tr["grid"].append(g)
            tr["p2p"].append(pp)
            tr["cost"].append(cost)
            tr["t_in"].append(self.t_in.copy())
            tr["hp"].append(hp)
            tr["on"].append(hp_on.copy())
            self.t_in, self.t_m = temperature_step(tout[:, None], self.t_in, self.t_m, hp, p)
        out = {k: np.stack(v) for k, v in tr.items()}
        out["hp_on"] = hp_on
        return out

    def _env(self, arr, t):
        return arr[:, t] if arr.shape[0] == self.S else np.broadcast_to(arr[0, t], (self.S,))

    def _row(self, it, iT, ib, ip):
        p = self.params
        return ((it * p.n_temp + iT) * p.n_bal + ib) * p.n_p2p + ip

    def run_episode(self, mode: str = "train", codes: Optional[np.ndarray] = None,
                    rng: str = "replay", seed: int = 42, episode: int = 0, eps=0.81,
                    agent_ids: Optional[np.ndarray] = None) -> Dict:
        """One episode of T steps.  mode 'train' = train_episode (community.py:149-182),
        'greedy' = run (community.py:95-123).  Replay codes: uint8 [T, R+1, S, N]."""
        p = self.params
        S, N, R, T = self.S, self.N, self.R, self.T
        A = S * N
        agents = np.arange(A).reshape(S, N)
        gids = agents if agent_ids is None else np.asarray(agent_ids).reshape(S, N)  # Philox counters
        tab = np.zeros_like(agents) if self.shared_q else agents  # which Q table each agent reads
        lv = self.hp_levels
        bat = self.battery_capacity is not None
        if bat:
            cap = np.asarray(self.battery_capacity, np.float64).reshape(S, N)
            smin, smax, eff = self.battery_bounds
            sqe = np.sqrt(eff)
        mi = self.max_in
        eps_arr = np.broadcast_to(np.asarray(eps, dtype=np.float64), (S, N))
        tr = {k: [] for k in ("action", "idx", "reward", "cost", "grid", "p2p", "t_in", "t_m", "hp")}
        qf = self.q.dtype.type
        for t in range(T):
            tn = (t + 1) % T  # np.roll(-1) next-step pairing (dataset.py:101)
            time_t = self._env(self.env_time, t)
            tout = self._env(self.env_tout, t)
            time_n = self._env(self.env_time, tn)
            buy = self._env(self.buy, t)
            inj = self._env(self.inj, t)
            p2pp = self._env(self.p2p, t)
            # RLAgent._get_balance agent.py:172-176
            bal = (self.load_w[:, :, t] - self.pv_w[:, :, t]) / mi
            baln = (self.load_w[:, :, tn] - self.pv_w[:, :, tn]) / mi
            # HPHeating.normalized_temperature heating.py:118-120
            tnorm = (self.t_in - F32(p.setpoint)) / F32(p.margin)
            it = state_index(np.broadcast_to(time_t[:, None], (S, N)), p.n_time, "time")
            iT = state_index(tnorm, p.n_temp, "temp")
            ib = state_index(bal, p.n_bal, "plain")
            P = np.zeros((S, N, N), dtype=F32)
            acts = np.zeros((R + 1, S, N), dtype=np.int64)
            idxs = np.zeros((R + 1, S, N, 4), dtype=np.int64)
            hp = np.zeros((S, N), dtype=F32)
            soc_r = self.soc.copy() if bat else None
            for r in range(R + 1):
                # P <- P - diag(diag(P))  community.py:76
                d = np.arange(N)
                P[:, d, d] = F32(0)
                powers = -np.swapaxes(P, 1, 2)  # powers[s, i, j] = -P[s, j, i]  community.py:81
                p2pf = (seq_sum(powers) / F32(N)) / mi  # agent.py:203
                ip = state_index(p2pf, p.n_p2p, "plain")
                row = self._row(it, iT, ib, ip)
                qrow = self.q[tab, row]  # (S, N, 3)
                greedy = np.argmax(qrow, axis=-1)  # first max wins (rl.py:116)
                if mode == "greedy":
                    a = greedy
                elif rng == "replay":
                    c = codes[t, r]
                    a = np.where(c == GREEDY, greedy, c.astype(np.int64))
                else:
                    u, ra = philox.decision_draws(seed, episode, gids.ravel(), t, r, R, eps=philox.launch_eps(eps_arr))
                    u = u.reshape(S, N)
                    ra = ra.reshape(S, N)
                    a = np.where(u < eps_arr, ra, greedy)
                hp = np.take_along_axis(lv, a[..., None], axis=-1)[..., 0]
                out = (bal * mi) + hp  # agent.py:210
                if bat:  # battery rule on the net power, SoC committed by the final round
                    ob_, soc_r = battery_rule(out.astype(np.float64), self.soc, cap, smin, smax, sqe)
                    out = np.where(cap > 0, ob_.astype(F32), out).astype(F32)
                P = divide_power(out, powers, N)  # rows stacked after all agents (Jacobi)
                acts[r] = a
                idxs[r] = np.stack([it, iT, ib, ip], axis=-1)
            if bat:
                self.soc = soc_r
            g, pp = assign_powers(P)
            cost = compute_costs(g, pp, buy[:, None], inj[:, None], p2pp[:, None], p)
            rew = reward(cost, self.t_in, p)
            if mode == "train":
                # QAgent.train agent.py:293-298 -> QActor.train rl.py:119-129
                itn = state_index(np.broadcast_to(time_n[:, None], (S, N)), p.n_time, "time")
                ibn = state_index(baln, p.n_bal, "plain")
                ipn = state_index(np.zeros((S, N), F32) / mi, p.n_p2p, "plain")
                nrow = self._row(itn, iT, ibn, ipn)
                qmax = self.q[tab, nrow].max(axis=-1)
                srow = self._row(it, iT, ib, idxs[R][..., 3])
                a = acts[R]
                qsa = self.q[tab, srow, a]
                if self.shared_q:
                    d = p.alpha * ((rew.astype(np.float64) + p.gamma * qmax.astype(np.float64)) - qsa.astype(np.float64))
                    np.add.at(self.q_delta, (srow.ravel(), a.ravel()), np.rint(d * DELTA_SCALE).astype(np.int64).ravel())
                elif qf is np.float64:
                    new = qsa + p.alpha * ((rew.astype(np.float64) + p.gamma * qmax) - qsa)
                else:
                    new = qsa + F32(p.alpha) * ((rew + F32(p.gamma) * qmax) - qsa)
                if not self.shared_q:
                    self.q[agents, srow, a] = new
            tr["action"].append(acts)
            tr["idx"].append(idxs)
            tr["reward"].append(rew)
            tr["cost"].append(cost)
            tr["grid"].append(g)
            tr["p2p"].append(pp)
            tr["t_in"].append(self.t_in.copy())
            tr["t_m"].append(self.t_m.copy())
            tr["hp"].append(hp)
            # CommunityMicrogrid._step community.py:184-188 -> HPHeating.step heating.py:138-143
            self.t_in, self.t_m = temperature_step(tout[:, None], self.t_in, self.t_m, hp, p)
        out = {k: np.stack(v) for k, v in tr.items()}
        # avg_reward = sum_t mean_i r  (community.py:179), canonical sequential order
        mean_t = seq_sum(out["reward"], axis=-1) / F32(N)  # [T, S]
        out["episode_reward"] = seq_sum(mean_t, axis=0)   # [S]
        out["t_in_final"] = self.t_in.copy()
        out["t_m_final"] = self.t_m.copy()
        return out
