"""DeviceCommunityBatch — S independent communities x N agents resident in HBM.

This is the batched entry point the reference lacks (SURVEY.md §8b "Add a batched entry
point over S scenarios"): one ``run_episode`` call is one ``CommunityMicrogrid.train_episode``
(community.py:149-182) or ``run`` (community.py:95-123) for every scenario at once, executed
by ONE HIP kernel launch (p2pmg_kernels.hip::episode_kernel).  The reference-shaped object API
(``community.CommunityMicrogrid`` & co.) is a thin layer over this class with S = 1.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Sequence

import numpy as np

from . import _lib
from . import setup as cfgmod

F32 = np.float32
RECORD_NAMES = ("reward", "cost", "grid", "p2p", "t_in", "action", "index")


def price_table(time_f32, grid_cost_avg=cfgmod.GRID_COST_AVG, amplitude=cfgmod.GRID_COST_AMPLITUDE,
                period=cfgmod.GRID_COST_PERIOD, phase=cfgmod.GRID_COST_PHASE,
                injection=cfgmod.GRID_INJECTION_PRICE):
    """GridAgent prices per timestep (agent.py:51-67) and the P2P midpoint (community.py:70).

    Host-side table computed once per environment with TF's f32 constant casting; the device
    consumes it as an input (SURVEY.md §3.4 item 1 — TF's Eigen sin is not reproducible).
    """
    t = np.asarray(time_f32, dtype=F32)
    freq = F32(2 * np.pi * cfgmod.HOURS_PER_DAY / period)
    s = np.sin((t * freq) - F32(phase)).astype(F32)
    buy = ((F32(grid_cost_avg) + F32(amplitude) * s) / F32(cfgmod.CENTS_PER_EURO)).astype(F32)
    inj = np.full_like(buy, F32(injection))
    p2p = ((buy + inj) / F32(2)).astype(F32)
    return buy, inj, p2p


class DeviceCommunityBatch:
    """Device-resident batch of S communities.  All compute runs in libp2pmg.so."""

    def __init__(self, n_scenarios: int, n_agents: int, rounds: int, horizon: int, q_dtype: str = "f64",
                 device: int = 0, seed: int = 42, scenario_offset: int = 0, shared_q: bool = False, **overrides):
        self.L = _lib.lib()
        cfg = _lib.default_config()
        cfg.n_scenarios, cfg.n_agents, cfg.rounds, cfg.horizon = n_scenarios, n_agents, rounds, horizon
        cfg.q_dtype = _lib.Q_F64 if q_dtype == "f64" else _lib.Q_F32
        cfg.seed = seed
        cfg.scenario_offset = scenario_offset
        cfg.shared_q = int(bool(shared_q))
        for k, v in overrides.items():
            setattr(cfg, k, v)
        self.cfg = cfg
        self.S, self.N, self.R, self.T = n_scenarios, n_agents, rounds, horizon
        self.A = n_scenarios * n_agents
        self.q_dtype = q_dtype
        self.device = device
        self.seed = seed
        self.scenario_offset = scenario_offset
        self.shared_q = bool(shared_q)
        self.n_tables = 1 if shared_q else self.A
        self.n_states = cfg.n_time_states * cfg.n_temp_states * cfg.n_balance_states * cfg.n_p2p_states
        self.q_shape = (cfg.n_time_states, cfg.n_temp_states, cfg.n_balance_states, cfg.n_p2p_states,
                        cfg.n_actions)
        ctx = C.c_void_p()
        _lib.check(self.L.p2pmg_create(C.byref(cfg), device, C.byref(ctx)), what="p2pmg_create")
        self._ctx = ctx
        self._recorded = 0

    # ----------------------------------------------------------------- lifetime
    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self.L.p2pmg_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _chk(self, status, what):
        _lib.check(status, self._ctx, what)

    def sync(self):
        self._chk(self.L.p2pmg_sync(self._ctx), "sync")

    def device_info(self):
        buf = C.create_string_buffer(256)
        mem = C.c_size_t(0)
        self._chk(self.L.p2pmg_device_info(self._ctx, buf, 256, C.byref(mem)), "device_info")
        return buf.value.decode(), mem.value

    # ----------------------------------------------------------------- inputs
    def set_env(self, time, t_out, buy=None, inj=None, p2p=None):
        """Environment rows (environment.py:26-45): time (slot/96) and outdoor temperature,
        shape [T] (shared by all scenarios) or [S, T]."""
        time = np.ascontiguousarray(np.atleast_2d(np.asarray(time, dtype=F32)))
        t_out = np.ascontiguousarray(np.atleast_2d(np.asarray(t_out, dtype=F32)))
        if buy is None:
            buy, inj, p2p = price_table(time)
        arrs = [np.ascontiguousarray(np.atleast_2d(np.asarray(x, dtype=F32))) for x in (buy, inj, p2p)]
        n_env = time.shape[0]
        for x in (time, t_out, *arrs):
            if x.shape != (n_env, self.T):
                raise ValueError(f"env arrays must be [{n_env}, {self.T}], got {x.shape}")
        self._chk(self.L.p2pmg_set_env(self._ctx, n_env, time, t_out, *arrs), "set_env")

    def set_profiles(self, load_w, pv_w):
        """Per-agent power profiles in W, shape [S, N, T] (community.py:219-224)."""
        lw = np.ascontiguousarray(np.asarray(load_w, dtype=F32).reshape(self.A, self.T))
        pw = np.ascontiguousarray(np.asarray(pv_w, dtype=F32).reshape(self.A, self.T))
        self._chk(self.L.p2pmg_set_profiles(self._ctx, lw, pw), "set_profiles")

    def set_max_in(self, max_in):
        m = np.ascontiguousarray(np.asarray(max_in, dtype=F32).reshape(self.A))
        self._chk(self.L.p2pmg_set_agent_params(self._ctx, m), "set_agent_params")

    def set_temperatures(self, t_in, t_m):
        a = np.ascontiguousarray(np.asarray(t_in, dtype=F32).reshape(self.A))
        b = np.ascontiguousarray(np.asarray(t_m, dtype=F32).reshape(self.A))
        self._chk(self.L.p2pmg_set_temperatures(self._ctx, a, b), "set_temperatures")

    def get_temperatures(self):
        a = np.empty(self.A, F32)
        b = np.empty(self.A, F32)
        self._chk(self.L.p2pmg_get_temperatures(self._ctx, a, b), "get_temperatures")
        return a.reshape(self.S, self.N), b.reshape(self.S, self.N)

    def reset_temperatures_philox(self, episode: int, sigma: float = 0.3):
        self._chk(self.L.p2pmg_reset_temperatures_philox(self._ctx, int(episode), float(sigma)), "reset_philox")

    def set_replay_codes(self, codes):
        """uint8 [T, R+1, S, N] (or [T, R+1, N] when S == 1); 255 = greedy."""
        c = np.ascontiguousarray(np.asarray(codes, dtype=np.uint8).reshape(self.T, self.R + 1, self.A))
        self._chk(self.L.p2pmg_set_replay_codes(self._ctx, c.ctypes.data), "set_replay_codes")

    # ----------------------------------------------------------------- Q tables
    def zero_q(self):
        self._chk(self.L.p2pmg_zero_q(self._ctx), "zero_q")

    def get_q(self, first: int = 0, count: Optional[int] = None, dtype=np.float64):
        count = self.n_tables - first if count is None else count
        out = np.empty((count, *self.q_shape), dtype=dtype)
        code = _lib.Q_F64 if np.dtype(dtype) == np.float64 else _lib.Q_F32
        self._chk(self.L.p2pmg_get_q(self._ctx, first, count, out.ctypes.data, code), "get_q")
        return out

    def set_q(self, tables, first: int = 0):
        t = np.asarray(tables)
        dtype = np.float64 if t.dtype == np.float64 else np.float32
        t = np.ascontiguousarray(t.astype(dtype, copy=False).reshape(-1, self.n_states * self.q_shape[-1]))
        code = _lib.Q_F64 if dtype == np.float64 else _lib.Q_F32
        self._chk(self.L.p2pmg_set_q(self._ctx, first, t.shape[0], t.ctypes.data, code), "set_q")

    # ----------------------------------------------------------------- heterogeneous agents / storage
    def set_hp_levels(self, levels):
        """Per-agent heat-pump power of actions 0..2 in W, [S, N, 3] (0 for agents without one)."""
        lv = np.ascontiguousarray(np.asarray(levels, dtype=F32).reshape(self.A, 3))
        self._chk(self.L.p2pmg_set_hp_levels(self._ctx, lv), "set_hp_levels")

    def set_battery(self, capacity=None, min_soc=0.1, max_soc=0.9, efficiency=0.9, soc0=None):
        """Battery per agent (capacity [S, N] in J, 0 = none); None disables storage."""
        if capacity is None:
            self._chk(self.L.p2pmg_set_battery(self._ctx, None, 0.1, 0.9, 1.0, None), "set_battery")
            return
        def per_agent(x):
            x = np.asarray(x, np.float64)
            return np.ascontiguousarray(x.reshape(self.A) if x.size == self.A else np.broadcast_to(x, (self.A,)))
        cap = per_agent(capacity)
        s0 = None if soc0 is None else per_agent(soc0)
        self._chk(self.L.p2pmg_set_battery(self._ctx, cap.ctypes.data, float(min_soc), float(max_soc),
                                           float(efficiency), None if s0 is None else s0.ctypes.data), "set_battery")

    def get_soc(self):
        out = np.empty(self.A, np.float64)
        self._chk(self.L.p2pmg_get_soc(self._ctx, out.ctypes.data), "get_soc")
        return out.reshape(self.S, self.N)

    def battery_seq(self, balance, soc, capacity, min_soc=0.1, max_soc=0.9, efficiency=0.9):
        """Battery rule (agent.py:138-153) over per-agent sequences [agents, steps] on the device."""
        b = np.ascontiguousarray(np.atleast_2d(np.asarray(balance, np.float64)))
        ag, st = b.shape
        ob = np.empty_like(b)
        sh = np.empty_like(b)
        s_ = np.ascontiguousarray(np.broadcast_to(np.asarray(soc, np.float64), (ag,))).copy()
        cap = np.ascontiguousarray(np.broadcast_to(np.asarray(capacity, np.float64), (ag,)))
        self._chk(self.L.p2pmg_battery_seq(self._ctx, ag, st, b.ctypes.data, ob.ctypes.data, sh.ctypes.data,
                                           s_.ctypes.data, cap.ctypes.data, float(min_soc), float(max_soc),
                                           float(efficiency)), "battery_seq")
        return ob, sh, s_

    # ----------------------------------------------------------------- shared policy table
    def apply_q_delta(self):
        self._chk(self.L.p2pmg_apply_q_delta(self._ctx), "apply_q_delta")

    def get_q_delta(self):
        out = np.empty((self.n_states, self.q_shape[-1]), np.int64)
        self._chk(self.L.p2pmg_get_q_delta(self._ctx, out.ctypes.data), "get_q_delta")
        return out.reshape(self.q_shape)

    def set_q_delta(self, delta):
        d = np.ascontiguousarray(np.asarray(delta, np.int64).reshape(self.n_states, self.q_shape[-1]))
        self._chk(self.L.p2pmg_set_q_delta(self._ctx, d.ctypes.data), "set_q_delta")

    def comm_init(self, unique_id: bytes, rank: int, nranks: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._chk(self.L.p2pmg_comm_init(self._ctx, buf, rank, nranks), "comm_init")

    def allreduce_q_delta(self):
        self._chk(self.L.p2pmg_allreduce_q_delta(self._ctx), "allreduce_q_delta")

    def comm_nranks(self) -> int:
        """Ranks of the RCCL communicator (1 without one)."""
        n = C.c_int(0)
        self._chk(self.L.p2pmg_comm_nranks(self._ctx, C.byref(n)), "comm_nranks")
        return int(n.value)

    def allreduce_metrics(self):
        """(sum of the last episode's rewards over every rank's scenarios, scenario count): the
        local sum on the device, then an RCCL all-reduce when a communicator exists."""
        out = np.zeros(2, np.float64)
        self._chk(self.L.p2pmg_allreduce_metrics(self._ctx, out.ctypes.data), "allreduce_metrics")
        return float(out[0]), int(out[1])

    def table_hash_allgather(self) -> np.ndarray:
        """64-bit fingerprints of every rank's Q-table replica, in rank order (RCCL all-gather)."""
        out = np.zeros(max(1, self.comm_nranks()), np.uint64)
        self._chk(self.L.p2pmg_table_hash_allgather(self._ctx, out.ctypes.data), "table_hash_allgather")
        return out

    # ----------------------------------------------------------------- the hot path
    def run_episode(self, mode: str = "train", rng: str = "replay", episode: int = 0, epsilon: float = 0.81,
                    record: Sequence[str] = (), philox: str = "auto", kernel: str = "auto",
                    scen_per_wave: int = 0, reset_sigma: Optional[float] = None,
                    next_epsilon: Optional[float] = None):
        """Launch one episode for all scenarios (asynchronous; stream-ordered).
        philox: 'auto' | 'prepass' | 'inkernel' placement of the Philox draws.
        kernel: 'auto' (the fast per-agent-table kernel whenever it applies) | 'general' | 'tile'
            (the general kernel's LDS-tile form, which every N outside {1..8, 16} runs, at any N).
        scen_per_wave: fast kernel only, scenarios per 64-lane wave (0 = full waves).
        reset_sigma: end the episode with agent.reset() (community.py:181), i.e. exactly
        reset_temperatures_philox(episode + 1, reset_sigma), fused into the episode launch.
        next_epsilon: the next episode's epsilon when the caller knows its decay schedule
        (community.py:279-286), so that the speculative pre-pass this launch writes for
        episode + 1 is a hit (None: the same epsilon)."""
        mask = 0
        for r in record:
            mask |= _lib.REC[r]
        flags = {"auto": 0, "prepass": _lib.FLAG_PHILOX_PREPASS, "inkernel": _lib.FLAG_PHILOX_INKERNEL}[philox]
        flags |= {"auto": 0, "general": _lib.FLAG_GENERAL_KERNEL, "tile": _lib.FLAG_TILE_KERNEL}[kernel]
        if reset_sigma is not None:
            flags |= _lib.FLAG_RESET_T0
        if next_epsilon is not None:  # a guess of 0.0 is a real guess (P2PMG_FLAG_NEXT_EPSILON)
            flags |= _lib.FLAG_NEXT_EPSILON
        args = _lib.EpisodeArgs(_lib.MODE_TRAIN if mode == "train" else _lib.MODE_GREEDY,
                                _lib.RNG_REPLAY if rng == "replay" else _lib.RNG_PHILOX,
                                int(episode), mask, float(epsilon), flags, int(scen_per_wave),
                                float(reset_sigma or 0.0), float(next_epsilon or 0.0))
        self._chk(self.L.p2pmg_run_episode(self._ctx, C.byref(args)), "run_episode")
        self._recorded = mask

    def run_episodes(self, episode: int, epsilons, reset_sigma: Optional[float] = None,
                     next_epsilons=None, scen_per_wave: int = 0, record: Sequence[str] = ()):
        """Train len(epsilons) consecutive episodes with Philox draws (community.py:279-286's loop
        body): episode + k at epsilons[k], each ending with the T0 reset when reset_sigma is given.
        Where the fast kernel applies, chained launches run up to 64 episodes each, every wave
        going through its episodes back to back; results are those of run_episode per episode,
        bit for bit.  next_epsilons: the next call's epsilons (its speculative pre-pass).  record:
        what the last episode leaves in the record buffers (as after run_episode per episode)."""
        eps = np.ascontiguousarray(epsilons, dtype=np.float64).reshape(-1)
        flags = _lib.FLAG_RESET_T0 if reset_sigma is not None else 0
        mask = 0
        for r in record:
            mask |= _lib.REC[r]
        args = _lib.EpisodeArgs(_lib.MODE_TRAIN, _lib.RNG_PHILOX, int(episode), mask, float(eps[0]), flags,
                                int(scen_per_wave), float(reset_sigma or 0.0), 0.0)
        nxt = None if next_epsilons is None else np.ascontiguousarray(next_epsilons, dtype=np.float64).reshape(-1)
        self._chain_eps = (eps, nxt)  # kept alive for the call
        self._chk(self.L.p2pmg_run_episodes(self._ctx, C.byref(args), int(eps.size), eps,
                                            0 if nxt is None else int(nxt.size),
                                            None if nxt is None else nxt.ctypes.data), "run_episodes")
        self._recorded = mask
        self._chain_len = int(eps.size)

    def episode_rewards(self) -> np.ndarray:
        """[n, S] episode rewards (community.py:179) of every episode of the last run_episodes."""
        n = getattr(self, "_chain_len", 0)
        out = np.empty((n, self.S), F32)
        self._chk(self.L.p2pmg_get_episode_rewards(self._ctx, n, out), "get_episode_rewards")
        return out

    def run_rule_episode(self, record: Sequence[str] = ()):
        """CommunityMicrogrid.run of a RuleAgent community (community.py:95-123, 237-238; agent.py:106-136):
        hysteresis heat pumps, no policy, R = 0.  Records: cost, grid, p2p, t_in, action (0 off, 2 on)."""
        mask = 0
        for r in record:
            mask |= _lib.REC[r]
        self._chk(self.L.p2pmg_run_rule_episode(self._ctx, mask), "run_rule_episode")
        self._recorded = mask

    def set_hp_state(self, on):
        """RuleAgent HeatPump.power per agent (0/1), [S, N]."""
        a = np.ascontiguousarray(np.asarray(on, dtype=F32).reshape(self.A))
        self._chk(self.L.p2pmg_set_hp_state(self._ctx, a), "set_hp_state")

    def get_hp_state(self) -> np.ndarray:
        out = np.empty(self.A, F32)
        self._chk(self.L.p2pmg_get_hp_state(self._ctx, out), "get_hp_state")
        return out.reshape(self.S, self.N)

    def prepass_stats(self):
        """(hits, misses): fast-path launches whose step pre-pass the previous launch had produced
        beside its own episode, and launches that had to run it themselves."""
        h, m = C.c_int64(0), C.c_int64(0)
        self._chk(self.L.p2pmg_prepass_stats(self._ctx, C.byref(h), C.byref(m)), "prepass_stats")
        return int(h.value), int(m.value)

    def last_kernel(self) -> str:
        """Name of the kernel the last episode launch ran (fast or general path)."""
        return (self.L.p2pmg_last_kernel(self._ctx) or b"").decode()

    def last_kernel_ms(self) -> float:
        ms = C.c_float(0)
        self._chk(self.L.p2pmg_last_kernel_ms(self._ctx, C.byref(ms)), "last_kernel_ms")
        return float(ms.value)

    def kernel_times(self, max_n: int = 4096) -> np.ndarray:
        """HIP-event durations (ms) of the episode kernels since the last reset (syncs)."""
        out = np.empty(max_n, F32)
        n = C.c_int(0)
        self._chk(self.L.p2pmg_kernel_times(self._ctx, out, max_n, C.byref(n)), "kernel_times")
        return out[:n.value].copy()

    def collective_ms(self):
        """(total ms, count) of the data-path RCCL collectives (shared-table delta all-reduce, DQN
        gradient-segment all-gather) since the last reset_kernel_times, every call counted (HIP
        events on the context's stream; syncs)."""
        ms, n = C.c_double(0.0), C.c_int(0)
        self._chk(self.L.p2pmg_collective_ms(self._ctx, C.byref(ms), C.byref(n)), "collective_ms")
        return float(ms.value), int(n.value)

    def reset_kernel_times(self):
        self._chk(self.L.p2pmg_reset_kernel_times(self._ctx), "reset_kernel_times")

    def set_timing_period(self, period: int):
        """Stamp timing events on every period-th episode launch only (timing-only setting)."""
        self._chk(self.L.p2pmg_set_timing_period(self._ctx, int(period)), "set_timing_period")

    def get_record(self, name: str) -> np.ndarray:
        """[T, S, N] for per-step records, [T, R+1, S, N] for action/index."""
        bit = _lib.REC[name]
        if name in ("action", "index"):
            shape = (self.T, self.R + 1, self.S, self.N)
            dt = np.uint8 if name == "action" else np.int32
        else:
            shape = (self.T, self.S, self.N)
            dt = np.float32
        out = np.empty(shape, dtype=dt)
        self._chk(self.L.p2pmg_get_record(self._ctx, bit, out.ctypes.data), f"get_record({name})")
        return out

    def get_records(self, names: Sequence[str]) -> Dict[str, np.ndarray]:
        return {n: self.get_record(n) for n in names}

    def episode_reward(self) -> np.ndarray:
        out = np.empty(self.S, F32)
        self._chk(self.L.p2pmg_get_episode_reward(self._ctx, out), "episode_reward")
        return out

    # ----------------------------------------------------------------- primitives
    def rc_step(self, t_out, t_in, t_m, hp):
        """Batched heating.temperature_simulation (heating.py:37-56) on the device."""
        arrs = [np.ascontiguousarray(np.asarray(x, dtype=F32).ravel()) for x in np.broadcast_arrays(t_out, t_in, t_m, hp)]
        n = arrs[0].size
        a = np.empty(n, F32)
        b = np.empty(n, F32)
        self._chk(self.L.p2pmg_rc_step(self._ctx, n, *arrs, a, b), "rc_step")
        shape = np.broadcast(t_out, t_in, t_m, hp).shape
        return a.reshape(shape), b.reshape(shape)

    def fdiv_check(self, a, b):
        """The kernels' fast f32 quotients of a / b and the IEEE one: [n, 4] (p2pmg_fdiv_check)."""
        a = np.ascontiguousarray(np.asarray(a, F32).ravel())
        b = np.ascontiguousarray(np.asarray(b, F32).ravel())
        out = np.empty((a.size, 4), F32)
        self._chk(self.L.p2pmg_fdiv_check(self._ctx, a.size, a.ctypes.data, b.ctypes.data, out.ctypes.data), "fdiv_check")
        return out

    def fdiv64_check(self, a, b):
        """The kernels' fast f64 quotients and the IEEE one: [n, 3] (p2pmg_fdiv64_check)."""
        a = np.ascontiguousarray(np.asarray(a, np.float64).ravel())
        b = np.ascontiguousarray(np.asarray(b, np.float64).ravel())
        out = np.empty((a.size, 3), np.float64)
        self._chk(self.L.p2pmg_fdiv64_check(self._ctx, a.size, a.ctypes.data, b.ctypes.data, out.ctypes.data),
                  "fdiv64_check")
        return out

    def state_indices(self, obs):
        """Batched QActor._get_state_indices (rl.py:89-95) on the device; obs [..., 4]."""
        o = np.ascontiguousarray(np.asarray(obs, dtype=F32).reshape(-1, 4))
        idx = np.empty(o.shape, np.int32)
        self._chk(self.L.p2pmg_state_indices(self._ctx, o.shape[0], o, idx.ctypes.data), "state_indices")
        return idx.reshape(np.shape(obs))


def _q_calls(eng: "DeviceCommunityBatch", agents, s_obs, codes, rewards=None, ns_obs=None, train=False):
    agents = np.ascontiguousarray(np.asarray(agents, dtype=np.int32).ravel())
    n = agents.size
    s_obs = np.ascontiguousarray(np.asarray(s_obs, dtype=F32).reshape(n, 4))
    codes = np.ascontiguousarray(np.asarray(codes, dtype=np.uint8).ravel())
    acts = np.empty(n, np.int32)
    qv = np.empty(n, np.float64)
    if train:
        rewards = np.ascontiguousarray(np.asarray(rewards, dtype=F32).ravel())
        ns_obs = np.ascontiguousarray(np.asarray(ns_obs, dtype=F32).reshape(n, 4))
    eng._chk(eng.L.p2pmg_q_calls(eng._ctx, n, agents.ctypes.data, s_obs.ctypes.data, codes.ctypes.data,
                                 rewards.ctypes.data if train else None, ns_obs.ctypes.data if train else None,
                                 int(bool(train)), acts.ctypes.data, qv.ctypes.data), "q_calls")
    return acts, qv


DeviceCommunityBatch.q_calls = _q_calls


def comm_unique_id() -> bytes:
    """ncclGetUniqueId through libp2pmg (RCCL loaded at run time); rank 0 shares it."""
    buf = (C.c_uint8 * 128)()
    _lib.check(_lib.lib().p2pmg_comm_unique_id(buf), what="comm_unique_id")
    return bytes(buf)


def unpack_index(packed: np.ndarray) -> np.ndarray:
    """P2PMG_REC_INDEX packing -> [..., 4] (it, iT, ib, ip)."""
    p = np.asarray(packed, dtype=np.int64)
    return np.stack([p & 0xFF, (p >> 8) & 0xFF, (p >> 16) & 0xFF, (p >> 24) & 0xFF], axis=-1)
