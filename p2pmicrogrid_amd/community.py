"""Community orchestration (mirrors microgrid/community.py:33-423).

``CommunityMicrogrid(timeline, agents, rounds)`` keeps the reference's interface; each
``train_episode`` / ``run`` is ONE device launch (p2pmg_run_episode) over the whole episode:
negotiation rounds, market clearing, costs, rewards, TD updates and the RC update of every
agent.  Exploration is replayed from the global ``np.random`` in the reference's consumption
order, so a seeded reference script and this package draw identical
streams.  Database logging, plotting and the REST data client are out of scope.
"""
from __future__ import annotations

import collections
import os
import statistics
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np

from . import database as db
from . import dataset as ds
from . import setup
from .agent import ActingAgent, Agent, DQNAgent, GridAgent, QAgent, RuleAgent, agent_kind
from .engine import DeviceCommunityBatch, price_table
from .environment import env
from .heating import HeatPump, HPHeating
from .production import PV, Prosumer
from .rng import ReferenceRNG, dqn_episode_draws, python_random
from .storage import BatteryStorage, NoStorage

F32 = np.float32


class CommunityMicrogrid:

    def __init__(self, timeline, agents: List[ActingAgent], rounds: int, q_dtype: Optional[str] = None,
                 device: Optional[int] = None, *, battery_rule: bool = False) -> None:
        """community.py:35-43.  ``battery_rule`` (an extension, off by default): apply the battery
        rule of RuleAgent._update_storage (agent.py:138-153) to the net power of every agent that
        carries a BatteryStorage, inside the episode kernel.  The reference never calls that rule
        from an RL agent (agent.py:200-213), so by default a battery is inert, exactly as there:
        powers and costs equal the NoStorage run and the SoC stays put."""
        self.timeline = timeline
        self.time_length = len(timeline)
        self.agents = agents
        self.grid = GridAgent()
        self._rounds = rounds
        self.decisions = np.zeros((len(env), self._rounds + 1, len(self.agents)))
        self._q_dtype = q_dtype or setup.q_dtype
        self._device = setup.device if device is None else device
        self._engine: Optional[DeviceCommunityBatch] = None
        self._uploaded: Dict[str, Any] = {}
        self._rng = ReferenceRNG()
        kinds = {agent_kind(a) for a in agents}
        if len(kinds) != 1 or None in kinds:
            raise ValueError(f"a community needs agents of one learner kind, got {kinds}")
        self._dqn = kinds == {"dqn"}
        self._rule = kinds == {"rule"}
        self._battery_rule = bool(battery_rule)
        if self._battery_rule and self._dqn:
            raise NotImplementedError("the in-kernel battery rule is supported for tabular communities")
        if self._battery_rule and self._rule:
            raise NotImplementedError("rule_episode_kernel does not apply the battery rule (the reference's "
                                      "RuleAgent.take_decision never calls _update_storage, agent.py:114-128)")

    # ------------------------------------------------------------ device state
    def _new_dqn_engine(self, T, N):
        from .dqn import DeviceDQNBatch
        old = self._engine
        carry = None
        if old is not None:  # horizon changed: carry networks, Adam state and memories over
            carry = ({w: old.get_weights(w) for w in ("adam_m", "adam_v")}, old.get_buffer(), old.step)
            for a in self.agents:
                a.actor.q_network.unbind()
                a.trainer.target_network.unbind()
            old.close()
        eng = DeviceDQNBatch(1, N, self._rounds, T, device=self._device, init_seed=None)
        for i, a in enumerate(self.agents):
            a.trainer.bind(eng, i)
        if carry is not None:
            for w, v in carry[0].items():
                eng.set_weights(w, v)
            eng.set_buffer(*carry[1])
            eng.step = carry[2]
        return eng

    def _ensure_engine(self) -> DeviceCommunityBatch:
        T, N = len(env), len(self.agents)
        if self._dqn and (self._engine is None or self._engine.T != T):
            self._engine = self._new_dqn_engine(T, N)
            self._uploaded = {}
        if self._engine is None or self._engine.T != T:
            if self._engine is not None:  # horizon changed: carry the learned tables over
                tables = self._engine.get_q()
            else:
                tables = None
            self._engine = DeviceCommunityBatch(1, N, self._rounds, T, q_dtype=self._q_dtype, device=self._device)
            for i, a in enumerate(self.agents):
                if self._rule:  # no policy to bind
                    continue
                if tables is None:
                    a.actor.bind(self._engine, i)
                else:
                    a.actor._engine = None
                    a.actor.set_qtable(tables[i])
                    a.actor.bind(self._engine, i)
            self._uploaded = {}
        eng = self._engine
        if self._uploaded.get("env") != env.version:
            time_f, t_out = env.arrays()
            eng.set_env(time_f, t_out, *price_table(time_f))
            self._uploaded["env"] = env.version
        prof_key = tuple((id(a._load), id(a.pv), id(getattr(a.pv, "pv", None) and a.pv.pv.production))
                         for a in self.agents)
        if self._uploaded.get("prof") != prof_key:
            load = np.stack([a.load_series(T) for a in self.agents])[None]
            pv = np.stack([a.pv.series(T) for a in self.agents])[None]
            eng.set_profiles(load, pv)
            eng.set_max_in(np.array([F32(a.max_in) for a in self.agents], F32)[None])
            self._uploaded["prof"] = prof_key
        return eng

    def _push_temperatures(self, eng):
        t_in = np.array([a.heating.temperature[0] for a in self.agents], F32)
        t_m = np.array([a.heating.building_mass_temperature[0] for a in self.agents], F32)
        eng.set_temperatures(t_in[None], t_m[None])
        self._push_storage(eng)

    def _batteries(self) -> List[Optional[BatteryStorage]]:
        return [a.storage if isinstance(a.storage, BatteryStorage) else None for a in self.agents]

    def _push_storage(self, eng):
        """With ``battery_rule``: capacities and SoC of the agents' batteries (NoStorage = capacity
        0) before a launch; the kernel applies the rule to every round's net power.  Without it
        nothing is uploaded (the reference's inert battery)."""
        bats = self._batteries()
        if not (self._battery_rule and any(bats)):
            if self._uploaded.get("battery"):
                eng.set_battery(None)
                self._uploaded["battery"] = False
            return
        ref = next(b for b in bats if b is not None).battery
        for b in bats:
            if b is not None and (b.battery.min_soc, b.battery.max_soc, b.battery.efficiency) != \
                    (ref.min_soc, ref.max_soc, ref.efficiency):
                raise ValueError("one community's batteries must share min_soc, max_soc and efficiency")
        cap = np.array([0.0 if b is None else b.capacity for b in bats])[None]
        soc = np.array([0.0 if b is None else b.soc for b in bats])[None]
        eng.set_battery(cap, ref.min_soc, ref.max_soc, ref.efficiency, soc0=soc)
        self._uploaded["battery"] = True

    def _pull_storage(self, eng, T: int):
        """After a launch.  The reference's inert battery: each BatteryStorage steps T times
        (storage.py:66-68), so its history holds T entries of its unchanged SoC.  With
        ``battery_rule``: the device's final SoC; the per-step SoC is not recorded on the device,
        so the history is left as it was (only the step counter advances)."""
        bats = [b for b in self._batteries() if b is not None]
        if self._uploaded.get("battery"):
            soc = eng.get_soc()[0]
            for b, x in zip(self._batteries(), soc):
                if b is not None:
                    b.set_soc(x)
                    b._time += T
            return
        for b in bats:
            for _ in range(T):
                b.step()

    def _pull_records(self, eng, T):
        act = eng.get_record("action")[:, :, 0, :]  # [T, R+1, N]
        levels = np.array([a.heating.hp.max_power for a in self.agents])
        self.decisions = np.array([0.0, 0.5, 1.0])[act] * levels[None, None, :]
        return act

    # ------------------------------------------------------------ the reference API
    def train_episode(self, all_rewards=None, all_losses=None, _rewards=None, _losses=None) -> Tuple[float, float]:
        """community.py:149-182: one training episode; returns (sum_t mean_i reward, mean loss)
        (the loss is 0 for tabular agents, agent.py:298)."""
        if self._dqn:
            return self._train_episode_dqn()
        if self._rule:  # community.py:160-171 calls agent.get_reward / agent.train, which RuleAgent lacks
            raise AttributeError("'RuleAgent' object has no attribute 'get_reward': rule-based communities "
                                 "only run() (agent.py:106-153)")
        eng = self._ensure_engine()
        T, N = eng.T, eng.N
        self._push_temperatures(eng)
        eps = [a.actor._epsilon for a in self.agents]
        codes = self._rng.episode_codes(T, self._rounds, N, eps)
        eng.set_replay_codes(codes)
        eng.run_episode("train", "replay", epsilon=float(eps[0]), record=("reward", "action"))
        self._pull_storage(eng, T)
        self._pull_records(eng, T)
        self.last_rewards = eng.get_record("reward")[:, 0, :]
        avg_reward = float(eng.episode_reward()[0])
        for agent in self.agents:  # reset iterators + new T0 (community.py:172-174)
            agent.reset()
        return avg_reward, 0.0

    def run(self) -> Tuple[np.ndarray, np.ndarray]:
        """community.py:95-123: greedy rollout; returns (grid + p2p power [T, N], costs [T, N])."""
        if self._rule:
            return self._run_rule()
        eng = self._ensure_engine()
        T = eng.T
        self._push_temperatures(eng)
        rec = ("grid", "p2p", "cost", "t_in", "action")
        eng.run_episode("greedy", record=rec)
        self._pull_storage(eng, T)
        r = eng.get_records(rec)
        self._pull_records(eng, T)
        t_in, t_m = eng.get_temperatures()
        hist = r["t_in"][:, 0, :]
        for i, a in enumerate(self.agents):
            a.heating._history = [float(x) for x in hist[:, i]]
            a.heating._power_history = list(self.decisions[:, -1, i])
            a.heating.set_state(t_in[0, i], t_m[0, i])
        power = (r["grid"][:, 0, :] + r["p2p"][:, 0, :]).astype(F32)
        return power, r["cost"][:, 0, :]

    def _run_rule(self) -> Tuple[np.ndarray, np.ndarray]:
        """run() of a RuleAgent community: one rule_episode_kernel launch (R = 0)."""
        if self._rounds != 0:
            raise ValueError("RuleAgent communities run with rounds = 0: with more rounds the reference's "
                             "tensor_diag_part on the (N, 1) proposal stack fails (community.py:76)")
        eng = self._ensure_engine()
        self._push_temperatures(eng)
        levels = np.array([[0.0, 0.5, 1.0]], F32) * np.array([[a.heating.hp.max_power] for a in self.agents], F32)
        eng.set_hp_levels(levels[None])
        eng.set_hp_state(np.array([float(np.asarray(a.heating.hp.power).reshape(-1)[0]) for a in self.agents], F32)[None])
        rec = ("grid", "p2p", "cost", "t_in", "action")
        eng.run_rule_episode(record=rec)
        r = eng.get_records(rec)
        self._pull_records(eng, eng.T)
        t_in, t_m = eng.get_temperatures()
        on = eng.get_hp_state()[0]
        hist = r["t_in"][:, 0, :] if r["t_in"].ndim == 3 else r["t_in"]
        for i, a in enumerate(self.agents):
            a.heating._history = [float(x) for x in hist[:, i]]
            a.heating._power_history = list(self.decisions[:, -1, i])
            a.heating.set_state(t_in[0, i], t_m[0, i])
            a.heating.hp.power = float(on[i])
        power = (r["grid"][:, 0, :] + r["p2p"][:, 0, :]).astype(F32)
        return power, r["cost"][:, 0, :]

    # ------------------------------------------------------------ DQN agents
    def _counts(self, eng):
        _, added = eng.get_buffer()
        return np.minimum(added, eng.capacity)

    def _train_episode_dqn(self) -> Tuple[float, float]:
        eng = self._ensure_engine()
        T, N = eng.T, eng.N
        self._push_temperatures(eng)
        eps = [a.actor._epsilon for a in self.agents]
        codes, samples = dqn_episode_draws(python_random(), self._rng.rs, T, self._rounds, N, eps,
                                           counts=self._counts(eng))
        eng.set_replay_codes(codes)
        eng.set_samples(samples)
        eng.run_episode("train", "replay", epsilon=float(eps[0]), record=("reward", "action", "loss"))
        self._pull_records(eng, T)
        self.last_rewards = eng.get_record("reward")[:, 0, :]
        self.last_losses = eng.get_record("loss")[:, 0, :]
        avg_reward = float(eng.episode_reward()[0])
        for agent in self.agents:
            agent.reset()
        return avg_reward, float(np.mean(self.last_losses, dtype=np.float32))

    def init_buffers(self) -> None:
        """community.py:125-147: five episodes of memory with the exploring actors (no training),
        then Trainer.initialize_target per agent.  Tabular agents have no memory."""
        if not self._dqn:
            return
        eng = self._ensure_engine()
        T, N = eng.T, eng.N
        for _ in range(5):
            self._push_temperatures(eng)
            eps = [a.actor._epsilon for a in self.agents]
            codes, _ = dqn_episode_draws(python_random(), self._rng.rs, T, self._rounds, N, eps)
            eng.set_replay_codes(codes)
            eng.run_episode("fill", "replay", epsilon=float(eps[0]))
            for agent in self.agents:
                agent.reset()
        for agent in self.agents:
            agent.trainer.initialize_target()

    # ------------------------------------------------------------ per-step API (host glue)
    # For callers that step the community themselves, as community.py:149-182 does: the same
    # TF op order on f32 host values (canonical sequential sums), with the agents'
    # per-step methods calling the device for the learner and the RC update.
    def _assign_powers(self, p2p_power) -> Tuple[np.ndarray, np.ndarray]:
        """community.py:45-54: opposite-sign pairs exchange min(|P_ij|, |P_ji|), the rest is grid."""
        P = np.asarray(p2p_power, F32)
        p_match = np.where(np.sign(P) != np.sign(P.T), P, F32(0.0)).astype(F32)
        exchange = (np.sign(p_match) * np.minimum(np.abs(p_match), np.abs(p_match).T)).astype(F32)
        diff = (P - exchange).astype(F32)
        p_grid = np.zeros(P.shape[0], F32)
        p_p2p = np.zeros(P.shape[0], F32)
        for j in range(P.shape[1]):
            p_grid = (p_grid + diff[:, j]).astype(F32)
            p_p2p = (p_p2p + exchange[:, j]).astype(F32)
        return p_grid, p_p2p

    def _compute_costs(self, grid_power, peer_power, buying_price, injection_price, p2p_price) -> np.ndarray:
        """community.py:56-65 (prices [T] or scalars; powers [..., N])."""
        g, pp = np.asarray(grid_power, F32), np.asarray(peer_power, F32)
        buy = np.asarray(buying_price, F32).reshape(-1)[:, None]
        inj = np.asarray(injection_price, F32).reshape(-1)[:, None]
        p2p = np.asarray(p2p_price, F32).reshape(-1)[:, None]
        c = (np.where(g >= F32(0.0), g * buy, g * inj) + pp * p2p).astype(F32)
        return ((((c * F32(setup.TIME_SLOT)) / F32(setup.MINUTES_PER_HOUR)).astype(F32)) * F32(1e-3)).astype(F32)

    def _run(self, time: int, state, training: bool = False):
        """community.py:67-93: prices, R + 1 Jacobi negotiation rounds (each agent answers the
        previous round's column, diagonal zeroed), market clearing on the final proposals."""
        st = np.asarray(state.numpy() if hasattr(state, "numpy") else state, F32).reshape(-1)
        buying_price, injection_price = self.grid.take_decision(st)
        p2p_price = ((F32(buying_price) + np.asarray(injection_price, F32)) / F32(2)).astype(F32)
        N = len(self.agents)
        P = np.zeros((N, N), F32)
        for r in range(self._rounds + 1):
            P = (P - np.diag(np.diag(P))).astype(F32)
            rows = []
            for i, agent in enumerate(self.agents):
                col = (-P[:, i]).astype(F32)
                if training:
                    action, _ = agent(st[None], col)
                else:
                    action, _ = agent.take_decision(st[None], col)
                rows.append(np.asarray(action, F32).reshape(-1))
            P = np.stack(rows).astype(F32)
            for a, agent in enumerate(self.agents):
                self.decisions[time, r, a] = float(agent.heating.power[0])
        p_grid, p_p2p = self._assign_powers(P)
        return p_grid, p_p2p, F32(buying_price), np.asarray(injection_price, F32), p2p_price

    def _step(self) -> None:
        for agent in self.agents:
            agent.step()
        self.grid.step()

    def reset(self) -> None:
        for agent in self.agents:
            agent.reset()
        self.grid.reset()
        self.decisions = np.zeros((len(env), self._rounds + 1, len(self.agents)))


def get_community(agent_constructor: Callable[..., ActingAgent], n_agents: int,
                  homogeneous: bool = False, rounds_: Optional[int] = None) -> CommunityMicrogrid:
    """community.py:198-234 with the same np.random consumption (ratings, then per agent
    HPHeating T_m, T_in) and the same derived quantities."""
    env_df, agent_dfs = ds.get_train_data()
    if homogeneous:
        agent_dfs = [agent_dfs[0]] * n_agents
    timeline = env_df['time'].map(lambda t: int(t * setup.MINUTES_PER_HOUR / setup.TIME_SLOT * setup.HOURS_PER_DAY))
    agents: List[ActingAgent] = []
    rng = ReferenceRNG()
    load_ratings, pv_ratings = rng.community_ratings(n_agents, homogeneous)
    Agent.reset_ids()
    for i in range(n_agents):
        max_power = max(load_ratings[i], pv_ratings[i])
        safety = 1.1
        agent_load = ds.dataframe_to_dataset(agent_dfs[i % len(agent_dfs)]['load'] * load_ratings[i] * 1e3)
        agent_pv = ds.dataframe_to_dataset(agent_dfs[i % len(agent_dfs)]['pv'] * pv_ratings[i] * 1e3)
        agents.append(agent_constructor(agent_load,
                                        Prosumer(PV(peak_power=pv_ratings[i] * 1e3, production=agent_pv)),
                                        NoStorage(),
                                        HPHeating(HeatPump(cop=3.0, max_power=3 * 1e3, power=0.0), 21.0, rng=rng),
                                        max_in=max_power * safety * 1e3,
                                        max_out=-(max_power + safety * 1e3)))
    env.setup(ds.dataframe_to_dataset(env_df))
    return CommunityMicrogrid(timeline, agents, setup.rounds if rounds_ is None else rounds_)


def get_rule_based_community(n_agents: int, homogeneous: bool) -> CommunityMicrogrid:
    """community.py:237-238, with rounds = 0: a RuleAgent ignores the proposals, and with more
    rounds the reference's run() fails on the (N, 1) proposal stack (tensor_diag_part)."""
    return get_community(RuleAgent, n_agents, homogeneous=homogeneous, rounds_=0)


def get_rl_based_community(n_agents: int, homogeneous: bool) -> CommunityMicrogrid:
    """community.py:240-245"""
    if setup.implementation == 'tabular':
        return get_community(QAgent, n_agents, homogeneous=homogeneous)
    if setup.implementation == 'dqn':
        return get_community(DQNAgent, n_agents, homogeneous=homogeneous)
    raise ValueError(f"unknown implementation {setup.implementation!r}")


def setting_name(nr_agents=None, rounds=None, homogeneous=None) -> str:
    """community.py:423"""
    n = setup.nr_agents if nr_agents is None else nr_agents
    r = setup.rounds if rounds is None else rounds
    h = setup.homogeneous if homogeneous is None else homogeneous
    return f'{n}-multi-agent-com-rounds-{r}-{"homo" if h else "hetero"}'


def _set_day_profiles(community: CommunityMicrogrid, agent_dfs, rows=None) -> None:
    """community.py:306-311 / :386-391: each agent's load and PV of the evaluation data, scaled by
    the homogeneous ratings or by fresh N(0.7, 0.2) / N(4, 0.2) draws (load first, then PV, per
    agent: the reference's np.random consumption order)."""
    for i, agent in enumerate(community.agents):
        df = agent_dfs[i] if rows is None else agent_dfs[i].loc[rows]
        agent_load = ds.dataframe_to_dataset(df['load'] * (0.7e3 if setup.homogeneous
                                                           else np.random.normal(0.7, 0.2, 1) * 1e3))
        agent_pv = ds.dataframe_to_dataset(df['pv'] * (4e3 if setup.homogeneous
                                                       else np.random.normal(4, 0.2, 1) * 1e3))
        agent.set_profiles(agent_load, agent_pv)


def main(con=None, load_agents: bool = False, analyse: bool = False, *, episodes: Optional[int] = None,
         save: bool = True, verbose: bool = True) -> Dict[str, Any]:
    """community.py:248-321 (same positional signature: ``main(db_connection, load_agents=True,
    analyse=True)`` as at community.py:436).  Episodes ``setup.starting_episodes`` ..
    ``setup.max_episodes`` (``episodes`` = a shorter run), epsilon decay after episodes 0, 50, ...,
    running means to ``training_progress`` (db.log_training_progress) when a connection is given,
    ``.npy`` checkpoints every ``setup.save_episodes`` and at the end.  ``analyse`` runs the
    reference's greedy validation rollout (community.py:302-316: validation split, fresh rating
    draws, community.run) and returns its power/cost; the plots of analyse_community_output
    (data_analysis.py, out of scope) and save_times' ../data JSON are not produced."""
    setting = setting_name()
    if verbose:
        print(setting)
    community = get_rl_based_community(setup.nr_agents, homogeneous=setup.homogeneous)
    if load_agents:
        for agent in community.agents:
            agent.load_from_file(setting, setup.implementation)
    if setup.implementation == 'dqn':
        community.init_buffers()  # community.py:265-267
    rewards_q: collections.deque = collections.deque(maxlen=setup.min_episodes_criterion)
    errors_q: collections.deque = collections.deque(maxlen=setup.min_episodes_criterion)
    history = []
    t0 = time.time()
    last = setup.max_episodes if episodes is None else setup.starting_episodes + episodes
    for episode in range(setup.starting_episodes, last):
        reward, error = community.train_episode()
        rewards_q.append(reward)
        errors_q.append(error)
        history.append(reward)
        if episode % setup.min_episodes_criterion == 0:
            if verbose:
                print(f'Average reward: {statistics.mean(rewards_q):.3f}. '
                      f'Average error: {statistics.mean(errors_q):.3f}')
            for agent in community.agents:
                agent.actor.decay_exploration()
            db.log_training_progress(con, setting, setup.implementation, episode, statistics.mean(rewards_q),
                                     statistics.mean(errors_q))
        if save and (episode + 1) % setup.save_episodes == 0:
            for agent in community.agents:
                agent.save_to_file(setting, setup.implementation)
    if history:
        db.log_training_progress(con, setting, setup.implementation, last - 1, statistics.mean(rewards_q),
                                 statistics.mean(errors_q))
    if save:
        for agent in community.agents:
            agent.save_to_file(setting, setup.implementation)
    out: Dict[str, Any] = {"community": community, "rewards": history, "train_time": time.time() - t0}
    if analyse:  # community.py:302-316
        env_df, agent_dfs = ds.get_validation_data()
        env.setup(ds.dataframe_to_dataset(env_df))
        _set_day_profiles(community, agent_dfs)
        t_run = time.time()
        power, cost = community.run()
        out.update(run_time=time.time() - t_run, power=power, cost=cost,
                   cost_per_agent=np.sum(cost, axis=0, dtype=np.float32), decisions=community.decisions.copy())
    return out


def save_community_results(con, is_testing: bool, setting: str, day: int, community: CommunityMicrogrid,
                           cost: np.ndarray) -> None:
    """community.py:333-353: one test/validation row per agent-step (time, load, pv, T_in, heat-pump
    power, cost) and, for test runs, the heat-pump decision of every negotiation round."""
    time_f, _ = env.arrays()
    T = len(time_f)
    times = [float(x) for x in time_f]
    days = [int(day)] * T
    impl = setup.implementation
    for i, agent in enumerate(community.agents):
        row = (agent.load_series(T), agent.pv.series(T), agent.heating.get_history(),
               agent.heating._power_history, cost[:, i])
        if is_testing:
            db.log_test_results(con, setting, i, days, times, *row, impl)
        else:
            db.log_validation_results(con, setting, i, days, times, *row, impl)
    if is_testing:
        for a in range(len(community.agents)):
            for r in range(community._rounds + 1):
                db.log_rounds_decision(con, setting, a, days, times, r, community.decisions[:, r, a].tolist())


def load_and_run(con=None, is_testing: bool = False, analyse: bool = True) -> Dict[int, Dict[str, np.ndarray]]:
    """community.py:364-412 (same signature: ``load_and_run(db_connection, is_testing=True,
    analyse=False)`` as at community.py:437): greedy evaluation per test/validation day from the
    saved tables, a fresh start each day; rows go to the DB when a connection is given
    (save_community_results); returns per-day power, cost and decisions.  ``analyse`` would only
    plot (data_analysis.py, out of scope), so it changes nothing here."""
    setting = setting_name()
    community = get_rl_based_community(setup.nr_agents, homogeneous=setup.homogeneous)
    for agent in community.agents:
        agent.load_from_file(setting, setup.implementation)
    env_df, agent_dfs = ds.get_test_data() if is_testing else ds.get_validation_data()
    days = np.unique(env_df['day'])
    day_indices = {day: env_df['day'] == day for day in days}
    env_df = env_df.drop(axis=1, labels='day')
    if setup.homogeneous:
        agent_dfs = [agent_dfs[0]] * setup.nr_agents
    out = {}
    for day in days:
        env.setup(ds.dataframe_to_dataset(env_df[day_indices[day]]))
        community.reset()
        _set_day_profiles(community, agent_dfs, day_indices[day])
        power, cost = community.run()
        if con is not None:
            save_community_results(con, is_testing, setting, int(day), community, np.asarray(cost))
        out[int(day)] = {"power": power, "cost": cost, "decisions": community.decisions.copy()}
    return out
