"""Profiles with the reference's schema (mirrors microgrid/dataset.py).

The reference reads a private SQLite database filled from a credentialed REST API
(dataset.py:61-80, database.py:128-147); neither is available, so this module generates
synthetic data with the SAME schema and splits:

  time        slot / 96 in [0, 1)                       (dataset.py:43-44)
  temperature outdoor temperature, degC (not normalised)
  pv          PV shape normalised by its max             (dataset.py:50)
  l0..l4      five household loads normalised by max    (dataset.py:30, 46-48)

``dataframe_to_dataset`` returns a ``ProfileDataset`` holding the f32 array and its
``np.roll(-1)`` partner (dataset.py:98-103), which is what the environment and agents stream.
``scenario_batch`` builds the device inputs for S independent communities at once.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from datetime import datetime, timedelta
from typing import List, Optional, Tuple

import numpy as np
import pandas as pd

from . import setup

# Data splits (dataset.py:17-25)
data_month = 10
testing_days = [8, 9, 10, 19, 20]
validation_days = [18]
training_days = list(range(11, 18))

env_cols = ['day', 'time', 'temperature']
agent_cols = ['pv']
load_cols = ['l0', 'l1', 'l2', 'l3', 'l4']
cols = env_cols + agent_cols + load_cols

SLOTS_PER_DAY = setup.HOURS_PER_DAY * setup.MINUTES_PER_HOUR // setup.TIME_SLOT  # 96


def _day_profiles(rs: np.random.RandomState, days: np.ndarray, shape_prefix=()):
    """Vectorised synthetic day profiles for the given day numbers -> dict of arrays [..., D*96]."""
    D = len(days)
    T = D * SLOTS_PER_DAY
    slot = np.arange(T) % SLOTS_PER_DAY
    hour = slot / 4.0
    day = np.arange(T) // SLOTS_PER_DAY
    sp = tuple(shape_prefix)
    day_temp = 8.0 + 4.0 * np.sin(2 * np.pi * (np.asarray(days) - 5) / 30.0)
    temp = (day_temp[day] + 5.0 * np.sin(2 * np.pi * (hour - 9.0) / 24.0)
            + rs.normal(0.0, 1.0, sp + (T,)))
    cloud = 0.55 + 0.45 * rs.rand(*(sp + (D,)))
    pv = np.clip(np.sin(np.pi * (hour - 7.0) / 10.0), 0, None) * np.take(cloud, day, axis=-1)
    loads = []
    for k in range(5):
        m = (0.25 + 0.35 * np.exp(-((hour - (7.5 + 0.3 * k)) ** 2) / 2.0)
             + 0.6 * np.exp(-((hour - (19.0 + 0.25 * k)) ** 2) / 3.0) + 0.15 * rs.rand(*(sp + (T,))))
        loads.append(m)
    return dict(time=slot / float(SLOTS_PER_DAY), temperature=temp, pv=pv, loads=np.stack(loads, axis=-2))


start_day = min(min(testing_days), min(validation_days), min(training_days))
end_day = max(max(testing_days), max(validation_days), max(training_days))
start = datetime(2021, data_month, start_day)
end = datetime(2021, data_month, end_day) + timedelta(days=1)  # dataset.py:22-25


def compute_time_slot(time: str) -> float:
    """dataset.py:33-36"""
    t = datetime.strptime(time, '%H:%M:%S')
    return (t.minute / setup.TIME_SLOT) + t.hour * setup.MINUTES_PER_HOUR / setup.TIME_SLOT


def process_dataframe(df: pd.DataFrame) -> pd.DataFrame:
    """dataset.py:39-54: time slot / 96, loads and PV normalised by their maxima."""
    df = df.copy()
    df['time'] = df['time'].map(compute_time_slot) / 96.
    for c in load_cols:
        df[c] = df[c].astype(float) / df[c].max().astype(float)
    df['pv'] = df['pv'].astype(float) / df['pv'].max().astype(float)
    return df[cols]


def get_data(days: List[int], seed: int = 2021) -> Tuple[pd.DataFrame, List[pd.DataFrame]]:
    """dataset.get_data (dataset.py:61-80).  With a database ($P2PMG_DB, the reference's schema:
    database.create_tables) the profiles come from it exactly as in the reference; without one
    (the reference's DB is private) a synthetic generator with the same columns and
    normalisation stands in.  One frame per load column renamed to 'load' (dataset.py:78)."""
    from . import database as db
    con = db.get_connection()
    if con is not None:
        try:
            df = db.get_data(con, start, end)
        finally:
            con.close()
        df['day'] = df['date'].map(lambda d: int(re.match(r'.*-([0-9]+)$', d).groups()[0]))
        df = df[df['day'].map(lambda d: d in days)]
        df = process_dataframe(df)
        agent_dfs = [df[[l] + agent_cols].rename(columns={l: 'load'}) for l in load_cols]
        return df[env_cols], agent_dfs
    rs = np.random.RandomState(seed + 1000 * min(days))
    prof = _day_profiles(rs, np.asarray(days))
    df = pd.DataFrame({
        'day': np.repeat(days, SLOTS_PER_DAY),
        'time': prof['time'],
        'temperature': prof['temperature'],
        'pv': prof['pv'] / prof['pv'].max(),
    })
    for k, c in enumerate(load_cols):
        df[c] = prof['loads'][k] / prof['loads'][k].max()
    df = df[cols]
    agent_dfs = [df[[l] + agent_cols].rename(columns={l: 'load'}) for l in load_cols]
    return df[env_cols], agent_dfs


def get_train_data() -> Tuple[pd.DataFrame, List[pd.DataFrame]]:
    env_df, agent_dfs = get_data(training_days)
    env_df = env_df.drop(axis=1, labels='day')
    return env_df, agent_dfs


def get_validation_data() -> Tuple[pd.DataFrame, List[pd.DataFrame]]:
    return get_data(validation_days)


def get_test_data() -> Tuple[pd.DataFrame, List[pd.DataFrame]]:
    return get_data(testing_days)


@dataclass
class ProfileDataset:
    """(x_t, x_{t+1}) pairs of an f32 table, as tf.data.Dataset.from_tensor_slices((data,
    np.roll(data, -1))) in dataset.py:98-103."""
    data: np.ndarray
    rolled: np.ndarray

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(zip(self.data, self.rolled))

    @property
    def current(self) -> np.ndarray:
        return self.data


def dataframe_to_dataset(df, roll_len: int = -1, axis: int = 0) -> ProfileDataset:
    data = np.array(df, dtype=np.float32)
    return ProfileDataset(data, np.roll(data, roll_len, axis=axis))


# ----------------------------------------------------------------------------- batched scenarios
@dataclass
class ScenarioInputs:
    """Device inputs for S independent communities (SURVEY.md §8d synthetic inputs)."""
    time: np.ndarray      # [T] f32
    t_out: np.ndarray     # [S, T] f32 (per-scenario weather) or [1, T]
    load_w: np.ndarray    # [S, N, T] f32
    pv_w: np.ndarray      # [S, N, T] f32
    max_in: np.ndarray    # [S, N] f32
    t_in0: np.ndarray     # [S, N] f32
    t_m0: np.ndarray      # [S, N] f32
    load_ratings: np.ndarray
    pv_ratings: np.ndarray


_BLOCK = 256  # scenarios per generator block: a scenario's data depends only on (seed, s)


def _scenario_block(seed: int, block: int, N: int, T: int, homogeneous: bool):
    days = np.arange(T // SLOTS_PER_DAY + (T % SLOTS_PER_DAY > 0)) + training_days[0]
    rs = np.random.RandomState((seed * 1_000_003 + block * 7_919 + 17) % (2 ** 32))
    prof = _day_profiles(rs, days, shape_prefix=(_BLOCK,))
    # normalise over the whole generated days (dataset.py:46-50), then cut to the horizon
    pv = (prof['pv'] / prof['pv'].max(axis=-1, keepdims=True))[..., :T]
    loads = (prof['loads'] / prof['loads'].max(axis=-1, keepdims=True))[..., :T]
    t_out = prof['temperature'][..., :T].astype(np.float32)
    if homogeneous:
        lr = np.full((_BLOCK, N), 0.7)
        pr = np.full((_BLOCK, N), 4.0)
        t_in0 = np.full((_BLOCK, N), np.float32(21.0), np.float32)
        t_m0 = t_in0.copy()
    else:
        lr = rs.normal(0.7, 0.2, (_BLOCK, N))
        pr = rs.normal(4, 0.2, (_BLOCK, N))
        t_m0 = rs.normal(21.0, 0.3, (_BLOCK, N)).astype(np.float32)
        t_in0 = rs.normal(21.0, 0.3, (_BLOCK, N)).astype(np.float32)
    cols_idx = np.arange(N) % 5
    load_w = ((loads[:, cols_idx, :] * lr[..., None]) * 1e3).astype(np.float32)
    pv_w = ((pv[:, None, :] * pr[..., None]) * 1e3).astype(np.float32)
    max_in = (np.maximum(lr, pr) * 1.1 * 1e3).astype(np.float32)
    return dict(t_out=t_out, load_w=load_w, pv_w=pv_w, max_in=max_in, t_in0=t_in0, t_m0=t_m0,
                load_ratings=lr, pv_ratings=pr)


def scenario_batch(S: int, N: int, T: int = SLOTS_PER_DAY, seed: int = setup.seed, homogeneous: bool = False,
                   shared_weather: bool = False, first_scenario: int = 0) -> ScenarioInputs:
    """Scenarios [first_scenario, first_scenario + S) of N agents, built as get_community does
    (community.py:198-234): ratings ~ N(0.7, 0.2) kW / N(4, 0.2) kW, max_in = max(load_kW,
    pv_kW) * 1.1e3, W profiles = f32((norm * rating) * 1e3), T0 ~ N(21, 0.3) (heterogeneous).
    Agent i uses load column l_{i mod 5} (the reference has 5, dataset.py:30).
    Scenario s's data depends only on (seed, s), so any shard of a multi-GPU run is generated
    alone and matches the single-GPU batch."""
    b0, b1 = first_scenario // _BLOCK, (first_scenario + S - 1) // _BLOCK
    parts = [_scenario_block(seed, b, N, T, homogeneous) for b in range(b0, b1 + 1)]
    cat = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    lo = first_scenario - b0 * _BLOCK
    sl = {k: np.ascontiguousarray(v[lo:lo + S]) for k, v in cat.items()}
    time = (np.arange(T) % SLOTS_PER_DAY / float(SLOTS_PER_DAY)).astype(np.float32)
    t_out = sl['t_out'][:1] if shared_weather else sl['t_out']
    return ScenarioInputs(time=time, t_out=t_out, load_w=sl['load_w'], pv_w=sl['pv_w'], max_in=sl['max_in'],
                          t_in0=sl['t_in0'], t_m0=sl['t_m0'], load_ratings=sl['load_ratings'],
                          pv_ratings=sl['pv_ratings'])


# ----------------------------------------------------------------------------- heterogeneous mixes
@dataclass
class AssetMix:
    """Per-agent asset mix of a heterogeneous community (BASELINE.json configs[3]).

    The reference builds every household as PV + 3 kW heat pump + NoStorage (community.py:219-228);
    the mixes are the build's extension along the reference's own asset classes: ``Consumer`` (no PV,
    production.py:44-58), a heat pump of another size (``HeatPump(cop, max_power, power)``,
    heating.py:158-163) or none, and ``BatteryStorage`` (storage.py:36-76) or ``NoStorage``."""
    has_pv: np.ndarray            # [S, N] bool
    hp_levels: np.ndarray         # [S, N, 3] f32 heat-pump power per action (0 = no heat pump)
    battery_capacity: np.ndarray  # [S, N] f64 J (0 = NoStorage)


def _unit_hash(seed: int, scen: np.ndarray, agent: np.ndarray, stream: int) -> np.ndarray:
    """Uniform [0, 1) from splitmix64 of (seed, global scenario, agent, stream): a scenario's mix
    depends only on its global index, so every shard of a multi-GPU run draws it alone."""
    with np.errstate(over='ignore'):
        x = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + scen.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)
             + agent.astype(np.uint64) * np.uint64(0x94D049BB133111EB) + np.uint64(stream) * np.uint64(0x2545F4914F6CDD1D))
        for m, s in ((0xBF58476D1CE4E5B9, 30), (0x94D049BB133111EB, 27)):
            x = (x ^ (x >> np.uint64(s))) * np.uint64(m)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) / float(1 << 53)


def asset_mix(S: int, N: int, first_scenario: int = 0, seed: int = setup.seed, p_no_pv: float = 0.2,
              p_no_hp: float = 0.25, p_big_hp: float = 0.3, p_no_battery: float = 0.4,
              battery_j: float = 10.0 * 3.6e6) -> AssetMix:
    """PV-only / heat-pump / battery mixes for scenarios [first_scenario, first_scenario + S)."""
    scen = np.arange(first_scenario, first_scenario + S)[:, None] + np.zeros((1, N), np.int64)
    agent = np.zeros((S, 1), np.int64) + np.arange(N)[None, :]
    has_pv = _unit_hash(seed, scen, agent, 1) >= p_no_pv
    lv = np.broadcast_to(np.array([0.0, 1500.0, 3000.0], np.float32), (S, N, 3)).copy()
    lv[_unit_hash(seed, scen, agent, 3) < p_big_hp] = np.array([0.0, 2500.0, 5000.0], np.float32)
    lv[_unit_hash(seed, scen, agent, 2) < p_no_hp] = 0.0
    cap = np.where(_unit_hash(seed, scen, agent, 4) < p_no_battery, 0.0, battery_j)
    return AssetMix(has_pv=has_pv, hp_levels=lv, battery_capacity=cap)


def apply_asset_mix(inp: ScenarioInputs, mix: AssetMix) -> ScenarioInputs:
    """Consumers get a zero PV profile and max_in = load_kW * 1.1e3 (community.py:220's formula
    with no PV rating)."""
    pv_w = np.where(mix.has_pv[..., None], inp.pv_w, np.float32(0.0)).astype(np.float32)
    max_in = np.where(mix.has_pv, inp.max_in,
                      (np.asarray(inp.load_ratings) * 1.1 * 1e3).astype(np.float32)).astype(np.float32)
    return ScenarioInputs(time=inp.time, t_out=inp.t_out, load_w=inp.load_w, pv_w=pv_w, max_in=max_in,
                          t_in0=inp.t_in0, t_m0=inp.t_m0, load_ratings=inp.load_ratings,
                          pv_ratings=np.where(mix.has_pv, inp.pv_ratings, 0.0))


# ----------------------------------------------------------------------------- parallel generation
def _shared_block_job(job):
    """One generator block of scenario_batch_shared (a spawned worker): generate it, write its part
    of [first, first + S) into the shared load / pv / t_out arrays, return the small per-agent ones."""
    from multiprocessing import shared_memory
    seed, b, N, T, homogeneous, first, S, names, has_pv = job
    d = _scenario_block(seed, b, N, T, homogeneous)
    lo, hi = max(first, b * _BLOCK), min(first + S, (b + 1) * _BLOCK)
    src, dst = slice(lo - b * _BLOCK, hi - b * _BLOCK), slice(lo - first, hi - first)
    shms = [shared_memory.SharedMemory(name=n) for n in names]
    try:
        load = np.ndarray((S, N, T), np.float32, buffer=shms[0].buf)
        pv = np.ndarray((S, N, T), np.float32, buffer=shms[1].buf)
        t_out = np.ndarray((S, T), np.float32, buffer=shms[2].buf)
        load[dst] = d['load_w'][src]
        pv[dst] = d['pv_w'][src] if has_pv is None else np.where(has_pv[..., None], d['pv_w'][src], np.float32(0.0))
        t_out[dst] = d['t_out'][src]
        del load, pv, t_out  # no view may outlive the mapping
    finally:
        for s in shms:
            s.close()
    return dst.start, {k: d[k][src] for k in ('max_in', 't_in0', 't_m0', 'load_ratings', 'pv_ratings')}


class SharedScenarioInputs:
    """scenario_batch (+ apply_asset_mix when ``mix`` is given) generated by ``workers`` spawned
    processes, one generator block each, straight into shared memory: the same arrays bit for bit
    (every block depends only on (seed, block)), for horizons where one process would take minutes
    (configs[3]: 8192 scenarios x 4 agents x 35,040 slots = 9.2 GB of profiles, ~3 s per 256-scenario
    block).  Use as a context manager; ``.inputs`` is valid until exit, which unlinks the memory."""

    def __init__(self, S: int, N: int, T: int, workers: int, seed: int = setup.seed, first_scenario: int = 0,
                 mix: Optional["AssetMix"] = None, homogeneous: bool = False):
        import concurrent.futures as cf
        import multiprocessing as mp
        from multiprocessing import shared_memory
        sizes = (S * N * T * 4, S * N * T * 4, S * T * 4)
        self._shm = [shared_memory.SharedMemory(create=True, size=max(1, n)) for n in sizes]
        try:
            names = [s.name for s in self._shm]
            b0, b1 = first_scenario // _BLOCK, (first_scenario + S - 1) // _BLOCK
            jobs = []
            for b in range(b0, b1 + 1):
                lo, hi = max(first_scenario, b * _BLOCK), min(first_scenario + S, (b + 1) * _BLOCK)
                hp = None if mix is None else mix.has_pv[lo - first_scenario:hi - first_scenario]
                jobs.append((seed, b, N, T, homogeneous, first_scenario, S, names, hp))
            small = {k: np.zeros((S, N), dt) for k, dt in (('max_in', np.float32), ('t_in0', np.float32),
                                                          ('t_m0', np.float32), ('load_ratings', np.float64),
                                                          ('pv_ratings', np.float64))}
            with cf.ProcessPoolExecutor(max(1, min(workers, len(jobs))), mp_context=mp.get_context("spawn")) as ex:
                for start, part in ex.map(_shared_block_job, jobs):
                    for k, v in part.items():
                        small[k][start:start + len(v)] = v
        except BaseException:
            self.close()
            raise
        load = np.ndarray((S, N, T), np.float32, buffer=self._shm[0].buf)
        pv = np.ndarray((S, N, T), np.float32, buffer=self._shm[1].buf)
        t_out = np.ndarray((S, T), np.float32, buffer=self._shm[2].buf)
        max_in, pr = small['max_in'], small['pv_ratings']
        if mix is not None:  # apply_asset_mix's per-agent part (the PV zeroing ran in the workers)
            max_in = np.where(mix.has_pv, max_in, (small['load_ratings'] * 1.1 * 1e3).astype(np.float32)).astype(np.float32)
            pr = np.where(mix.has_pv, pr, 0.0)
        time = (np.arange(T) % SLOTS_PER_DAY / float(SLOTS_PER_DAY)).astype(np.float32)
        self.inputs = ScenarioInputs(time=time, t_out=t_out, load_w=load, pv_w=pv, max_in=max_in, t_in0=small['t_in0'],
                                     t_m0=small['t_m0'], load_ratings=small['load_ratings'], pv_ratings=pr)

    def close(self):
        self.inputs = None
        for s in getattr(self, "_shm", []):
            try:
                s.unlink()  # the name goes now; the memory when the last mapping closes
            except FileNotFoundError:
                pass
            try:
                s.close()
            except BufferError:  # a caller still holds a view: the mapping lives until it is dropped
                pass
        self._shm = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
