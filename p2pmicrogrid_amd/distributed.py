"""Scenario sharding over GPUs (one process per GPU).

Scenarios are independent communities, so S_total scenarios are split into contiguous shards,
one per rank, with no per-step exchange.  With per-agent Q-tables (the reference's semantics)
every rank's tables are private: this is "replicas only" — the only collective is an
end-of-episode reduction of the episode metrics (a few bytes, over torch.distributed).
Philox counters use global agent ids and scenario data depend only on (seed, scenario), so
any world size reproduces the single-GPU results scenario for scenario.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np


@dataclass
class Shard:
    rank: int
    world: int
    first: int
    count: int


def shard(n_total: int, rank: int, world: int) -> Shard:
    """Contiguous split, the first (n_total % world) ranks get one extra scenario."""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return Shard(rank, world, first, base + (1 if rank < extra else 0))


def init_from_env(backend: str = "gloo"):
    """(rank, world, local_rank) from torchrun's environment; initialises torch.distributed
    when world > 1 (gloo by default: metrics only, no device memory involved)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


def all_reduce_sum(values: np.ndarray, world: int) -> np.ndarray:
    if world == 1:
        return np.asarray(values, dtype=np.float64)
    import torch
    import torch.distributed as dist
    t = torch.as_tensor(np.asarray(values, dtype=np.float64))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.numpy()


def all_gather_concat(values: np.ndarray, world: int) -> np.ndarray:
    """Concatenate per-rank 1-D arrays in rank order (ragged allowed)."""
    if world == 1:
        return np.asarray(values)
    import torch.distributed as dist
    out: List = [None] * world
    dist.all_gather_object(out, np.asarray(values))
    return np.concatenate(out)


class ShardedTrainer:
    """Tabular training of S_total scenarios sharded over the ranks.

    engine_factory(shard, S, N, R, T, q_dtype, device, seed) -> an object with the
    DeviceCommunityBatch interface; the default is the HIP engine."""

    def __init__(self, n_scenarios: int, n_agents: int = 2, rounds: int = 1, horizon: int = 96,
                 q_dtype: str = "f64", seed: int = 42, rank: int = 0, world: int = 1, device: int = 0,
                 engine_factory: Optional[Callable] = None):
        from .dataset import scenario_batch
        self.sh = shard(n_scenarios, rank, world)
        self.S_total, self.N, self.R, self.T = n_scenarios, n_agents, rounds, horizon
        self.world = world
        inp = scenario_batch(self.sh.count, n_agents, horizon, seed=seed, first_scenario=self.sh.first)
        if engine_factory is None:
            from .engine import DeviceCommunityBatch

            def engine_factory(sh, S, N, R, T, q_dtype, device, seed):
                return DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype, device=device, seed=seed,
                                            scenario_offset=sh.first)
        self.eng = engine_factory(self.sh, self.sh.count, n_agents, rounds, horizon, q_dtype, device, seed)
        self.eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        self.eng.set_profiles(inp.load_w, inp.pv_w)
        self.eng.set_max_in(inp.max_in)
        self.eng.set_temperatures(inp.t_in0, inp.t_m0)
        self.episode = 0

    def train_episode(self, epsilon: float, reset_sigma: float = 0.3) -> float:
        """One training episode on every shard; returns the global mean over scenarios of the
        episode reward (sum_t mean_i r, community.py:179)."""
        self.eng.run_episode("train", "philox", episode=self.episode, epsilon=epsilon)
        local = self.eng.episode_reward().astype(np.float64)
        self.eng.reset_temperatures_philox(self.episode + 1, reset_sigma)
        self.episode += 1
        tot = all_reduce_sum(np.array([local.sum(), local.size]), self.world)
        return float(tot[0] / tot[1])

    def episode_rewards_global(self) -> np.ndarray:
        return all_gather_concat(self.eng.episode_reward(), self.world)
