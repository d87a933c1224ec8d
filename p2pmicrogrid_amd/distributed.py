"""Scenario sharding over GPUs (one process per GPU).

Scenarios are independent communities, so S_total scenarios are split into contiguous shards,
one per rank, with no per-step exchange.  With per-agent Q-tables (the reference's semantics)
every rank's tables are private: this is "replicas only" — the only collective is an
end-of-episode reduction of the episode metrics (a few bytes, over torch.distributed).
Philox counters use global agent ids and scenario data depend only on (seed, scenario), so
any world size reproduces the single-GPU results scenario for scenario.

With ONE shared policy table (config 3, ``shared_q=True``) there is a real exchange step: every
rank accumulates its scenarios' TD deltas in int64 fixed point, the deltas are summed over the
ranks once per episode (RCCL all-reduce on the device stream, or a host-side sum over the
process group), and each rank applies the identical sum.  Integer addition is associative, so
the table after each episode is bit-identical for every world size.

With ONE shared DQN network (config 5, ``learner="dqn"``) the exchange is per env step: every
rank sums its agents' gradients into fixed gradient segments (contiguous runs of whole scenarios,
each folded in a fixed block order), the segments of all ranks are gathered (RCCL all-gather on the
device stream, or a host all-gather over the process group) and every rank adds them in global
segment order before the same Adam step.  With the total segment count and the agents per block
fixed, 1 rank x G segments and W ranks x G/W segments give the same weights bit for bit.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np


DQN_TRAIN_SLOTS = 512  # dqn_train_kernel workgroups resident at once on MI355X: 256 CUs x 2


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


def all_reduce_int64(values: np.ndarray, world: int) -> np.ndarray:
    """Exact int64 sum over ranks (host fallback of the shared-table delta exchange)."""
    if world == 1:
        return np.asarray(values, dtype=np.int64)
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(values, dtype=np.int64))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.numpy()


def all_gather_rows(rows: np.ndarray, rank: int, world: int) -> None:
    """In-place all-gather of a [world, n] float32 array whose row `rank` is filled in (the host
    exchange of the DQN gradient segments), over the torch process group."""
    if world == 1:
        return
    import torch
    import torch.distributed as dist
    mine = torch.from_numpy(np.ascontiguousarray(rows[rank]))
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine)
    for r in range(world):
        if r != rank:
            rows[r] = out[r].numpy()


def broadcast_bytes(data: Optional[bytes], world: int, src: int = 0) -> bytes:
    if world == 1:
        return data
    import torch.distributed as dist
    box = [data]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def all_gather_concat(values: np.ndarray, world: int) -> np.ndarray:
    """Concatenate per-rank 1-D arrays in rank order (ragged allowed)."""
    if world == 1:
        return np.asarray(values)
    import torch.distributed as dist
    out: List = [None] * world
    dist.all_gather_object(out, np.asarray(values))
    return np.concatenate(out)


class ShardedTrainer:
    """Training of S_total scenarios sharded over the ranks: tabular Q-learning (the reference's
    QAgent) or, with learner="dqn", DQN agents sharing ONE Q-network (config 5).

    engine_factory(shard, S, N, R, T, q_dtype, device, seed, shared_q, **dqn) -> an object with the
    DeviceCommunityBatch (DeviceDQNBatch) interface; the default is the HIP engine.

    shared_q: one policy table for every agent of every scenario on every rank (config 3).
    exchange: how the shared-table deltas and the episode metrics are summed over ranks — "rccl"
    (device all-reduce over xGMI through the context's RCCL communicator, the production path),
    "host" (copy out, sum over the torch process group, copy back) or "auto" (rccl when the
    process group is nccl/RCCL, host otherwise).
    battery: kwargs for ``set_battery`` (scalars), enabling the storage rule.
    learner="dqn": grad_segments = the TOTAL gradient segment count (default: one per rank; must be
    a multiple of world and divide n_scenarios) and agents_per_block (default 0: ceil(agents of all
    ranks / (512 x grad_segments)), a function of global sizes only) fix the gradient's summation
    structure, so a run with the same grad_segments is bit-identical for every world size that
    divides it; the gradient exchange ("rccl" | "host") runs once per env step."""

    def __init__(self, n_scenarios: int, n_agents: int = 2, rounds: int = 1, horizon: int = 96,
                 q_dtype: str = "f64", seed: int = 42, rank: int = 0, world: int = 1, device: int = 0,
                 engine_factory: Optional[Callable] = None, shared_q: bool = False, exchange: str = "auto",
                 battery: Optional[dict] = None, homogeneous: bool = False, learner: str = "tabular",
                 grad_segments: Optional[int] = None, agents_per_block: int = 0):
        from .dataset import scenario_batch
        if learner not in ("tabular", "dqn"):
            raise ValueError(f"learner must be 'tabular' or 'dqn', got {learner!r}")
        self.learner = learner
        dqn_kw = {}
        if learner == "dqn":
            G = world if grad_segments is None else int(grad_segments)
            if G < 1 or G % world or n_scenarios % G:
                raise ValueError(f"grad_segments={G} must be a multiple of world={world} and divide "
                                 f"n_scenarios={n_scenarios}")
            self.grad_segments = G
            if agents_per_block <= 0:
                # rank-independent default: the block size must not follow the shard size (the device's
                # own default, ceil(A_local / train slots), would change the summation order, and so the
                # bits, with the world size).  ceil(A_total / (512 G)) gives every rank >= 512 train
                # workgroups (2 per CU on 256 CUs) whatever the world, and depends on global sizes only.
                agents_per_block = max(1, -(-(n_scenarios * n_agents) // (DQN_TRAIN_SLOTS * G)))
            self.agents_per_block = int(agents_per_block)
            dqn_kw = dict(learner="dqn", grad_segments=G // world, agents_per_block=self.agents_per_block)
            shared_q = True
            self.filled = False
        self.sh = shard(n_scenarios, rank, world)
        self.S_total, self.N, self.R, self.T = n_scenarios, n_agents, rounds, horizon
        self.rank, self.world, self.shared_q = rank, world, bool(shared_q)
        inp = scenario_batch(self.sh.count, n_agents, horizon, seed=seed, first_scenario=self.sh.first,
                             homogeneous=homogeneous)
        if engine_factory is None:
            def engine_factory(sh, S, N, R, T, q_dtype, device, seed, shared_q=False, learner="tabular",
                               grad_segments=1, agents_per_block=0):
                if learner == "dqn":
                    from .dqn import DeviceDQNBatch
                    return DeviceDQNBatch(S, N, R, T, shared=True, device=device, seed=seed, scenario_offset=sh.first,
                                          grad_segments=grad_segments, agents_per_block=agents_per_block, init_seed=0)
                from .engine import DeviceCommunityBatch
                return DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype, device=device, seed=seed,
                                            scenario_offset=sh.first, shared_q=shared_q)
        self.shared_q = bool(shared_q)
        self.eng = engine_factory(self.sh, self.sh.count, n_agents, rounds, horizon, q_dtype, device, seed,
                                  shared_q=self.shared_q, **dqn_kw)
        self.eng.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        self.eng.set_profiles(inp.load_w, inp.pv_w)
        self.eng.set_max_in(inp.max_in)
        self.eng.set_temperatures(inp.t_in0, inp.t_m0)
        if battery is not None:
            self.eng.set_battery(**battery)
        self.exchange = None
        if world > 1:
            if exchange == "auto":
                import torch.distributed as dist
                exchange = "rccl" if dist.is_initialized() and dist.get_backend() == "nccl" else "host"
            if exchange not in ("rccl", "host"):
                raise ValueError(f"exchange must be 'rccl', 'host' or 'auto', got {exchange!r}")
            if exchange == "rccl":
                from .engine import comm_unique_id
                uid = broadcast_bytes(comm_unique_id() if rank == 0 else None, world)
                self.eng.comm_init(uid, rank, world)
            elif learner == "dqn":  # the per-env-step gradient gather, over the process group
                self.eng.set_grad_exchange(lambda rows: all_gather_rows(rows, rank, world), rank, world)
            self.exchange = exchange
        self.episode = 0

    def exchange_q_delta(self):
        """Sum the shared-table deltas over the ranks and apply them (once per episode)."""
        if self.exchange == "rccl":
            self.eng.allreduce_q_delta()
        elif self.exchange == "host":
            self.eng.set_q_delta(all_reduce_int64(self.eng.get_q_delta(), self.world))
        self.eng.apply_q_delta()

    def fill_buffers(self, episodes: int = 1, reset_sigma: float = 0.3):
        """DQN: CommunityMicrogrid.init_buffers (community.py:125-147): episodes of acting at
        epsilon 1 that only store transitions (>= 31 per agent before training can start)."""
        for _ in range(episodes):
            self.eng.run_episode("fill", "philox", episode=self.episode, epsilon=1.0)
            self.eng.reset_temperatures_philox(self.episode + 1, reset_sigma)
            self.episode += 1
        self.filled = True

    def _metrics(self):
        if self.exchange == "rccl":  # episode metrics over RCCL, reduced on the device
            return self.eng.allreduce_metrics()
        local = self.eng.episode_reward().astype(np.float64)
        return all_reduce_sum(np.array([local.sum(), local.size]), self.world)

    def train_episode(self, epsilon: float, reset_sigma: float = 0.3,
                      next_epsilon: Optional[float] = None) -> float:
        """One training episode on every shard; returns the global mean over scenarios of the
        episode reward (sum_t mean_i r, community.py:179).  next_epsilon: the next episode's
        epsilon (the decay schedule, community.py:279-286), for the speculative pre-pass.
        DQN: the replay memory is filled first if it was not (fill_buffers); every env step's
        gradient exchange happens inside the episode call."""
        if self.learner == "dqn":
            if not self.filled:
                self.fill_buffers()
            self.eng.run_episode("train", "philox", episode=self.episode, epsilon=epsilon)
            total, count = self._metrics()
            self.eng.reset_temperatures_philox(self.episode + 1, reset_sigma)
            self.episode += 1
            return float(total / count)
        self.eng.run_episode("train", "philox", episode=self.episode, epsilon=epsilon,
                             next_epsilon=next_epsilon)
        if self.shared_q:
            self.exchange_q_delta()
        total, count = self._metrics()
        self.eng.reset_temperatures_philox(self.episode + 1, reset_sigma)
        self.episode += 1
        return float(total / count)

    def train_episodes(self, epsilons, reset_sigma: float = 0.3, next_epsilons=None) -> np.ndarray:
        """len(epsilons) training episodes on every shard (community.py:279-286's loop body, each
        ending with agent.reset()); returns the global mean episode reward of each.  Per-agent
        tables run as chained launches (p2pmg_run_episodes: the episodes back to back in every
        wave, results identical to train_episode per episode); a shared table or DQN network needs
        its exchange between episodes and runs train_episode per episode."""
        eps = [float(e) for e in epsilons]
        if self.learner == "dqn" or self.shared_q:
            out = [self.train_episode(e, reset_sigma, eps[k + 1] if k + 1 < len(eps) else None)
                   for k, e in enumerate(eps)]
            return np.array(out)
        self.eng.run_episodes(self.episode, eps, reset_sigma=reset_sigma, next_epsilons=next_epsilons)
        local = self.eng.episode_rewards().astype(np.float64)  # [n, S]
        tot = all_reduce_sum(np.concatenate([local.sum(axis=1), [local.shape[1]]]), self.world)
        self.episode += len(eps)
        return tot[:-1] / tot[-1]

    def episode_rewards_global(self) -> np.ndarray:
        return all_gather_concat(self.eng.episode_reward(), self.world)
