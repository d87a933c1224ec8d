"""Test-only engine for ``bench.py`` on CPU (P2PMG_BENCH_TEST_ENGINE=bench_test_engine:BenchOracleEngine):
the oracle-backed OracleEngine behind the DeviceCommunityBatch constructor and the bench's timing /
communicator calls, so the launcher, sharding and gloo collectives run end to end without a GPU."""
import numpy as np

from oracle_engine import OracleEngine
from p2pmicrogrid_amd.distributed import Shard


class BenchOracleEngine(OracleEngine):
    def __init__(self, S, N, R, T, q_dtype="f64", device=0, scenario_offset=0, shared_q=False, seed=42):
        import os
        fail = os.environ.get("P2PMG_BENCH_TEST_FAIL_RANK")
        if fail is not None and fail == os.environ.get("RANK"):
            raise RuntimeError("test: this rank fails at engine construction")
        super().__init__(Shard(0, 1, scenario_offset, S), S, N, R, T, q_dtype, device, seed, shared_q=shared_q)
        noise = int(os.environ.get("P2PMG_BENCH_TEST_NOISE", "0"))  # a chatty rank (launcher pipe test)
        for _ in range(noise // 1000):
            print("x" * 999, flush=False)
        self.device = device
        self._times = []

    def run_episode(self, mode="train", rng="philox", episode=0, epsilon=0.81, record=(), philox="auto",
                    next_epsilon=None, reset_sigma=None):
        super().run_episode(mode, rng, episode=episode, epsilon=epsilon, record=record)
        if reset_sigma is not None:
            self.reset_temperatures_philox(episode + 1, reset_sigma)
        self._times.append(float("nan"))

    def comm_init(self, uid, rank, world):
        raise RuntimeError("no RCCL in the CPU test engine")

    def sync(self):
        pass

    def set_timing_period(self, p):
        pass

    def reset_kernel_times(self):
        self._times = []

    def kernel_times(self):
        return np.array([], np.float64)

    def last_kernel(self):
        return "oracle (CPU test engine)"

    def close(self):
        pass

    def allreduce_metrics(self):  # world 1 only (comm_init refuses a communicator)
        r = self.episode_reward().astype(np.float64)
        return float(r.sum()), int(r.size)

    def comm_nranks(self):
        return 1

    def table_hash_allgather(self):
        import hashlib
        h = hashlib.blake2b(np.ascontiguousarray(self.ob.q).tobytes(), digest_size=8).digest()
        return np.array([int.from_bytes(h, "little")], np.uint64)


class BenchOracleDQNEngine:
    """The DeviceDQNBatch calls run_dqn makes, on oracle/dqn.py (one shared network)."""

    def __init__(self, S, N, R, T, shared=True, device=0, scenario_offset=0, init_seed=0, seed=42, grad_segments=1,
                 agents_per_block=0):
        import os
        fail = os.environ.get("P2PMG_BENCH_TEST_FAIL_DQN_RANK")  # a setup failure on one rank (bench.agree_setup)
        if fail is not None and os.environ.get("RANK", "0") == fail:
            raise MemoryError("test: DQN context setup failed on this rank")
        from oracle_engine import OracleDQNEngine
        self._e = OracleDQNEngine(Shard(0, 1, scenario_offset, S), S, N, R, T, "f32", device, seed,
                                  grad_segments=grad_segments, agents_per_block=agents_per_block)
        self.S, self.N, self.R, self.T = S, N, R, T

    def __getattr__(self, name):  # set_env, set_profiles, ..., run_episode, episode_reward, get_weights
        return getattr(self._e, name)

    def comm_init(self, uid, rank, world):
        raise RuntimeError("no RCCL in the CPU test engine")

    def sync(self):
        pass

    def reset_kernel_times(self):
        pass

    def kernel_times(self):
        return np.array([], np.float64)

    def close(self):
        pass

    def allreduce_metrics(self):
        r = self.episode_reward().astype(np.float64)
        return float(r.sum()), int(r.size)

    def comm_nranks(self):
        return 1

    def grad_layout(self):
        return {"segments": self._e.grad_segments, "agents_per_block": self._e.agents_per_block, "blocks": None}
