"""Test-only stand-in with the DeviceCommunityBatch interface, computed by the oracle, so the
multi-process orchestration (sharding, collectives) can be exercised on CPU with gloo."""
import numpy as np

from oracle import philox
from oracle.restatement import OracleBatch


class OracleEngine:
    def __init__(self, sh, S, N, R, T, q_dtype, device, seed, shared_q=False):
        self.S, self.N, self.R, self.T, self.seed = S, N, R, T, seed
        self.shared_q = shared_q
        self._battery = None
        self.gids = (np.arange(sh.first, sh.first + S)[:, None] * N + np.arange(N)[None, :])
        self.q_dtype = q_dtype
        self._env = self._prof = self._mi = None
        self.ob = None
        self.last = None

    def set_env(self, time, t_out, *prices):
        self._env = (np.asarray(time, np.float32)[:1], np.asarray(t_out, np.float32))

    def set_profiles(self, load, pv):
        self._prof = (np.asarray(load, np.float32), np.asarray(pv, np.float32))

    def set_max_in(self, mi):
        self._mi = np.asarray(mi, np.float32)

    def _ensure(self):
        if self.ob is None:
            self.ob = OracleBatch(S=self.S, N=self.N, R=self.R, load_w=self._prof[0], pv_w=self._prof[1],
                                  max_in=self._mi, env_time=self._env[0], env_tout=self._env[1],
                                  q_dtype=self.q_dtype, shared_q=self.shared_q)
        return self.ob

    def set_temperatures(self, t_in, t_m):
        ob = self._ensure()
        ob.t_in = np.asarray(t_in, np.float32).reshape(self.S, self.N).copy()
        ob.t_m = np.asarray(t_m, np.float32).reshape(self.S, self.N).copy()

    def reset_temperatures_philox(self, episode, sigma=0.3):
        a, b = philox.t0_draws(self.seed, episode, self.gids.ravel(), sigma=sigma)
        self.set_temperatures(a, b)

    def run_episode(self, mode="train", rng="philox", episode=0, epsilon=0.81, record=(), philox="auto",
                    next_epsilon=None):  # next_epsilon: a device pre-pass hint, no effect on results
        self.last = self._ensure().run_episode(mode, rng="philox", seed=self.seed, episode=episode, eps=epsilon,
                                               agent_ids=self.gids)

    def episode_reward(self):
        return self.last["episode_reward"]

    def run_episodes(self, episode, epsilons, reset_sigma=None, next_epsilons=None, record=()):
        """p2pmg_run_episodes: the same episodes one by one (the device chains them in one launch)."""
        self._chain = []
        for k, eps in enumerate(epsilons):
            self.run_episode("train", "philox", episode=episode + k, epsilon=eps, record=record)
            if reset_sigma is not None:
                self.reset_temperatures_philox(episode + k + 1, reset_sigma)
            self._chain.append(self.episode_reward())

    def episode_rewards(self):
        return np.stack(self._chain)

    def set_hp_levels(self, levels):
        ob = self._ensure()
        ob.hp_levels = np.asarray(levels, np.float32).reshape(self.S, self.N, 3).copy()

    def set_battery(self, capacity, min_soc=0.1, max_soc=0.9, efficiency=0.9, soc0=0.5):
        ob = self._ensure()
        ob.battery_capacity = np.broadcast_to(np.asarray(capacity, np.float64), (self.S, self.N)).copy()
        ob.battery_bounds = (min_soc, max_soc, efficiency)
        ob.soc = np.full((self.S, self.N), float(soc0))

    def get_soc(self):
        return self.ob.soc.copy()

    def get_q_delta(self):
        return self.ob.q_delta.copy()

    def set_q_delta(self, d):
        self.ob.q_delta[:] = np.asarray(d, np.int64).reshape(self.ob.q_delta.shape)

    def apply_q_delta(self):
        self.ob.apply_q_delta()

    def get_q(self, first=0, count=None):
        q = self.ob.q
        return q[first:first + (len(q) - first if count is None else count)].copy()


class OracleDQNEngine(OracleEngine):
    """DeviceDQNBatch's interface (one shared network) computed by oracle/dqn.py, with the same
    gradient layout (grad_segments, agents_per_block) and host exchange hook."""

    def __init__(self, sh, S, N, R, T, q_dtype, device, seed, shared_q=True, learner="dqn", grad_segments=1,
                 agents_per_block=0):
        super().__init__(sh, S, N, R, T, q_dtype, device, seed, shared_q=True)
        self.grad_segments, self.agents_per_block = grad_segments, agents_per_block
        self._xchg = (None, 0, 1)

    def _ensure(self):
        if self.ob is None:
            from oracle import dqn as odqn
            gather, rank, world = self._xchg
            self.ob = odqn.OracleDQNBatch(S=self.S, N=self.N, R=self.R, load_w=self._prof[0], pv_w=self._prof[1],
                                          max_in=self._mi, env_time=self._env[0], env_tout=self._env[1],
                                          theta0=odqn.glorot_init(1, 0), shared=True,
                                          agents_per_block=self.agents_per_block, grad_segments=self.grad_segments,
                                          rank=rank, world=world, exchange=gather)
        return self.ob

    def set_grad_exchange(self, gather, rank, world):
        self._xchg = (gather, rank, world)
        if self.ob is not None:
            self.ob.exchange, self.ob.rank, self.ob.world = gather, rank, world

    def run_episode(self, mode="train", rng="philox", episode=0, epsilon=1.0, record=(), philox="auto"):
        self.last = self._ensure().run_episode(mode, rng="philox", seed=self.seed, episode=episode, eps=epsilon,
                                               agent_ids=self.gids)

    def get_weights(self, which="online", first=0, count=None):
        arr = {"online": self.ob.theta, "target": self.ob.target, "adam_m": self.ob.m, "adam_v": self.ob.v}[which]
        return arr.copy()
