"""world_size-2 gloo runs of the sharded trainer on CPU (oracle-backed stand-in engine):
sharding + metric collectives reproduce the single-process result scenario for scenario."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from p2pmicrogrid_amd.distributed import ShardedTrainer, shard

S_TOTAL, N, R, T, EPISODES = 9, 2, 1, 24, 3
PRIMARY_ONLY = ("--schedule-episodes", "0", "--secondary", "none", "--extra", "")  # bench.py: configs[1] line only


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, kw):
    import torch.distributed as dist
    from oracle_engine import OracleEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    chain = kw.pop("_chain", False)
    tr = ShardedTrainer(S_TOTAL, N, R, T, rank=rank, world=world, engine_factory=OracleEngine, **kw)
    if chain:  # train_episodes: chained launches on the device, one per call
        means = list(tr.train_episodes([0.81 * 0.9 ** e for e in range(EPISODES)]))
    else:
        means = [tr.train_episode(0.81 * 0.9 ** e) for e in range(EPISODES)]
    per_scen = tr.episode_rewards_global()
    if rank == 0:
        q.put((means, per_scen, tr.eng.get_q(0, 1) if kw.get("shared_q") else None))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(kw, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kw)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _run_two_ranks(kw):
    return _run_ranks(kw, 2)


def test_shard_split():
    parts = [shard(10, r, 4) for r in range(4)]
    assert [p.count for p in parts] == [3, 3, 2, 2] and [p.first for p in parts] == [0, 3, 6, 8]
    assert sum(shard(4096, r, 8).count for r in range(8)) == 4096


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_process():
    from oracle_engine import OracleEngine
    single = ShardedTrainer(S_TOTAL, N, R, T, engine_factory=OracleEngine)
    means1 = [single.train_episode(0.81 * 0.9 ** e) for e in range(EPISODES)]
    per1 = single.episode_rewards_global()
    means2, per2, _ = _run_two_ranks({})
    assert np.array_equal(per1, per2)
    assert np.allclose(means1, means2, rtol=0, atol=1e-9)


@pytest.mark.timeout(300)
def test_two_rank_train_episodes_match_single_process_episode_loop():
    """ShardedTrainer.train_episodes (chained launches per rank) over gloo at world 2 equals the
    single-process train_episode loop: per-scenario rewards and the global means."""
    from oracle_engine import OracleEngine
    single = ShardedTrainer(S_TOTAL, N, R, T, engine_factory=OracleEngine)
    means1 = [single.train_episode(0.81 * 0.9 ** e) for e in range(EPISODES)]
    per1 = single.episode_rewards_global()
    means2, per2, _ = _run_two_ranks({"_chain": True})
    assert np.array_equal(per1, per2)
    assert np.allclose(means1, means2, rtol=0, atol=1e-9)


@pytest.mark.timeout(300)
def test_two_rank_shared_table_exchange_is_world_size_invariant():
    """Config 3: one shared table, int64 deltas summed over the ranks (host exchange over gloo)
    -> the table and every scenario's rewards equal the single-process run bit for bit."""
    from oracle_engine import OracleEngine
    kw = dict(shared_q=True, exchange="host", battery=dict(capacity=4.0e6 * 3600))
    single = ShardedTrainer(S_TOTAL, N, R, T, engine_factory=OracleEngine, **kw)
    means1 = [single.train_episode(0.81 * 0.9 ** e) for e in range(EPISODES)]
    per1 = single.episode_rewards_global()
    q1 = single.eng.get_q(0, 1)
    assert np.count_nonzero(q1) > 0
    means2, per2, q2 = _run_two_ranks(kw)
    assert np.array_equal(per1, per2) and np.array_equal(q1, q2)
    assert np.allclose(means1, means2, rtol=0, atol=1e-9)


@pytest.fixture(scope="module")
def single_tabular():
    from oracle_engine import OracleEngine
    single = ShardedTrainer(S_TOTAL, N, R, T, engine_factory=OracleEngine)
    means = [single.train_episode(0.81 * 0.9 ** e) for e in range(EPISODES)]
    return means, single.episode_rewards_global()


@pytest.fixture(scope="module")
def single_shared():
    from oracle_engine import OracleEngine
    single = ShardedTrainer(S_TOTAL, N, R, T, engine_factory=OracleEngine, **SHARED_KW)
    means = [single.train_episode(0.81 * 0.9 ** e) for e in range(EPISODES)]
    return means, single.episode_rewards_global(), single.eng.get_q(0, 1)


SHARED_KW = dict(shared_q=True, exchange="host", battery=dict(capacity=4.0e6 * 3600))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [4, 8])
def test_gloo_world_4_8_replicas_match_single_process(world, single_tabular):
    """world in {1, 2, 4, 8} gives identical per-scenario results.  At world 8 the 9
    scenarios shard as 2 + 1 x 7 (shard boundaries with ragged shards)."""
    means1, per1 = single_tabular
    means, per, _ = _run_ranks({}, world)
    assert np.array_equal(per1, per)
    assert np.allclose(means1, means, rtol=0, atol=1e-9)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [4, 8])
def test_gloo_world_4_8_shared_table_is_world_size_invariant(world, single_shared):
    """configs[2]'s exchange at world 4 and 8: the int64 deltas of every rank summed over gloo ->
    the shared table and every scenario's rewards equal the single-process run bit for bit."""
    means1, per1, q1 = single_shared
    means, per, q = _run_ranks(SHARED_KW, world)
    assert np.array_equal(per1, per) and np.array_equal(q1, q)
    assert np.allclose(means1, means, rtol=0, atol=1e-9)


def _dqn_worker(rank, world, port, q, kw):
    import torch.distributed as dist
    from oracle_engine import OracleDQNEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kw = dict(kw)
    S, Tdq, n_ep = kw.pop("_shape", (DQN_S, DQN_T, 2))
    tr = ShardedTrainer(S, N, R, Tdq, rank=rank, world=world, engine_factory=OracleDQNEngine, learner="dqn",
                        exchange="host", **kw)
    means = [tr.train_episode(0.9 ** (1 + e)) for e in range(n_ep)]
    per = tr.episode_rewards_global()
    q.put((rank, means, per, tr.eng.get_weights("online"), tr.eng.get_weights("adam_v")))
    dist.barrier()
    dist.destroy_process_group()


DQN_S, DQN_T = 4, 36


@pytest.mark.timeout(300)
def test_two_rank_dqn_gradient_exchange_is_world_size_invariant():
    """Config 5 on CPU: one shared DQN network, the gradient segments of both ranks gathered over
    gloo every env step (host exchange) -> the weights, Adam state and every scenario's rewards equal
    the single-process run with the same TOTAL segment count and block size, bit for bit."""
    from oracle_engine import OracleDQNEngine
    kw = dict(grad_segments=2, agents_per_block=3)
    single = ShardedTrainer(DQN_S, N, R, DQN_T, engine_factory=OracleDQNEngine, learner="dqn", **kw)
    means1 = [single.train_episode(0.9 ** (1 + e)) for e in range(2)]
    per1 = single.episode_rewards_global()
    w1, v1 = single.eng.get_weights("online"), single.eng.get_weights("adam_v")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dqn_worker, args=(r, 2, port, q, kw)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=240) for _ in range(2)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, means2, per2, w2, v2 in got:
        assert np.array_equal(w1, w2) and np.array_equal(v1, v2), f"rank {rank} weights differ"
        assert np.array_equal(per1, per2)
        assert np.allclose(means1, means2, rtol=0, atol=1e-9)
    from oracle.dqn import glorot_init
    assert not np.array_equal(w1, glorot_init(1, 0))  # the network did train
    # a different segment count changes the summation order (and so, in general, the bits)
    other = ShardedTrainer(DQN_S, N, R, DQN_T, engine_factory=OracleDQNEngine, learner="dqn", grad_segments=1,
                           agents_per_block=3)
    [other.train_episode(0.9 ** (1 + e)) for e in range(2)]
    assert np.allclose(other.eng.get_weights("online"), w1, rtol=1e-5, atol=1e-7)


G8_S, G8_T = 8, 32  # 8 gradient segments of one scenario each; 32 fill steps >= the 31 a batch needs


@pytest.mark.timeout(600)
def test_dqn_eight_segments_world_4_and_8_match_single_process():
    """configs[4]'s exchange with G = 8 segments: 1 rank x 8, 4 ranks x 2 and 8 ranks x 1 segments
    (the driver's 8-GPU layout) give the same weights, Adam state and rewards bit for bit."""
    from oracle_engine import OracleDQNEngine
    kw = dict(grad_segments=8, agents_per_block=2)
    single = ShardedTrainer(G8_S, N, R, G8_T, engine_factory=OracleDQNEngine, learner="dqn", **kw)
    means1 = [single.train_episode(0.9)]
    per1 = single.episode_rewards_global()
    w1, v1 = single.eng.get_weights("online"), single.eng.get_weights("adam_v")
    for world in (4, 8):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        wkw = dict(kw, _shape=(G8_S, G8_T, 1))
        procs = [ctx.Process(target=_dqn_worker, args=(r, world, port, q, wkw)) for r in range(world)]
        for p in procs:
            p.start()
        got = [q.get(timeout=400) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert sorted(g[0] for g in got) == list(range(world))
        for rank, means2, per2, w2, v2 in got:
            assert np.array_equal(w1, w2) and np.array_equal(v1, v2), f"world {world} rank {rank} weights differ"
            assert np.array_equal(per1, per2)
            assert np.allclose(means1, means2, rtol=0, atol=1e-9)


def test_dqn_trainer_rejects_segments_world_cannot_divide():
    """grad_segments must be a multiple of the world size (whole segments per rank) and divide the
    scenarios: 8 segments over 3 ranks, or 8 segments of 12 scenarios, are refused."""
    from oracle_engine import OracleDQNEngine
    with pytest.raises(ValueError):
        ShardedTrainer(G8_S, N, R, G8_T, world=3, rank=0, engine_factory=OracleDQNEngine, learner="dqn",
                       grad_segments=8)
    with pytest.raises(ValueError):
        ShardedTrainer(12, N, R, G8_T, world=4, rank=0, engine_factory=OracleDQNEngine, learner="dqn",
                       grad_segments=8)


def test_dqn_trainer_rejects_bad_segments():
    from oracle_engine import OracleDQNEngine
    with pytest.raises(ValueError):
        ShardedTrainer(DQN_S, N, R, DQN_T, engine_factory=OracleDQNEngine, learner="dqn", grad_segments=3)


@pytest.mark.timeout(300)
def test_bench_gpus_2_spawns_two_ranks():
    """``bench.py --gpus 2`` without torchrun starts 2 rank processes itself (gloo rendezvous on
    127.0.0.1), shards the scenarios and prints ONE line from rank 0 with n_gpus = 2; the per-rank
    times and the launcher's record come with it.  The engine is the oracle stand-in."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["P2PMG_BENCH_TEST_ENGINE"] = "bench_test_engine:BenchOracleEngine"
    env["PYTHONPATH"] = os.pathsep.join([root, os.path.join(root, "tests"), env.get("PYTHONPATH", "")])
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--scenarios", "3", "--horizon", "12", "--no-cpu-baseline", *PRIMARY_ONLY]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and len(d["rank_times_s"]) == 2
    assert d["launcher"]["ranks"] == 2 and d["launcher"]["rank_exit_codes"] == [0, 0]
    assert d["config"]["agent_steps_per_step"] == 2 * 3 * 2 * 12
    assert d["test_engine"] and d["rccl_nranks"] == 0 and "rccl_error" in d
    assert d["ms_per_step"] == pytest.approx(max(d["rank_times_s"]) / 2 * 1e3)
    # the same episodes in one process (world 1, 6 scenarios) give the same global mean reward
    cmd1 = [sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
            "--scenarios", "6", "--horizon", "12", "--no-cpu-baseline", *PRIMARY_ONLY]
    p1 = subprocess.run(cmd1, env=env, capture_output=True, text=True, timeout=240)
    assert p1.returncode == 0, p1.stderr[-3000:]
    d1 = json.loads([x for x in p1.stdout.splitlines() if x.startswith("{")][0])
    assert d1["n_gpus"] == 1
    assert d1["mean_episode_reward"] == pytest.approx(d["mean_episode_reward"], rel=1e-12)


def _bench_env(**extra):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["P2PMG_BENCH_TEST_ENGINE"] = "bench_test_engine:BenchOracleEngine"
    env["PYTHONPATH"] = os.pathsep.join([root, os.path.join(root, "tests"), env.get("PYTHONPATH", "")])
    env.update(extra)
    return root, env


def _bench_line(root, env, *args):
    import json
    import subprocess
    import sys
    cmd = [sys.executable, os.path.join(root, "bench.py"), *args, "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    return lines[0]


@pytest.mark.timeout(300)
def test_bench_launcher_survives_chatty_rank0():
    """Rank 0 writing more than 1 MB before its JSON line (a verbose library) must not block on a
    full pipe: the launcher collects its output in a file and still returns the line."""
    root, env = _bench_env(P2PMG_BENCH_TEST_NOISE=str(1_200_000))
    d = _bench_line(root, env, "--gpus", "2", "--steps", "1", "--warmup", "0", "--scenarios", "2", "--horizon", "8",
                    *PRIMARY_ONLY)
    assert d["n_gpus"] == 2 and d["launcher"]["rank_exit_codes"] == [0, 0]


@pytest.mark.timeout(300)
def test_bench_host_rehearsal_shared_table():
    """configs[2]'s exchange step at --gpus 2 with --exchange host (the one-GPU rehearsal): int64
    deltas summed over gloo, every replica's table fingerprint equal, and the same mean reward as
    one rank with both shards (integer sums do not depend on the split)."""
    root, env = _bench_env()
    common = ["--workload", "config3", "--agents", "4", "--horizon", "12", "--steps", "2", "--warmup", "1"]
    d = _bench_line(root, env, "--gpus", "2", "--exchange", "host", "--scenarios", "3", *common)
    assert d["exchange"] == "host-rehearsal" and d["table_replicas_identical"] and d["n_gpus"] == 2
    d1 = _bench_line(root, env, "--scenarios", "6", *common)
    assert d1["mean_episode_reward"] == pytest.approx(d["mean_episode_reward"], rel=1e-12)


@pytest.mark.timeout(300)
def test_bench_host_rehearsal_dqn():
    """configs[4] at --gpus 2 with --exchange host: the gradient segments gathered over gloo every env
    step; the shared network's replicas on both ranks are bit-identical."""
    root, env = _bench_env(P2PMG_BENCH_TEST_DQN_ENGINE="bench_test_engine:BenchOracleDQNEngine")
    d = _bench_line(root, env, "--gpus", "2", "--exchange", "host", "--workload", "config5", "--scenarios", "2",
                    "--horizon", "40", "--steps", "1", "--warmup", "0")
    assert d["exchange"] == "host-rehearsal" and d["network_replicas_identical"] and d["n_gpus"] == 2


SMALL_DEFAULT_LINE = ("--steps", "2", "--warmup", "1", "--horizon", "12", "--schedule-episodes", "24",
                      "--eps-windows", "6,15", "--eps-window-steps", "3", "--secondary-agents", "4",
                      "--secondary-horizon", "12", "--secondary-steps", "2", "--secondary-warmup", "1",
                      "--extra-horizon", "12", "--extra-steps", "2", "--extra-warmup", "1")


def _default_line(world, scen_per_rank):
    root, env = _bench_env(P2PMG_BENCH_TEST_DQN_ENGINE="bench_test_engine:BenchOracleDQNEngine")
    extra = ("--gpus", str(world)) if world > 1 else ()
    return _bench_line(root, env, *extra, "--scenarios", str(scen_per_rank),
                       "--secondary-scenarios", str(scen_per_rank), "--extra-scenarios", str(scen_per_rank),
                       *SMALL_DEFAULT_LINE)


@pytest.mark.timeout(300)
def test_bench_setup_failure_on_one_rank_drops_the_workload_everywhere():
    """configs[4]'s context fails to set up on rank 1 only (P2PMG_BENCH_TEST_FAIL_DQN_RANK): every rank
    learns it before the workload's first collective (bench.agree_setup), the record carries the
    error, and the ranks go on to the next record instead of waiting for rank 1 in a collective."""
    root, env = _bench_env(P2PMG_BENCH_TEST_DQN_ENGINE="bench_test_engine:BenchOracleDQNEngine",
                           P2PMG_BENCH_TEST_FAIL_DQN_RANK="1")
    d = _bench_line(root, env, "--gpus", "2", "--scenarios", "4", "--secondary-scenarios", "4",
                    "--extra-scenarios", "4", *SMALL_DEFAULT_LINE)
    assert "error" in d["secondary_dqn"] and "rank(s) [1]" in d["secondary_dqn"]["error"]
    assert d["secondary_year"]["value"] > 0 and d["value"] > 0


@pytest.fixture(scope="module")
def default_line_world1():
    return _default_line(1, 8)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 8])
def test_bench_default_line_carries_configs2_secondary_and_value_at_eps(world, default_line_world1):
    """The driver's default command: the configs[1] line, then configs[2] (shared table, int64 delta
    exchange) measured by the same ranks as ``secondary``, and configs[1] continued through the
    reference's epsilon schedule as ``value_at_eps``.  World 1, 2 and 8 (the driver's SCALE points)
    process the same global scenarios (8 per job), so every mean reward equals world 1's."""
    d = default_line_world1 if world == 1 else _default_line(world, 8 // world)
    assert d["n_gpus"] == world and d["config"]["agent_steps_per_step"] == 8 * 2 * 12
    assert d["epsilon_range"] == [0.729, 0.729] or np.allclose(d["epsilon_range"], [0.729, 0.729])
    ve = d["value_at_eps"]
    assert [w["first_episode"] for w in ve["windows"]] == [6, 15]
    assert all(w["episodes"] == 3 and w["value"] > 0 for w in ve["windows"])
    assert ve["continuation"]["first_episode"] == 3 and ve["continuation"]["episodes"] == 21
    s = d["secondary"]
    assert "error" not in s, s
    assert s["config"]["shared_q"] and s["config"]["battery"] and s["config"]["agent_steps_per_step"] == 8 * 4 * 12
    assert s["steps"] == 2 and s["value"] > 0 and s["ms_per_step"] > 0 and "roofline" in s
    assert s["table_replicas_identical"]
    # per-agent tables run chained launches: contiguous from episode 0 to the schedule's end, at most
    # 64 episodes each, every one ending at a metric point of its call (warm-up 1, timed 2, the
    # schedule's calls to the windows at 6 and 15 and to episode 24); the timed call is one launch
    la = d["launch"]
    assert la["mode"].startswith("chained")
    firsts = [f for f, _ in la["launches"]]
    assert firsts[0] == 0 and all(f + n == g for (f, n), g in zip(la["launches"], firsts[1:]))
    assert sum(n for _, n in la["launches"]) == 24 and all(1 <= n <= 64 for _, n in la["launches"])
    assert [1, 2] == [n for f, n in la["launches"] if f in (0, 1)]
    assert {6, 9, 15, 18} <= set(firsts) and d["roofline"]["episodes_per_launch"] == [2]
    if world > 1:
        assert len(d["launcher"]["rank_exit_codes"]) == world
        assert s["exchange"] == "host-rehearsal" and "exchange_fallback" in s  # no RCCL in the test engine
        assert len(s["rank_times_s"]) == world
    # the further BASELINE configs on the same ranks: configs[4] (DQN, shared network, gradient-segment
    # exchange at world > 1) and configs[3] (heterogeneous mixes, per-agent tables, battery)
    q, y = d["secondary_dqn"], d["secondary_year"]
    assert "error" not in q and "error" not in y, (q, y)
    assert q["steps"] == 2 and q["value"] > 0 and q["roofline"]["bound"] == "mfma"
    assert q["config"]["agent_steps_per_step"] == 8 * 2 * 12 and q["network_replicas_identical"]
    assert q["grad_layout"] and "setup_s" in q
    assert y["steps"] == 2 and y["value"] > 0 and y["config"]["battery"] and not y["config"]["shared_q"]
    assert y["config"]["agent_steps_per_step"] == 8 * 4 * 12 and y["config"]["workload"].startswith("configs[3]")
    assert y["setup_s"]["inputs"] >= 0
    if world > 1:
        assert q["exchange"] == "host-rehearsal" and "exchange_fallback" in q and len(q["rank_times_s"]) == world
    w1 = default_line_world1
    assert q["mean_episode_reward"] == pytest.approx(w1["secondary_dqn"]["mean_episode_reward"], rel=1e-6)
    assert y["mean_episode_reward"] == pytest.approx(w1["secondary_year"]["mean_episode_reward"], rel=1e-12)
    assert d["mean_episode_reward"] == pytest.approx(w1["mean_episode_reward"], rel=1e-12)
    assert ve["mean_episode_reward_last"] == pytest.approx(w1["value_at_eps"]["mean_episode_reward_last"], rel=1e-12)
    assert s["mean_episode_reward"] == pytest.approx(w1["secondary"]["mean_episode_reward"], rel=1e-12)


def test_visible_gpus_without_runtime(monkeypatch):
    """The launcher counts GPUs from the KFD topology (no HIP / torch.cuda in the parent) and
    honours a *_VISIBLE_DEVICES list."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.delenv("P2PMG_BENCH_TEST_ENGINE", raising=False)
    n = bench.visible_gpus()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert bench.visible_gpus() == min(n, 1)


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)


def test_bench_launcher_stops_surviving_ranks_when_one_fails():
    """A rank that dies (here rank 1, at engine construction) must not leave rank 0 waiting in a
    collective forever: the launcher kills the survivors and exits non-zero with the exit codes."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["P2PMG_BENCH_TEST_ENGINE"] = "bench_test_engine:BenchOracleEngine"
    env["P2PMG_BENCH_TEST_FAIL_RANK"] = "1"
    env["PYTHONPATH"] = os.pathsep.join([root, os.path.join(root, "tests"), env.get("PYTHONPATH", "")])
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--scenarios", "3", "--horizon", "12", "--no-cpu-baseline", *PRIMARY_ONLY]
    t0 = time.time()
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200)
    assert p.returncode != 0
    assert "rank exit codes" in p.stderr
    assert not [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert time.time() - t0 < 150
