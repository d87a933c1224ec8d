#!/usr/bin/env python
"""bench.py — agent-steps/s of the P2PMicrogrid hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 independent scenarios x the reference thesis community
(N = 2 PV + heat-pump households, R = 1 -> 2 negotiation rounds, T = 96 quarter-hour slots per
episode, heterogeneous ratings/T0, per-agent float64 Q-tables, epsilon-greedy tabular Q-learning
with the reference's epsilon schedule).  One bench "step" = one training episode
(CommunityMicrogrid.train_episode, community.py:149-182) for every scenario of the rank:
T0 reset (heating.py:145-152) + exploration draws + the fused episode kernel.  Data are
synthetic profiles with the reference schema (the SQLite source is not available).

N GPUs: one process per GPU (torchrun), scenarios sharded with no data-path collective (each
scenario's tables are private: "replicas only").  Every workload creates an RCCL communicator
over the ranks (xGMI); the episode metrics (sum and count of the episode rewards, community.py:179)
are all-reduced over it every ``--metric-every`` episodes (the reference's logging cadence,
community.py:279-288) and after the last one, and the line reports ``rccl_nranks`` as the
communicator counts them.  torch.distributed(gloo) carries only the id broadcast, the barrier and
the max-over-ranks time.  value = all ranks' agent-steps / max time (weak scaling).

``--workload config4`` (BASELINE.json configs[3]): 8192 scenarios x 4 households per GPU with
heterogeneous asset mixes (dataset.asset_mix: Consumers without PV, no / 3 kW / 5 kW heat pumps,
10 kWh battery or NoStorage), one-year episodes (T = 35,040 quarter-hour slots), per-agent f64
Q-tables (168 GB per GPU, sized to HBM): replicas only, like configs[1].

``--workload config3`` (BASELINE.json configs[2]): 1M scenarios x 16 agents with battery storage
over 8 GPUs = 125,000 scenarios (2M agents) per GPU, ONE shared f32 Q-table whose int64
fixed-point TD deltas are all-reduced over RCCL once per episode (the path's real exchange step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-steps/sec (whole node, rollout+Q-update) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes_per_agent_step(R: int, q_bytes: int, outputs: int = 2) -> int:
    """8 (load_w, pv_w) + q_bytes * (3(R+1) + 3 + 2) (greedy gathers per round,
    next-state max, Q[s,a] read+write) + 4 * outputs (reward, cost).  The persistent variant keeps
    T_in/T_m in registers for the whole episode, so the 16 B of state traffic is dropped."""
    return 8 + q_bytes * (3 * (R + 1) + 3 + 2) + 4 * outputs


def sector_model_per_agent_step(N: int, R: int, eps: float, battery: bool, q_bytes: int = 8):
    """The HBM bytes the fast per-agent-table kernel moves per agent-step at the memory system's
    32-B sector granularity (what the FETCH_SIZE / WRITE_SIZE passes count), next to the
    algorithmic bytes of SURVEY §8(d).  Components (p2pmg_kernels.hip::episode_fast_kernel):
    reads -- the profile pair (8 B, coalesced), the step pre-pass word (8 B), the exploration code
    word (4 B), for N = 2 without a battery the round-1 bins word (4 B); Q rows as whole sectors:
    round 0's row only when round 0 is greedy (1 - eps), the round-1 row(s) (3 candidates for N = 2
    without a battery, else the one dependent row), the next-state row; the producer blocks' re-read
    of the profiles for the next episode's pre-pass (8 B).  Writes -- the TD store (8 B landing in a
    32-B sector), the {reward, cost} record row (8 B), the next episode's pre-pass words (8 + 4 B,
    + 4 B of bins for the N = 2 path).  The Q-row sectors and the TD sector are the 2x over the
    algorithmic bytes that the PMC traffic shows (VERDICT r02 'wasted traffic')."""
    sector = 32 if q_bytes == 8 else 16
    cand = N == 2 and R >= 1 and not battery
    rows = (1.0 - eps) + (3 if cand else R) + 1
    reads = {"profile": 8, "prepass_word": 8, "code_word": 4, "round1_bins": 4 if cand else 0,
             "q_rows_sectors": rows * sector, "producer_profile_reread": 8}
    writes = {"td_store_sector": 32, "record_row": 8, "next_prepass_words": 12 + (4 if cand else 0)}
    return {"read": reads, "write": writes, "read_total": sum(reads.values()), "write_total": sum(writes.values()),
            "total": sum(reads.values()) + sum(writes.values()), "epsilon": eps,
            "note": "per agent-step, at 32-B sectors; q_rows = (1 - eps) round-0 row + round-1 row(s) + next-state row"}


def algorithmic_bytes_per_agent_step_shared(agents: int, q_bytes: int, battery: bool, outputs: int = 2) -> float:
    """SURVEY.md §8(d), shared table: 8 (load_w, pv_w) + 4 * outputs + the table read once and its
    int64 delta buffer read+written once per step, amortised over the agents of the step
    (2 * |Q| * q_bytes + 2 * |Q| * 8) / agents.  T_in/T_m/SoC live in registers for the episode.
    Per-agent gathers hit the same 1.9 MB table and are cache traffic, not HBM traffic."""
    q_entries = 20 ** 4 * 3
    return 8 + 4 * outputs + (2 * q_entries * q_bytes + 2 * q_entries * 8) / agents


def epsilon_at(episode: int, eps0: float = 0.81, decay: float = 0.9, every: int = 50, floor: float = 0.1) -> float:
    """community.py:279-286 + rl.py:131-132: decay after episodes 0, 50, 100, ... (floor 0.1)."""
    n = 0 if episode == 0 else (episode - 1) // every + 1
    eps = eps0
    for _ in range(n):
        eps = max(floor, decay * eps)
    return eps


def dist_setup(gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpus is None:  # torchrun without --gpus: one rank per GPU of the launch
        gpus = world
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: launch N ranks with torchrun "
                         f"--nproc-per-node N, or run bench.py --gpus N without WORLD_SIZE (it spawns them)")
    # rehearsal only (more ranks than GPUs on one box): the launcher maps rank -> device
    local = int(os.environ.get("P2PMG_BENCH_DEVICE", local))
    if world > 1:
        import torch.distributed as dist  # gloo: barrier + max-time only, no GPU interaction
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    """GPUs this node exposes, counted without any GPU runtime in this process (the launcher must
    stay GPU-free: its children are the ranks).  The KFD topology lists one node per CPU socket and
    GPU; GPU nodes carry a non-zero gpu_id.  A *_VISIBLE_DEVICES list narrows the count as the HIP
    runtime would."""
    if os.environ.get("P2PMG_BENCH_TEST_ENGINE"):
        return 0
    import glob
    n = 0
    for path in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            n += int(open(path).read().strip() or 0) != 0
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(argv, gpus: int) -> int:
    """``bench.py --gpus N`` without WORLD_SIZE: start N rank processes of this same script (one
    per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, as torchrun would), wait for all of
    them, and print rank 0's JSON line with the launcher's facts added.  This process never
    touches the GPU and never re-execs: the ranks are fresh child processes.  With fewer visible
    GPUs than ranks (a one-GPU rehearsal) ranks share devices round-robin and the line says so."""
    import subprocess
    import tempfile
    n_dev = visible_gpus()
    if n_dev == 0 and not os.environ.get("P2PMG_BENCH_TEST_ENGINE"):
        print("bench.py launcher: no GPU found in the KFD topology (/sys/class/kfd) for the ranks",
              file=sys.stderr, flush=True)
        return 2
    port = _free_port()
    procs = []
    # rank 0's stdout goes to a file, read after the ranks exit: a pipe nobody reads while they run
    # would block rank 0 once it filled (verbose libraries), and the others in its collectives
    out_file = tempfile.TemporaryFile(mode="w+")
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if 0 < n_dev < gpus:
            env["P2PMG_BENCH_DEVICE"] = str(r % n_dev)
            env["P2PMG_BENCH_RANKS_SHARE_GPU"] = "1"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out_file if r == 0 else subprocess.DEVNULL, text=True))
    # wait for every rank; if one fails, stop the others (they would wait in a collective forever)
    import time as _t
    while any(p.poll() is None for p in procs):
        if any(p.poll() not in (None, 0) for p in procs):
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        _t.sleep(0.2)
    rcs = [p.wait() for p in procs]
    out_file.seek(0)
    out0 = out_file.read()
    out_file.close()
    line = None
    for ln in (out0 or "").splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                continue
        elif ln:
            print(ln, flush=True)
    if any(rcs) or line is None:
        print(f"bench.py launcher: rank exit codes {rcs}", file=sys.stderr, flush=True)
        return next((rc for rc in rcs if rc), 1)
    line["launcher"] = {"kind": "bench.py spawn (subprocess per rank)", "ranks": gpus, "rank_exit_codes": rcs,
                        "visible_gpus": n_dev, "ranks_share_gpus": bool(0 < n_dev < gpus)}
    print(json.dumps(line), flush=True)
    return 0


def engine_class():
    """The HIP engine.  P2PMG_BENCH_TEST_ENGINE=module:Class swaps in a host stand-in so the CPU
    test suite can drive the launcher and the collectives end to end; a line produced that way
    carries ``test_engine`` and is not a measurement."""
    spec = os.environ.get("P2PMG_BENCH_TEST_ENGINE")
    if not spec:
        from p2pmicrogrid_amd.engine import DeviceCommunityBatch
        return DeviceCommunityBatch
    import importlib
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)


def dqn_engine_class():
    """DeviceDQNBatch, or the CPU test suite's stand-in (P2PMG_BENCH_TEST_DQN_ENGINE=module:Class)."""
    spec = os.environ.get("P2PMG_BENCH_TEST_DQN_ENGINE")
    if not spec:
        from p2pmicrogrid_amd.dqn import DeviceDQNBatch
        return DeviceDQNBatch
    import importlib
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)


def weights_fingerprint(w) -> int:
    """64-bit fingerprint of an array's bits (host side; the shared network is 18 KB)."""
    import hashlib
    return int.from_bytes(hashlib.blake2b(np.ascontiguousarray(w).tobytes(), digest_size=8).digest(), "little")


def all_gather_float(x: float, world: int):
    if world == 1:
        return [x]
    import torch
    import torch.distributed as dist
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, torch.tensor([x], dtype=torch.float64))
    return [float(t.item()) for t in out]


def agree_setup(err, world: int):
    """A workload's setup (inputs, context, uploads) went through on every rank, or the workload is
    dropped on every rank: the ranks exchange one flag over gloo before their first collective, so a
    rank whose setup failed (device or shared memory) never leaves the others waiting in one."""
    flags = all_gather_float(0.0 if err is not None else 1.0, world)
    if err is not None:
        raise err
    bad = [r for r, f in enumerate(flags) if f != 1.0]
    if bad:
        raise RuntimeError(f"workload setup failed on rank(s) {bad}")


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def exchange_kind(args, world: int) -> str:
    """How the shared-state workloads sum their data-path state over the ranks: "rccl" (device
    collectives over xGMI, the production path and the default) or "host" (gloo over the host,
    a labelled rehearsal for ranks that share one GPU, where RCCL refuses a second rank)."""
    if world == 1:
        return "none"
    if args.exchange != "auto":
        return args.exchange
    return "host" if os.environ.get("P2PMG_BENCH_RANKS_SHARE_GPU") else "rccl"


def rccl_comm(eng, rank: int, world: int, required: bool = False, world1: bool = False) -> str:
    """The RCCL communicator of the rank's context (rank 0's unique id broadcast over gloo).
    Returns "" or the error; a rank without a communicator reports its metrics over gloo, so a
    replicas-only workload still runs (required=True: the shared-state workloads need it).
    world1 (--rccl-world1): a one-rank communicator too, so the data-path collectives of the
    multi-GPU code path run on one GPU (their cost without the xGMI transfer)."""
    if world == 1 and world1 and not os.environ.get("P2PMG_BENCH_TEST_ENGINE"):
        from p2pmicrogrid_amd.engine import comm_unique_id
        try:
            eng.comm_init(comm_unique_id(), 0, 1)
        except Exception as e:  # noqa: BLE001
            return f"{type(e).__name__}: {e}"
        return ""
    if world == 1:
        return ""
    from p2pmicrogrid_amd.distributed import broadcast_bytes
    from p2pmicrogrid_amd.engine import comm_unique_id
    uid = None
    if rank == 0 and not os.environ.get("P2PMG_BENCH_TEST_ENGINE"):
        try:
            uid = comm_unique_id()
        except Exception:  # noqa: BLE001  (every rank learns it from the empty id)
            uid = b""
    uid = broadcast_bytes(uid, world)
    if not uid:
        if required:
            raise RuntimeError("RCCL unavailable: the shared-state workloads need the device all-reduce")
        return "no RCCL unique id"
    try:
        eng.comm_init(uid, rank, world)
    except Exception as e:  # noqa: BLE001
        if required:
            raise
        return f"{type(e).__name__}: {e}"
    return ""


def episode_metrics(eng, world: int, comm_err: str):
    """(sum, count) of the episode rewards over every rank: RCCL, or gloo without a communicator."""
    if not comm_err:
        return eng.allreduce_metrics()
    from p2pmicrogrid_amd.distributed import all_reduce_sum
    local = eng.episode_reward().astype(np.float64)
    tot = all_reduce_sum(np.array([local.sum(), local.size]), world)
    return float(tot[0]), int(tot[1])


BATTERY_J = 10.0 * 3.6e6  # 10 kWh per household battery (config 3; the reference fixes no size)

WORKLOADS = {
    # name: (scenarios per GPU, agents, rounds R, horizon, q dtype, shared table, battery)
    "config2": (4096, 2, 1, 96, "f64", False, False),
    "config3": (125000, 16, 1, 96, "f32", True, True),
    "config5": (4096, 2, 1, 96, "f32", True, False),  # DQN, one shared network (data-parallel)
    # configs[3]: heterogeneous PV / heat-pump / battery mixes, 1-year episodes, per-agent tables
    "config4": (8192, 4, 1, 365 * 96, "f64", False, True),  # 32,768 f64 tables = 168 GB of HBM
}
HETERO = {"config4"}

MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA (v_mfma_f32_16x16x4_f32) = f32 vector rate
DQN_FWD_FLOP = 2 * (5 * 64 + 64 * 64 + 64 * 1)  # QNetwork (rl.py:135-148): 8,960 FLOP per row


def collective_record(eng, world: int, steps: int, kind: str = "RCCL allReduce (data path)", world1: bool = False):
    """The data-path collectives of the timed episodes (shared-table delta all-reduce once per
    episode, DQN gradient-segment all-gather once per env step): HIP-event time on the rank's
    stream, every call counted, rank 0's view (world > 1, or a --rccl-world1 communicator)."""
    if (world <= 1 and not world1) or not hasattr(eng, "collective_ms"):
        return None
    total, n = eng.collective_ms()
    return {"kind": kind, "calls": n, "ms_total": total,
            "ms_per_step": total / max(steps, 1), "us_per_call": 1e3 * total / n if n else None}


def dqn_flop_per_agent_step(R: int) -> int:
    """Trainer._train (rl.py:307-333) = 3 target forwards x 32 samples +
    1 online forward + backward (2x forward) x 32 = 32 * 6 * 8,960; the greedy action choice
    adds 3 forwards per negotiation round (ActorModel rl.py:186-194)."""
    return 32 * 6 * DQN_FWD_FLOP + 3 * (R + 1) * DQN_FWD_FLOP


def _cpu_worker(job):
    """One process of the all-cores CPU baseline: a bench.py CPU-baseline function by name."""
    name, kw = job
    return globals()[name](**kw)


def cpu_workers():
    """(workers, rule): host cores the CPU baseline may use = one GPU's share of the box.  A GPU box
    gives each GPU 16 host cores and says so in OMP_NUM_THREADS (= MAX_JOBS = 16 there), while
    os.cpu_count() reports the whole machine; so the share is OMP_NUM_THREADS when it is set, else
    os.cpu_count() // the GPUs the node exposes (all cores without a GPU), never more than this
    process's CPU affinity.  P2PMG_CPU_WORKERS overrides."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    if os.environ.get("P2PMG_CPU_WORKERS"):
        n, rule = int(os.environ["P2PMG_CPU_WORKERS"]), "P2PMG_CPU_WORKERS"
    elif os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n, rule = int(os.environ["OMP_NUM_THREADS"]), "OMP_NUM_THREADS (the box's per-GPU CPU share)"
    else:
        g = visible_gpus()
        n, rule = (os.cpu_count() or 1) // max(1, g), f"os.cpu_count() // {max(1, g)} visible GPU(s)"
    n = max(1, min(n, aff))
    return n, f"{rule}, capped by the CPU affinity ({aff})"


def cpu_baseline_all_cores(name: str, kw: dict, workers: int) -> dict:
    """The same CPU-baseline function in `workers` concurrent single-threaded processes, each on its
    own scenario slice (first_scenario = k * S), started together; value = the sum of their rates.
    The one-core figure of the same run is kept under "one_core"."""
    import concurrent.futures as cf
    import multiprocessing as mp
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"  # one thread per worker process (NumPy / BLAS)
    try:
        jobs = [(name, dict(kw, first=k * kw.get("S", 1))) for k in range(workers)]
        with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
            res = list(ex.map(_cpu_worker, jobs))
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old
    out = dict(res[0])
    out["one_core"] = {"value": res[0]["value"], "sample": res[0]["sample"]}
    out.update(value=sum(r["value"] for r in res), cores=workers, workers=workers, threads_per_worker=1,
               per_worker=[r["value"] for r in res],
               sample=f"{workers} concurrent processes x ({res[0]['sample']})")
    return out


def cpu_baseline_dqn(seconds: float, S: int = 2, N: int = 2, R: int = 1, T: int = 96, first: int = 0):
    """oracle/dqn.py (NumPy, one thread) on a bounded sample: one fill episode, then train episodes."""
    from oracle import dqn as odqn
    from p2pmicrogrid_amd.dataset import scenario_batch
    inp = scenario_batch(S, N, T, first_scenario=first)
    th0 = odqn.glorot_init(1, 0)
    ob = odqn.OracleDQNBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                             env_time=inp.time[None], env_tout=inp.t_out, theta0=th0, shared=True,
                             order="matmul")  # the vectorised NumPy form (the kernel-order form is a checker)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    ob.run_episode("fill", rng="philox", episode=0, eps=1.0)
    t0 = time.perf_counter()
    done = 0
    while True:
        ob.run_episode("train", rng="philox", episode=1 + done, eps=0.9 ** (1 + done))
        done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": S * N * T * done / dt, "unit": "agent-steps/s", "cores": 1, "kind": "port",
            "label": "CPU restatement (oracle/dqn.py, NumPy matmul order)",
            "sample": f"{S} scenarios x N={N} DQN agents (R={R}, T={T}, shared network), {done} training "
                      f"episodes after one fill episode, oracle/dqn.py NumPy, {dt:.1f} s"}


def run_dqn(args, rank, world, local, S, N, R, T, steps, warmup, cpu_seconds):
    """configs[4]: DQN agents with ONE shared Q-network (data-parallel): every env step runs the
    act launch (greedy forwards on the Q-MLP, market, reward, replay append, RC update) and the
    train launch (32-sample batches on f32 MFMA) + gradient reduce (+ RCCL all-gather of the
    gradient segments over ranks) + Adam/soft update.  One bench step = one training episode
    (T env steps) of every scenario.  Rank 0 returns the record, the other ranks None."""
    from p2pmicrogrid_amd.dataset import scenario_batch
    t_setup = time.perf_counter()
    first = rank * S

    def build():
        inp = scenario_batch(S, N, T, first_scenario=first)
        dkw = {}
        if args.grad_segments:  # the split path (segment fold -> exchange -> dqn_adam_shared_kernel) at any world
            dkw["grad_segments"] = args.grad_segments
        if args.agents_per_block:
            dkw["agents_per_block"] = args.agents_per_block
        e = dqn_engine_class()(S, N, R, T, shared=True, device=local, scenario_offset=first, init_seed=0, **dkw)
        e.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
        e.set_profiles(inp.load_w, inp.pv_w)
        e.set_max_in(inp.max_in)
        e.set_temperatures(inp.t_in0, inp.t_m0)
        return e

    eng, err = None, None
    try:
        eng = build()
    except Exception as e:  # noqa: BLE001  (agree_setup re-raises it on this rank, and on the others)
        err = e
    agree_setup(err, world)
    xk = exchange_kind(args, world)
    fallback, comm_err = None, ""
    if xk != "host":  # gradient-segment all-gather every env step + metrics over RCCL
        comm_err = rccl_comm(eng, rank, world, required=args.exchange == "rccl", world1=args.rccl_world1)
        if comm_err and world > 1:  # --exchange auto without a communicator: the labelled host exchange
            fallback, xk = comm_err, "host"
    if xk == "host":  # rehearsal: the gradient segments gathered over gloo every env step
        from p2pmicrogrid_amd.distributed import all_gather_rows
        eng.set_grad_exchange(lambda rows: all_gather_rows(rows, rank, world), rank, world)
        comm_err = comm_err or "host-rehearsal exchange (no RCCL communicator)"
    record = ("reward", "cost")
    eng.run_episode("fill", "philox", episode=0, epsilon=1.0, record=record)  # community.init_buffers
    eng.reset_temperatures_philox(1, 0.3)

    def episode(e):  # rl.py:196-197: epsilon 1 x 0.9 per episode, no floor
        eng.run_episode("train", "philox", episode=e, epsilon=0.9 ** e, record=record)
        eng.reset_temperatures_philox(e + 1, 0.3)

    eng.sync()
    t_fill = time.perf_counter() - t_setup
    for e in range(1, 1 + warmup):
        episode(e)
    if world > 1 and warmup > 0:  # the first metric all-reduce sets up the communicator: not timed
        episode_metrics(eng, world, comm_err)
    eng.sync()
    eng.reset_kernel_times()
    barrier(world)
    eng.sync()
    t0 = time.perf_counter()
    metrics = None
    for k, e in enumerate(range(1 + warmup, 1 + warmup + steps)):
        episode(e)
        if (k + 1) % args.metric_every == 0 or k + 1 == steps:
            metrics = episode_metrics(eng, world, comm_err)  # RCCL, the reference's 50-episode log
    eng.sync()
    t1 = time.perf_counter()  # before the trailing barrier, as in timed()
    barrier(world)
    rank_times = all_gather_float(t1 - t0, world)
    dt = max(rank_times)
    kms = eng.kernel_times()
    coll = collective_record(eng, world, steps, "RCCL allGather of the gradient segments (data path)",
                             world1=args.rccl_world1 and not comm_err)
    # every rank's replica of the shared network (the same Adam step on the same gathered sum)
    from p2pmicrogrid_amd.distributed import all_gather_concat
    fps = all_gather_concat(np.array([weights_fingerprint(eng.get_weights("online"))], np.uint64), world)
    steps_per_episode = S * N * T
    flop = dqn_flop_per_agent_step(R)
    episode_ms = float(np.mean(kms)) if len(kms) else float("nan")
    achieved = flop * steps_per_episode / (episode_ms * 1e-3) / 1e12
    out = None
    if rank == 0:
        out = {
            "metric": METRIC, "value": world * steps_per_episode * steps / dt, "unit": "agent-steps/s",
            "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": dt / steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic profiles with the reference dataset schema (seed 42), Glorot-uniform init",
            "config": {"workload": f"configs[4]: {S} scenarios/GPU x {N} DQN agents (R={R}, T={T}), one shared "
                                   f"5-64-64-1 Q-network, 32-sample batches per agent-step, Adam + soft update "
                                   f"per step, gradient all-reduce over ranks (RCCL)",
                       "scenarios_per_gpu": S, "agents_per_scenario": N, "rounds": R, "negotiation_rounds": R + 1, "horizon": T,
                       "agent_steps_per_step": world * steps_per_episode,
                       "parallelism": f"scenario-sharded x{world}, data-parallel shared network"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": achieved / MFMA_F32_PEAK_TFS, "traffic": None,
                         "kernel": "DQN episode: the replay-draw pre-pass + T x (act + train + reduce + adam)",
                         "kernel_ms": episode_ms, "flop_per_agent_step": flop,
                         "flop_per_episode": flop * steps_per_episode, "timed_launches": int(len(kms))},
            "mean_episode_reward": metrics[0] / metrics[1],
            "rccl_nranks": eng.comm_nranks() if not comm_err else 0,
            "rank_times_s": rank_times,
            "grad_layout": eng.grad_layout(),
            "network_replicas_identical": bool(np.all(fps == fps[0])),
            "setup_s": {"inputs_context_and_fill_episode": t_fill},
        }
        assert out["network_replicas_identical"], f"shared-network replicas differ across ranks: {fps}"
        if world > 1:
            out["exchange"] = "host-rehearsal" if xk == "host" else "rccl"
        if fallback:
            out["exchange_fallback"] = f"RCCL unavailable ({fallback}): gradient segments gathered over gloo"
        if coll and xk != "host":
            out["collective"] = coll
        if os.environ.get("P2PMG_BENCH_TEST_DQN_ENGINE"):
            out["test_engine"] = os.environ["P2PMG_BENCH_TEST_DQN_ENGINE"]
    eng.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu_seconds > 0:
        workers, rule = cpu_workers()
        out["cpu_baseline"] = cpu_baseline_all_cores("cpu_baseline_dqn", dict(seconds=cpu_seconds, R=R, T=T),
                                                     workers)
        out["cpu_baseline"].update(os_cpu_count=os.cpu_count(), cores_rule=rule)
    return out


def cpu_baseline(seconds: float, S: int = 256, N: int = 2, R: int = 1, T: int = 96, q_dtype: str = "f64",
                 shared: bool = False, battery: bool = False, hetero: bool = False, t_sample: int = 0,
                 first: int = 0):
    """The oracle (NumPy CPU restatement, oracle/restatement.py) on a bounded sample of the same
    workload, single-threaded, Philox exploration.  t_sample > 0: episodes cut to the first
    t_sample slots of the generated horizon (per-step cost does not depend on T)."""
    from oracle.restatement import OracleBatch
    from p2pmicrogrid_amd.dataset import apply_asset_mix, asset_mix, scenario_batch
    inp = scenario_batch(S, N, T, first_scenario=first)
    lv, cap = None, (np.full((S, N), BATTERY_J) if battery else None)
    if hetero:
        mix = asset_mix(S, N, first_scenario=first, battery_j=BATTERY_J)
        inp, lv, cap = apply_asset_mix(inp, mix), mix.hp_levels, mix.battery_capacity
    full_T = T
    if t_sample and t_sample < T:
        T = t_sample
        inp.load_w, inp.pv_w, inp.t_out = inp.load_w[..., :T], inp.pv_w[..., :T], inp.t_out[..., :T]
        inp.time = inp.time[:T]
    ob = OracleBatch(S=S, N=N, R=R, load_w=inp.load_w, pv_w=inp.pv_w, max_in=inp.max_in,
                     env_time=inp.time[None], env_tout=inp.t_out, q_dtype=q_dtype, shared_q=shared,
                     hp_levels=lv, battery_capacity=cap)
    ob.t_in, ob.t_m = inp.t_in0.copy(), inp.t_m0.copy()
    t0 = time.perf_counter()
    eps_done = 0
    while True:
        ob.run_episode("train", rng="philox", episode=eps_done, eps=epsilon_at(eps_done))
        if shared:
            ob.apply_q_delta()
        eps_done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    what = "shared table + battery, " if shared else ""
    if hetero:
        what = f"heterogeneous mixes + battery, first {T} of {full_T} slots, "
    return {"value": S * N * T * eps_done / dt, "unit": "agent-steps/s", "cores": 1, "kind": "port",
            "label": "CPU restatement (oracle/restatement.py)",
            "sample": f"{S} scenarios x N={N} (R={R}, T={T}, {what}{q_dtype} Q), {eps_done} training episodes, "
                      f"oracle/restatement.py vectorised NumPy, {dt:.1f} s"}


def cpu_baseline_per_object(seconds: float, N: int = 2, R: int = 1, T: int = 96):
    """SURVEY.md §8(d) reference-shaped leg: oracle/scalar_loop.py, one object per agent and the
    community.py:149-182 loop nesting (t -> round -> agent) in scalar float32, one thread,
    exploration drawn from np.random in the reference's order, ε schedule of community.py:279-286."""
    from oracle.scalar_loop import ScalarCommunity, ScalarQAgent
    from p2pmicrogrid_amd.dataset import scenario_batch
    inp = scenario_batch(1, N, T)
    agents = [ScalarQAgent(inp.load_w[0, i], inp.pv_w[0, i], inp.max_in[0, i], inp.t_in0[0, i], inp.t_m0[0, i])
              for i in range(N)]
    com = ScalarCommunity(agents, inp.time, inp.t_out[0], R)
    rs = np.random.RandomState(42)
    t0 = time.perf_counter()
    done = 0
    while True:
        com.train_episode(rs=rs, eps=epsilon_at(done))
        done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": N * T * done / dt, "unit": "agent-steps/s", "cores": 1, "kind": "port",
            "sample": f"1 scenario x N={N} (R={R}, T={T}), {done} training episodes, oracle/scalar_loop.py "
                      f"per-object scalar loop (reference loop nesting), {dt:.1f} s"}


CLOCK_GHZ = 2.4          # MI355X peak engine clock
SIMDS = 256 * 4          # 256 CUs x 4 SIMDs
# A SIMD is 16 lanes wide: a wave64 VALU instruction occupies it for one quad-cycle (the SQ counts
# SQ_ACTIVE_INST_VALU = SQ_INSTS_VALU quad-cycles; the f32 vector peak of 157 TF counts packed
# v_pk_fma_f32, two FMAs per lane).  Chip peak: one wave-instruction per SIMD per 4 cycles; a wave
# that has its SIMD to itself issues at most that too (MI355X_MICROARCH.md 'ISSUE cost': 4 cycles).
VALU_PEAK_G = SIMDS * CLOCK_GHZ / 4
SQ_ENGINES = 32          # shader engines whose SQ_BUSY_CYCLES rocprofv3 sums (8 XCDs x 4)
ONE_WAVE_PEAK_G = CLOCK_GHZ / 4


def issue_roofline(workload: str, kernel_ms: float, sizes=None):
    """Instruction-issue roofline of the episode kernel: the VALU wave-instructions one launch
    issues (SQ_INSTS_VALU from the committed rocprofv3 counter pass, profiles/sq_<workload>.json,
    scripts/gpu_sq_counters.sh) over the live kernel time, against the chip's VALU issue peak and,
    when every wave has a SIMD to itself, against that wave's own issue ceiling.  The counter pass
    ran the workload's default sizes: a run at other (scenarios, agents, rounds, horizon) gets no block."""
    path = os.path.join(ROOT, "profiles", f"sq_{workload}.json")
    if not os.path.exists(path) or not kernel_ms == kernel_ms:
        return None
    if sizes is not None and workload in WORKLOADS:
        if tuple(sizes) != tuple(WORKLOADS[workload][:4]):
            return None
    try:
        d = json.load(open(path))
    except Exception:  # noqa: BLE001
        return None
    valu, waves = d["counters_per_launch"]["SQ_INSTS_VALU"], d["counters_per_launch"]["SQ_WAVES"]
    achieved = valu / (kernel_ms * 1e-3) / 1e9
    out = {"unit": "G VALU wave-instructions/s", "achieved": achieved, "peak": VALU_PEAK_G,
           # one VALU per 4 SIMD cycles: nominal, not a ceiling (gfx950 issues v_mul / v_add_f32 at
           # 2.6 / 2.9 SIMD cycles, profiles/r04_ubench_rate.jsonl), so the fractions can pass 1
           "peak_kind": "nominal (1 VALU / 4 SIMD cycles)",
           "frac": achieved / VALU_PEAK_G, "peak_clock_ghz": CLOCK_GHZ, "valu_insts_per_launch": valu, "waves": waves,
           "kernel": d.get("kernel"), "source": os.path.relpath(path, ROOT),
           # from the counter run itself: share of wave cycles issuing any instruction / waiting
           "active_frac": d["derived"].get("frac_active_inst_any"), "wait_frac": d["derived"].get("frac_wait_any")}
    busy = d["counters_per_launch"].get("SQ_BUSY_CYCLES")
    if busy:
        # the same issue fraction at the clock the chip actually ran: SQ_BUSY_CYCLES is summed over
        # the 32 shader engines, so busy / 32 = the launch's length in cycles (at the implied clock
        # it matches the live kernel time); frac_busy_clock = VALU wave-instructions / (SIMDs x
        # cycles / 4), independent of any clock assumption
        cycles = busy / SQ_ENGINES
        out["launch_cycles"] = cycles
        out["frac_busy_clock"] = valu * 4.0 / (SIMDS * cycles)
        out["implied_clock_ghz"] = cycles / (kernel_ms * 1e-3) / 1e9
    if waves <= SIMDS:  # one wave per SIMD at most: each wave is capped at one VALU per 4 cycles
        per_wave = achieved / waves
        out["one_wave_peak"] = ONE_WAVE_PEAK_G
        out["frac_of_one_wave_peak"] = per_wave / ONE_WAVE_PEAK_G
    return out


def gather_roofline(n_agents: int, horizon: int, kernel_ms: float, stages: int = 1, agents_per_wave: int = 32,
                    pool: int = 381, rows: int = 5, source: str = "r02_ubench_gather.jsonl"):
    """Dependent-gather floor of the per-agent-table fast kernel: the same geometry (one 5.12 MB
    f64 table per agent, `agents_per_wave` agents per wave, row gathers whose addresses depend on
    the previous step's rows) with everything else stripped, timed by scripts/ubench_gather.hip
    (scripts/gpu_ubench_gather.sh).  configs[1]: one stage of 5 rows per step, 32 agents per wave
    (profiles/r02_ubench_gather.jsonl).  configs[3]: two DEPENDENT stages per step (the round-0 and
    next-state rows, then the round-1 row addressed from the partners' round-0 actions), 64 agents
    per wave, 32,768 tables, a pool of 400 rows per agent (the oracle's year visits ~334 distinct
    rows per agent in rounds 0-1) (profiles/r04_ubench_gather.jsonl).  frac = that floor over the
    live kernel time: how much of the episode is the memory round trip the reference's
    act -> T_in -> next-state dependency forces, and how much is the decision chain on top of it."""
    path = os.path.join(ROOT, "profiles", source)
    if not os.path.exists(path) or not kernel_ms == kernel_ms:
        return None
    for line in open(path):
        try:
            d = json.loads(line)
        except Exception:  # noqa: BLE001
            continue
        if (d.get("tables") == n_agents and d.get("steps") == horizon and d.get("rows_per_step") == rows
                and d.get("stages", 1) == stages and d.get("agents_per_wave") == agents_per_wave
                and not d.get("pair_lanes") and d.get("pool_rows") == pool):
            floor_us = d["kernel_us"]
            return {"unit": "us per episode", "floor": floor_us, "achieved": kernel_ms * 1e3,
                    "frac": floor_us / (kernel_ms * 1e3), "floor_cycles_per_step": d["cycles_per_step"],
                    "source": os.path.relpath(path, ROOT)}
    return None


def load_traffic(path: str, workload: str):
    """HBM bytes per episode-kernel launch from a committed rocprofv3 PMC summary (or None)."""
    if not path or not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
    except Exception:  # noqa: BLE001
        return None
    if d.get("workload") != workload:
        return None
    return d


MAX_CHAIN = 64  # episodes per chained launch (p2pmg.h p2pmg_run_episodes)
PARALLEL_GEN_ELEMS = 100_000_000  # agent-slots above which the inputs are generated by a worker pool
def traffic_per_episode(traffic, chained: bool):
    """HBM bytes per episode from a PMC summary (profiles/pmc_traffic*.json): its chained-launch
    figure when the run chained its episodes, its one-launch-per-episode figure otherwise."""
    if not traffic:
        return None
    if chained and "hbm_bytes_per_episode" in traffic:
        return traffic.get("hbm_bytes_calibrated_per_episode", traffic["hbm_bytes_per_episode"])
    single = traffic.get("one_launch_per_episode")
    if single:
        return single.get("hbm_bytes_calibrated_per_launch", single.get("hbm_bytes_per_launch"))
    # round 6: counter factors measured per access pattern (scripts/recalibrate_traffic.py)
    return traffic.get("hbm_bytes_calibrated_per_launch", traffic.get("hbm_bytes_per_launch"))


REFERENCE_EPISODES = 1000  # setup.py:30 max_episodes: the reference's training run (community.py:272-298)


def timed(eng, world, fn):
    """Run fn() between a barrier + device sync on both sides; the MAX of every rank's wall time.
    A rank's clock runs from the leading barrier's release to its own device sync after fn(): the
    trailing barrier still brackets the region (no rank moves on early) but its own latency (a gloo
    round over the host, ~0.1 ms at 8 ranks against a 1.5 ms configs[1] region) is not work."""
    eng.sync()
    barrier(world)
    eng.sync()
    t0 = time.perf_counter()
    fn()
    eng.sync()
    t1 = time.perf_counter()
    barrier(world)
    rank_times = all_gather_float(t1 - t0, world)
    return max(rank_times), rank_times


def run_tabular(args, rank, world, local, wl, *, S=None, N=None, R=None, T=None, q_dtype=None, steps=20,
                warmup=5, cpu_seconds=10.0, schedule_to=0, eps_windows=(), window_steps=20):
    """One tabular workload (configs[1], [2] or [3]) on this rank: build the context, run `warmup`
    untimed then `steps` timed training episodes, and (rank 0) return its bench record; other ranks
    return None.  schedule_to > 0 (per-agent tables): the same context then continues the
    reference's epsilon schedule up to that episode (community.py:272-298), timing `window_steps`
    episodes from each start in eps_windows and the whole continuation (value_at_eps)."""
    from p2pmicrogrid_amd.dataset import SharedScenarioInputs, apply_asset_mix, asset_mix, scenario_batch
    t_setup = time.perf_counter()
    DeviceCommunityBatch = engine_class()
    S0, N0, R0, T0, qd0, shared, battery = WORKLOADS[wl]
    hetero = wl in HETERO
    S, N, T, q_dtype = S or S0, N or N0, T or T0, q_dtype or qd0
    R = R0 if R is None else R
    first = rank * S

    def build():
        mix = asset_mix(S, N, first_scenario=first, battery_j=BATTERY_J) if hetero else None
        gen = None
        if S * N * T >= PARALLEL_GEN_ELEMS and not os.environ.get("P2PMG_BENCH_TEST_ENGINE"):
            # configs[3]'s year of profiles (9.2 GB per GPU): generator blocks on the host cores, into shared memory
            # (at most 16 generator processes per rank: 8 ranks of a node stay within a few hundred)
            gen = SharedScenarioInputs(S, N, T, min(16, cpu_workers()[0]), first_scenario=first, mix=mix)
            inp = gen.inputs
        else:
            inp = scenario_batch(S, N, T, first_scenario=first)
            if hetero:
                inp = apply_asset_mix(inp, mix)
        tg = time.perf_counter() - t_setup
        try:
            e = DeviceCommunityBatch(S, N, R, T, q_dtype=q_dtype, device=local, scenario_offset=first, shared_q=shared)
            e.set_env(np.broadcast_to(inp.time, inp.t_out.shape), inp.t_out)
            e.set_profiles(inp.load_w, inp.pv_w)
            e.set_max_in(inp.max_in)
            e.set_temperatures(inp.t_in0, inp.t_m0)
        finally:
            del inp
            if gen is not None:
                gen.close()
        if mix is not None:
            e.set_hp_levels(mix.hp_levels)
            e.set_battery(mix.battery_capacity)
        elif battery:
            e.set_battery(BATTERY_J)
        return e, tg, gen is not None

    eng, t_gen, parallel_gen, err = None, 0.0, False, None
    try:
        eng, t_gen, parallel_gen = build()
    except Exception as e:  # noqa: BLE001  (agree_setup re-raises it on this rank, and on the others)
        err = e
    agree_setup(err, world)
    # episode metrics (+ the shared table's per-episode delta all-reduce, which needs RCCL)
    xk = exchange_kind(args, world)
    fallback = None
    if xk == "host":  # rehearsal: int64 deltas and metrics summed over gloo
        comm_err = "host-rehearsal exchange (no RCCL communicator)"
    else:
        comm_err = rccl_comm(eng, rank, world, required=shared and args.exchange == "rccl", world1=args.rccl_world1)
        if comm_err and shared:  # --exchange auto without a communicator: the labelled host exchange
            fallback, xk = comm_err, "host"
    record = ("reward", "cost")
    metrics = [None]

    def episode(e):
        if shared:  # agent.reset() at the end of train_episode fused into the launch, as below
            eng.run_episode("train", "philox", episode=e, epsilon=epsilon_at(e), record=record, reset_sigma=0.3,
                            next_epsilon=epsilon_at(e + 1))
            if world > 1 and xk == "host":
                from p2pmicrogrid_amd.distributed import all_reduce_int64
                eng.set_q_delta(all_reduce_int64(eng.get_q_delta(), world))
            elif world > 1 or (args.rccl_world1 and not comm_err):
                eng.allreduce_q_delta()
            eng.apply_q_delta()
        else:
            eng.run_episode("train", "philox", episode=e, epsilon=epsilon_at(e), record=record, reset_sigma=0.3,
                            next_epsilon=epsilon_at(e + 1))

    # per-agent tables: chained launches (p2pmg_run_episodes), each running the episodes up to the
    # next metric point back to back in every wave; same results as one launch per episode
    chain = not shared and args.chain == "auto"
    launch_eps = []  # episodes of every launch since the last reset_kernel_times (chained mode)
    launch_log = []  # [first episode, episodes] of every chained launch of this context (rocprof trace split)
    # the schedule as one array, sliced per chain (building the lists inside the timed region cost ~30 us)
    sched = np.array([epsilon_at(e) for e in range(max(schedule_to, warmup + steps) + 2 * MAX_CHAIN
                                                   + args.metric_every)])

    def first_chain(e0, e1):  # the episodes of the first launch of episodes(e0, e1)
        return min(e1, e0 + args.metric_every, e0 + MAX_CHAIN) - e0

    def episodes(e0, e1, metric=True, next_end=None):
        """Episodes [e0, e1) with the metric all-reduce every --metric-every episodes and after the
        last; next_end: where the caller's next episodes(e1, next_end) ends (the pre-pass guess).
        A timed call's last chain pre-passes at most its own length of the next call's episodes:
        its producer blocks share the CUs with it (configs[1]: 71.8 us per episode with the cap,
        73.2 us producing the continuation's 50 inside the 20-episode timed chain), and a short
        miss costs one step_prepass_kernel launch outside the timed call."""
        if not chain:
            for k, e in enumerate(range(e0, e1)):
                episode(e)
                if metric and ((k + 1) % args.metric_every == 0 or e + 1 == e1):
                    metrics[0] = episode_metrics(eng, world, comm_err)  # RCCL, the reference's 50-episode log
            return
        k0 = e0
        while k0 < e1:
            k1 = k0 + first_chain(k0, e1)
            if k1 < e1:
                n_next = first_chain(k1, e1)
            else:
                n_next = first_chain(e1, next_end) if next_end else k1 - k0
                n_next = min(n_next, k1 - k0) if metric else n_next
            eng.run_episodes(k0, sched[k0:k1], reset_sigma=0.3, record=record, next_epsilons=sched[k1:k1 + n_next])
            launch_eps.append(k1 - k0)
            launch_log.append([k0, k1 - k0])
            if metric:
                metrics[0] = episode_metrics(eng, world, comm_err)  # every chain ends at a metric point
            k0 = k1

    def kernel_ms_per_episode(kms):
        """HIP-event kernel time per episode: chained launches cover launch_eps[i] episodes each."""
        if not len(kms):
            return None
        if not chain:
            return float(np.mean(kms))
        return float(np.sum(kms)) / float(np.sum(launch_eps[-len(kms):]))

    eng.sync()
    t_upload = time.perf_counter() - t_setup - t_gen
    episodes(0, warmup, metric=False, next_end=warmup + steps)
    if world > 1 and warmup > 0:  # the first collective on a communicator sets up its connections: not timed
        episode_metrics(eng, world, comm_err)
    eng.sync()
    eng.reset_kernel_times()
    launch_eps.clear()
    # HIP events on every launch cost ~4 us per configs[1] episode: sample every 5th launch (every
    # chained launch: one per metric period)
    timing_period = 5 if steps >= 20 and not chain else 1
    eng.set_timing_period(timing_period)
    nxt_end = min(schedule_to, warmup + steps + args.metric_every) if schedule_to > warmup + steps else None
    dt, rank_times = timed(eng, world, lambda: episodes(warmup, warmup + steps, next_end=nxt_end))
    kms = eng.kernel_times()
    kernel_ms_ep = kernel_ms_per_episode(kms)
    timed_launch_eps = list(launch_eps)  # the timed region's launches (the schedule's reuse the list)
    coll = collective_record(eng, world, steps, world1=args.rccl_world1 and not comm_err)
    ep_reward = metrics[0][0] / metrics[0][1]
    nranks = eng.comm_nranks() if not comm_err else 0
    if shared and xk == "host":  # every replica's fingerprint, gathered over gloo
        from p2pmicrogrid_amd.distributed import all_gather_concat
        hashes = all_gather_concat(eng.table_hash_allgather().astype(np.uint64), world)
    else:
        hashes = eng.table_hash_allgather() if shared else None  # every replica of the shared table
    steps_per_episode = S * N * T

    # the rest of the reference's schedule on the same context: epsilon windows + the whole continuation
    at_eps = None
    if schedule_to and not shared and schedule_to > warmup + steps:
        at_eps = {"episodes_total": schedule_to, "windows": []}
        cur = warmup + steps
        t_all = 0.0
        for w0 in sorted(w for w in eps_windows if cur <= w and w + window_steps <= schedule_to):
            dt_gap, _ = timed(eng, world, lambda: episodes(cur, w0, next_end=w0 + window_steps))
            eng.reset_kernel_times()
            launch_eps.clear()
            dt_w, _ = timed(eng, world, lambda: episodes(w0, w0 + window_steps, next_end=schedule_to))
            kw_ = eng.kernel_times()
            at_eps["windows"].append({
                "first_episode": w0, "episodes": window_steps, "epsilon": epsilon_at(w0),
                "epsilon_last": epsilon_at(w0 + window_steps - 1),
                "value": world * steps_per_episode * window_steps / dt_w, "ms_per_step": dt_w / window_steps * 1e3,
                "kernel_ms": kernel_ms_per_episode(kw_), "timed_launches": int(len(kw_))})
            t_all += dt_gap + dt_w
            cur = w0 + window_steps
        dt_tail, _ = timed(eng, world, lambda: episodes(cur, schedule_to))
        t_all += dt_tail
        n_cont = schedule_to - (warmup + steps)
        at_eps["continuation"] = {
            "first_episode": warmup + steps, "episodes": n_cont,
            "epsilon_range": [epsilon_at(warmup + steps), epsilon_at(schedule_to - 1)],
            "value": world * steps_per_episode * n_cont / t_all, "ms_per_step": t_all / n_cont * 1e3,
            "note": "wall time of every episode after the timed region up to the reference's max_episodes "
                    "(setup.py:30), metric all-reduce every --metric-every episodes, max over ranks"}
        at_eps["mean_episode_reward_last"] = metrics[0][0] / metrics[0][1]

    out = None
    if rank == 0:
        value = world * steps_per_episode * steps / dt
        q_bytes = 8 if q_dtype == "f64" else 4
        if shared:
            bpa = algorithmic_bytes_per_agent_step_shared(S * N, q_bytes, battery, outputs=len(record))
            workload = (f"configs[2]: {S} scenarios/GPU x {N} agents (R={R}, T={T}) with battery storage, one "
                        f"shared {q_dtype} Q-table, int64 delta all-reduce per episode, Philox exploration, "
                        f"train episodes")
        elif hetero:
            bpa = algorithmic_bytes_per_agent_step(R, q_bytes, outputs=len(record))
            workload = (f"configs[3]: {S} scenarios/GPU x {N} heterogeneous households (R={R}, T={T} = "
                        f"{T // 96} days; no-PV / heat-pump size / battery mixes), per-agent {q_dtype} Q-tables, "
                        f"Philox exploration, train episodes")
        else:
            bpa = algorithmic_bytes_per_agent_step(R, q_bytes, outputs=len(record))
            workload = (f"configs[1]: {S} scenarios/GPU x thesis community (N={N}, R={R}, T={T}), per-agent "
                        f"{q_dtype} Q-tables, Philox exploration, train episodes")
        kernel_ms = kernel_ms_ep if kernel_ms_ep is not None else float("nan")
        achieved = bpa * steps_per_episode / (kernel_ms * 1e-3) / 1e9
        tj = args.traffic_json if (args.traffic_json and wl == args.workload) else os.path.join(
            ROOT, "profiles", "pmc_traffic.json" if wl == "config2" else f"pmc_traffic_{wl}.json")
        traffic = load_traffic(tj, workload)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": dt / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 simulation, f64 Q-table" if q_dtype == "f64" else "f32",
            "data": "synthetic profiles with the reference dataset schema (seed 42)",
            "config": {"workload": workload, "scenarios_per_gpu": S, "agents_per_scenario": N,
                       "rounds": R, "negotiation_rounds": R + 1, "horizon": T, "q_dtype": q_dtype, "shared_q": shared,
                       "battery": battery, "agent_steps_per_step": world * steps_per_episode,
                       "parallelism": (f"scenario-sharded x{world}, shared-table delta all-reduce (RCCL)" if shared
                                       else f"scenario-sharded x{world} (replicas, no data-path collective)")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         # per episode: the PMC summary's chained figure, or its one-launch-per-episode one
                         "traffic": traffic_per_episode(traffic, chain),
                         "kernel": eng.last_kernel(),
                         "kernel_ms": kernel_ms,  # per episode (a chained launch runs several)
                         "kernel_ms_per_launch": float(np.mean(kms)) if len(kms) else None,
                         "episodes_per_launch": timed_launch_eps if chain else 1,
                         "algorithmic_bytes_per_agent_step": bpa,
                         "algorithmic_bytes_per_episode": bpa * steps_per_episode,
                         "algorithmic_bytes_per_launch": bpa * steps_per_episode * (
                             float(np.mean(timed_launch_eps)) if chain and timed_launch_eps else 1.0),
                         "timed_launches": int(len(kms)), "timing_period": timing_period},
            "mean_episode_reward": ep_reward,
            "epsilon_range": [epsilon_at(warmup), epsilon_at(warmup + steps - 1)],
            "launch": ({"mode": "chained (p2pmg_run_episodes)", "launches": launch_log} if chain
                       else {"mode": "one launch per episode"}),
            "rccl_nranks": nranks,
            "rank_times_s": rank_times,
            # outside the timed region: host input generation (parallel above PARALLEL_GEN_ELEMS) and the
            # context build + upload + zeroed tables
            "setup_s": {"inputs": t_gen, "context_and_upload": t_upload,
                        "input_generation": "parallel (dataset.SharedScenarioInputs)" if parallel_gen else "serial"},
        }
        if os.environ.get("P2PMG_BENCH_TEST_ENGINE"):
            out["test_engine"] = os.environ["P2PMG_BENCH_TEST_ENGINE"]
        if comm_err:
            out["rccl_error"] = comm_err
        if world > 1:
            out["exchange"] = "host-rehearsal" if xk == "host" else "rccl"
        if fallback:
            out["exchange_fallback"] = f"RCCL unavailable ({fallback}): int64 deltas summed over gloo"
        if coll and xk != "host":
            out["collective"] = coll
        if shared:
            out["table_replicas_identical"] = bool(np.all(hashes == hashes[0]))
            assert out["table_replicas_identical"], f"shared-table replicas differ across ranks: {hashes}"
        if traffic:
            out["roofline"]["traffic_source"] = traffic.get("source")
            if "calibration" in traffic:  # round 6: per-pattern counter factors, not a uniform x2
                out["roofline"]["traffic_calibration"] = traffic["calibration"]["source"]
        if not shared and q_dtype == "f64" and N <= 8:  # the fast kernel's sector-granular traffic model
            eps_mid = epsilon_at(warmup + steps // 2)
            sm = sector_model_per_agent_step(N, R, eps_mid, battery or hetero)
            sm["bytes_per_launch"] = sm["total"] * steps_per_episode
            out["roofline"]["sector_model"] = sm
        issue = issue_roofline(wl, kernel_ms, (S, N, R, T))
        if issue:
            out["roofline"]["issue"] = issue
        # What binds the kernel: achieved/peak/frac above stay the HBM roofline
        # (algorithmic bytes); "bound" names the limit the measurements point to and
        # "binding_frac" is the fraction against that limit.
        if not (shared or battery or hetero) and q_dtype == "f64" and N == 2 and R == 1:
            gather = gather_roofline(S * N, T, kernel_ms)
            if gather:
                out["roofline"]["gather_floor"] = gather
                out["roofline"]["bound"] = "latency"  # one wave per CU: the dependent row-gather chain
                out["roofline"]["binding_frac"] = gather["frac"]
        elif hetero and q_dtype == "f64" and N == 4 and R == 1:
            gather = gather_roofline(S * N, T, kernel_ms, stages=2, agents_per_wave=64, pool=400, rows=3,
                                     source="r04_ubench_gather.jsonl")
            if gather:  # two dependent gather round trips per step + the f64 battery rules on the chain
                out["roofline"]["gather_floor"] = gather
                out["roofline"]["bound"] = "latency"
                out["roofline"]["binding_frac"] = gather["frac"]
        elif shared and issue and issue["frac"] > 0.5:
            out["roofline"]["bound"] = "valu-issue"  # every SIMD busy: VALU instructions per agent-step
            out["roofline"]["binding_frac"] = issue["frac"]
        if at_eps:
            out["value_at_eps"] = at_eps
    eng.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu_seconds > 0:
        workers, rule = cpu_workers()
        cb = cpu_baseline_all_cores("cpu_baseline", dict(
            seconds=cpu_seconds, S=(64 if hetero else 256) if N <= 4 else 64, N=N, R=R, T=T, q_dtype=q_dtype,
            shared=shared, battery=battery, hetero=hetero, t_sample=960 if T > 960 else 0), workers)
        cb.update(os_cpu_count=os.cpu_count(), cores_rule=rule)
        if not (shared or battery or hetero):  # the per-object loop restates the tabular path only
            cb["per_object"] = cpu_baseline_per_object(min(cpu_seconds, 5.0), N=N, R=R, T=T)
        out["cpu_baseline"] = cb
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (default 1; under torchrun the launch's WORLD_SIZE)")
    ap.add_argument("--steps", type=int, default=50, help="timed episodes")
    ap.add_argument("--warmup", type=int, default=5, help="untimed episodes")
    ap.add_argument("--workload", default="config2", choices=sorted(WORKLOADS),
                    help="config2 = BASELINE configs[1] (default); config3 = configs[2] per-GPU slice; "
                         "config4 = configs[3]; config5 = configs[4] (DQN)")
    ap.add_argument("--scenarios", type=int, default=None, help="override scenarios per GPU")
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=None)
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--q-dtype", default=None, choices=["f64", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--metric-every", type=int, default=50,
                    help="episodes between RCCL all-reduces of the episode metrics (community.py:279)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exchange", default="auto", choices=["auto", "rccl", "host"],
                    help="data-path exchange over ranks: rccl (xGMI, default when every rank has its own GPU) or "
                         "host (gloo rehearsal; auto picks it only when the launcher maps ranks onto shared GPUs)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary for roofline.traffic (default profiles/pmc_traffic[_<workload>].json)")
    ap.add_argument("--schedule-episodes", type=int, default=None,
                    help="per-agent tables: continue the same context through the reference's epsilon schedule up "
                         f"to this episode and time it (value_at_eps; default {REFERENCE_EPISODES} for config2, "
                         "0 = off)")
    ap.add_argument("--eps-windows", default="500,960",
                    help="first episodes of the timed windows inside the schedule continuation")
    ap.add_argument("--eps-window-steps", type=int, default=20)
    ap.add_argument("--grad-segments", type=int, default=0,
                    help="config5: gradient segments of this rank (0 = one; > 1 takes the split fold -> exchange "
                         "-> Adam path even at world 1)")
    ap.add_argument("--agents-per-block", type=int, default=0, help="config5: agents per train workgroup (0 = auto)")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="at --gpus 1: a one-rank RCCL communicator, so the shared-state workloads run their "
                         "multi-GPU exchange path (delta all-reduce / gradient all-gather) on one GPU")
    ap.add_argument("--chain", default="auto", choices=["auto", "off"],
                    help="per-agent tables: chained launches (p2pmg_run_episodes, every wave running the "
                         "episodes up to the next metric point back to back) or one launch per episode")
    ap.add_argument("--secondary", default="auto", choices=["auto", "none", "config3"],
                    help="a second workload measured by the same ranks after the first (auto: configs[2], the "
                         "shared-table workload with the int64 delta all-reduce, after the default config2)")
    ap.add_argument("--secondary-scenarios", type=int, default=None)
    ap.add_argument("--secondary-agents", type=int, default=None)
    ap.add_argument("--secondary-horizon", type=int, default=None)
    ap.add_argument("--secondary-steps", type=int, default=10)
    ap.add_argument("--secondary-warmup", type=int, default=2)
    ap.add_argument("--secondary-cpu-seconds", type=float, default=5.0)
    ap.add_argument("--extra", default="auto",
                    help="further workloads measured by the same ranks after the secondary, comma-separated (auto: "
                         "config5,config4 = configs[4] DQN and configs[3] one-year mixes after the default config2; "
                         "'' = none)")
    ap.add_argument("--extra-scenarios", type=int, default=None, help="override the extras' scenarios per GPU")
    ap.add_argument("--extra-horizon", type=int, default=None, help="override the extras' horizon")
    ap.add_argument("--extra-steps", type=int, default=5)
    ap.add_argument("--extra-warmup", type=int, default=1)
    args = ap.parse_args()
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        args.gpus = args.gpus or 1
        if args.gpus > 1:
            return launch_ranks(sys.argv[1:], args.gpus)

    rank, world, local = dist_setup(args.gpus)
    args.gpus = world
    if args.workload == "config5":
        S, N, R, T, _, _, _ = WORKLOADS["config5"]
        R = R if args.rounds is None else args.rounds
        out = run_dqn(args, rank, world, local, args.scenarios or S, args.agents or N, R, args.horizon or T,
                      args.steps, args.warmup, args.cpu_seconds)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return 0
    sched = args.schedule_episodes
    if sched is None:
        sched = REFERENCE_EPISODES if args.workload == "config2" else 0
    windows = [int(x) for x in args.eps_windows.split(",") if x.strip()]
    out = run_tabular(args, rank, world, local, args.workload, S=args.scenarios, N=args.agents, R=args.rounds,
                      T=args.horizon, q_dtype=args.q_dtype, steps=args.steps, warmup=args.warmup,
                      cpu_seconds=args.cpu_seconds, schedule_to=sched, eps_windows=windows,
                      window_steps=args.eps_window_steps)
    sec_wl = args.secondary
    if sec_wl == "auto":
        sec_wl = "config3" if args.workload == "config2" else "none"
    if sec_wl != "none" and sec_wl != args.workload:
        # SURVEY §8d judges the roofline on configs[2]; at world > 1 its per-episode int64 delta
        # all-reduce is the path's real exchange over xGMI, so the driver's scaling runs carry it too
        try:
            sec = run_tabular(args, rank, world, local, sec_wl, S=args.secondary_scenarios, N=args.secondary_agents,
                              T=args.secondary_horizon, steps=args.secondary_steps, warmup=args.secondary_warmup,
                              cpu_seconds=args.secondary_cpu_seconds)
        except Exception as e:  # noqa: BLE001  (the primary line stands; the failure is reported in it)
            print(f"bench.py: secondary workload {sec_wl} failed on rank {rank}: {type(e).__name__}: {e}",
                  file=sys.stderr, flush=True)
            sec = {"error": f"{type(e).__name__}: {e}", "workload": sec_wl}
        if rank == 0:
            for k in ("metric", "higher_is_better", "scaling", "vs_baseline", "n_gpus"):
                sec.pop(k, None)
            out["secondary"] = sec
    # the other BASELINE configs on the same ranks, after the primary line's (auto: behind the default
    # configs[1] + configs[2]): configs[4] (DQN, the gradient-segment all-gather over xGMI at world > 1)
    # and configs[3] (one-year heterogeneous episodes)
    extra = args.extra
    if extra == "auto":
        extra = "config5,config4" if args.workload == "config2" else ""
    for wl in [x.strip() for x in extra.split(",") if x.strip() and x.strip() != args.workload]:
        key = {"config5": "secondary_dqn", "config4": "secondary_year"}.get(wl, f"secondary_{wl}")
        try:
            if wl == "config5":
                S5, N5, R5, T5, _, _, _ = WORKLOADS["config5"]
                rec = run_dqn(args, rank, world, local, args.extra_scenarios or S5, N5, R5, args.extra_horizon or T5,
                              args.extra_steps, args.extra_warmup, args.secondary_cpu_seconds)
            else:
                rec = run_tabular(args, rank, world, local, wl, S=args.extra_scenarios, T=args.extra_horizon,
                                  steps=args.extra_steps, warmup=args.extra_warmup,
                                  cpu_seconds=args.secondary_cpu_seconds)
        except Exception as e:  # noqa: BLE001  (the primary line stands; the failure is reported in it)
            print(f"bench.py: extra workload {wl} failed on rank {rank}: {type(e).__name__}: {e}",
                  file=sys.stderr, flush=True)
            rec = {"error": f"{type(e).__name__}: {e}", "workload": wl}
        if rank == 0:
            for k in ("metric", "higher_is_better", "scaling", "vs_baseline", "n_gpus"):
                rec.pop(k, None)
            out[key] = rec
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
