"""ctypes binding to libp2pmg.so (include/p2pmg.h).

The HIP library is the only compute path: if it cannot be loaded this module raises —
there is no CPU fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

from . import _build

P2PMG_OK = 0
STATUS = {0: "OK", 1: "INVALID", 2: "HIP", 3: "NOMEM", 4: "STATE", 5: "UNSUPPORTED"}
Q_F64, Q_F32 = 0, 1
MODE_TRAIN, MODE_GREEDY, MODE_FILL = 0, 1, 2
LEARNER_TABULAR, LEARNER_DQN = 0, 1
DQN_ONLINE, DQN_TARGET, DQN_ADAM_M, DQN_ADAM_V = 0, 1, 2, 3
DQN_PARAMS = 4609
RNG_REPLAY, RNG_PHILOX = 0, 1
REC = {"reward": 1, "cost": 2, "grid": 4, "p2p": 8, "t_in": 16, "action": 32, "index": 64, "loss": 128}
GREEDY = 255

EXPORTS = [
    "p2pmg_abi_version", "p2pmg_config_default", "p2pmg_create", "p2pmg_destroy", "p2pmg_last_error", "p2pmg_last_kernel",
    "p2pmg_sync", "p2pmg_device_info", "p2pmg_set_env", "p2pmg_set_profiles", "p2pmg_set_agent_params",
    "p2pmg_set_temperatures", "p2pmg_get_temperatures", "p2pmg_reset_temperatures_philox",
    "p2pmg_set_replay_codes", "p2pmg_zero_q", "p2pmg_set_q", "p2pmg_get_q", "p2pmg_run_episode",
    "p2pmg_get_record", "p2pmg_get_episode_reward", "p2pmg_last_kernel_ms", "p2pmg_rc_step",
    "p2pmg_state_indices", "p2pmg_replay_decode", "p2pmg_device_count", "p2pmg_kernel_times",
    "p2pmg_reset_kernel_times", "p2pmg_collective_ms", "p2pmg_set_timing_period", "p2pmg_q_calls", "p2pmg_set_hp_levels", "p2pmg_set_battery", "p2pmg_get_soc",
    "p2pmg_battery_seq", "p2pmg_apply_q_delta", "p2pmg_get_q_delta", "p2pmg_set_q_delta", "p2pmg_comm_unique_id", "p2pmg_comm_init",
    "p2pmg_allreduce_q_delta", "p2pmg_comm_destroy", "p2pmg_run_rule_episode", "p2pmg_set_hp_state",
    "p2pmg_get_hp_state",
    "p2pmg_dqn_config_default", "p2pmg_dqn_setup", "p2pmg_dqn_set_weights", "p2pmg_dqn_get_weights",
    "p2pmg_dqn_set_step", "p2pmg_dqn_get_step", "p2pmg_dqn_set_samples", "p2pmg_dqn_get_buffer",
    "p2pmg_dqn_set_buffer", "p2pmg_dqn_forward", "p2pmg_dqn_train_batch", "p2pmg_prepass_stats",
    "p2pmg_dqn_get_net_steps", "p2pmg_fdiv_check", "p2pmg_fdiv64_check", "p2pmg_comm_nranks",
    "p2pmg_allreduce_metrics", "p2pmg_table_hash_allgather", "p2pmg_dqn_set_exchange", "p2pmg_dqn_grad_layout",
    "p2pmg_run_episodes", "p2pmg_get_episode_rewards",
]


class Config(C.Structure):
    _fields_ = [
        ("n_scenarios", C.c_int32), ("n_agents", C.c_int32), ("rounds", C.c_int32), ("horizon", C.c_int32),
        ("q_dtype", C.c_int32), ("n_time_states", C.c_int32), ("n_temp_states", C.c_int32),
        ("n_balance_states", C.c_int32), ("n_p2p_states", C.c_int32), ("n_actions", C.c_int32),
        ("alpha", C.c_double), ("gamma", C.c_double), ("hp_levels", C.c_float * 4),
        ("setpoint", C.c_float), ("temp_margin", C.c_float), ("lower_bound", C.c_float), ("upper_bound", C.c_float),
        ("inv_ci", C.c_float), ("inv_cm", C.c_float), ("inv_ri", C.c_float), ("inv_re", C.c_float),
        ("inv_rvent", C.c_float), ("one_minus_frad", C.c_float), ("frad", C.c_float), ("solar_gain", C.c_float),
        ("hp_cop", C.c_float), ("seconds_per_minute", C.c_float), ("time_slot", C.c_float),
        ("minutes_per_hour", C.c_float), ("kilo", C.c_float), ("penalty_weight", C.c_float),
        ("seed", C.c_uint64), ("scenario_offset", C.c_int64), ("shared_q", C.c_int32), ("learner", C.c_int32),
    ]


class DqnConfig(C.Structure):
    _fields_ = [("gamma", C.c_double), ("tau", C.c_double), ("lr", C.c_double), ("beta1", C.c_double),
                ("beta2", C.c_double), ("adam_eps", C.c_double), ("clip", C.c_double), ("batch", C.c_int32),
                ("capacity", C.c_int32), ("agents_per_block", C.c_int32), ("grad_segments", C.c_int32)]


ABI_VERSION = 8  # include/p2pmg.h P2PMG_ABI_VERSION

# p2pmg_exchange_fn: int (*)(void* user, float* segments, int64_t floats_per_rank, int rank, int nranks)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_int64, C.c_int, C.c_int)


class EpisodeArgs(C.Structure):
    _fields_ = [("mode", C.c_int32), ("rng", C.c_int32), ("episode", C.c_int32), ("record", C.c_int32),
                ("epsilon", C.c_double), ("flags", C.c_int32), ("scen_per_wave", C.c_int32),
                ("reset_sigma", C.c_double), ("next_epsilon", C.c_double)]


FLAG_PHILOX_PREPASS, FLAG_PHILOX_INKERNEL, FLAG_GENERAL_KERNEL, FLAG_RESET_T0, FLAG_NEXT_EPSILON = 1, 2, 4, 8, 16
FLAG_TILE_KERNEL = 32


class P2PMGError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()
P = C.c_void_p


def _declare(lib):
    vp, i32, sz = C.c_void_p, C.c_int, C.c_size_t
    fp = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    sig = {
        "p2pmg_abi_version": ([], i32),
        "p2pmg_config_default": ([C.POINTER(Config)], i32),
        "p2pmg_create": ([C.POINTER(Config), i32, C.POINTER(vp)], i32),
        "p2pmg_destroy": ([vp], i32),
        "p2pmg_last_error": ([vp], C.c_char_p),
        "p2pmg_last_kernel": ([vp], C.c_char_p),
        "p2pmg_sync": ([vp], i32),
        "p2pmg_device_info": ([vp, C.c_char_p, sz, C.POINTER(sz)], i32),
        "p2pmg_set_env": ([vp, i32, fp, fp, fp, fp, fp], i32),
        "p2pmg_set_profiles": ([vp, fp, fp], i32),
        "p2pmg_set_agent_params": ([vp, fp], i32),
        "p2pmg_set_temperatures": ([vp, fp, fp], i32),
        "p2pmg_get_temperatures": ([vp, fp, fp], i32),
        "p2pmg_reset_temperatures_philox": ([vp, i32, C.c_double], i32),
        "p2pmg_set_replay_codes": ([vp, vp], i32),
        "p2pmg_zero_q": ([vp], i32),
        "p2pmg_set_q": ([vp, i32, i32, vp, i32], i32),
        "p2pmg_get_q": ([vp, i32, i32, vp, i32], i32),
        "p2pmg_run_episode": ([vp, C.POINTER(EpisodeArgs)], i32),
        "p2pmg_run_episodes": ([vp, C.POINTER(EpisodeArgs), i32, dp, i32, vp], i32),
        "p2pmg_get_episode_rewards": ([vp, i32, fp], i32),
        "p2pmg_get_record": ([vp, i32, vp], i32),
        "p2pmg_get_episode_reward": ([vp, fp], i32),
        "p2pmg_last_kernel_ms": ([vp, C.POINTER(C.c_float)], i32),
        "p2pmg_rc_step": ([vp, i32, fp, fp, fp, fp, fp, fp], i32),
        "p2pmg_state_indices": ([vp, i32, fp, vp], i32),
        "p2pmg_replay_decode": ([vp, sz, sz, vp, sz, vp, C.POINTER(sz)], i32),
        "p2pmg_device_count": ([C.POINTER(C.c_int)], i32),
        "p2pmg_kernel_times": ([vp, fp, i32, C.POINTER(C.c_int)], i32),
        "p2pmg_reset_kernel_times": ([vp], i32),
        "p2pmg_collective_ms": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_int)], i32),
        "p2pmg_set_timing_period": ([vp, i32], i32),
        "p2pmg_q_calls": ([vp, i32, vp, vp, vp, vp, vp, i32, vp, vp], i32),
        "p2pmg_set_hp_levels": ([vp, fp], i32),
        "p2pmg_run_rule_episode": ([vp, i32], i32),
        "p2pmg_set_hp_state": ([vp, fp], i32),
        "p2pmg_get_hp_state": ([vp, fp], i32),
        "p2pmg_set_battery": ([vp, vp, C.c_double, C.c_double, C.c_double, vp], i32),
        "p2pmg_get_soc": ([vp, vp], i32),
        "p2pmg_battery_seq": ([vp, i32, i32, vp, vp, vp, vp, vp, C.c_double, C.c_double, C.c_double], i32),
        "p2pmg_apply_q_delta": ([vp], i32),
        "p2pmg_get_q_delta": ([vp, vp], i32),
        "p2pmg_set_q_delta": ([vp, vp], i32),
        "p2pmg_comm_unique_id": ([vp], i32),
        "p2pmg_comm_init": ([vp, vp, i32, i32], i32),
        "p2pmg_allreduce_q_delta": ([vp], i32),
        "p2pmg_comm_destroy": ([vp], i32),
        "p2pmg_dqn_config_default": ([C.POINTER(DqnConfig)], i32),
        "p2pmg_dqn_setup": ([vp, C.POINTER(DqnConfig)], i32),
        "p2pmg_dqn_set_weights": ([vp, i32, i32, i32, vp], i32),
        "p2pmg_dqn_get_weights": ([vp, i32, i32, i32, vp], i32),
        "p2pmg_dqn_set_step": ([vp, C.c_int64], i32),
        "p2pmg_dqn_get_step": ([vp, C.POINTER(C.c_int64)], i32),
        "p2pmg_dqn_set_samples": ([vp, vp], i32),
        "p2pmg_dqn_get_buffer": ([vp, i32, i32, vp, vp], i32),
        "p2pmg_dqn_set_buffer": ([vp, i32, i32, vp, vp], i32),
        "p2pmg_dqn_forward": ([vp, i32, i32, vp, vp], i32),
        "p2pmg_dqn_train_batch": ([vp, i32, vp, vp], i32),
        "p2pmg_prepass_stats": ([vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)], i32),
        "p2pmg_dqn_get_net_steps": ([vp, i32, i32, vp], i32),
        "p2pmg_fdiv_check": ([vp, i32, vp, vp, vp], i32),
        "p2pmg_fdiv64_check": ([vp, i32, vp, vp, vp], i32),
        "p2pmg_comm_nranks": ([vp, C.POINTER(C.c_int)], i32),
        "p2pmg_allreduce_metrics": ([vp, vp], i32),
        "p2pmg_table_hash_allgather": ([vp, vp], i32),
        "p2pmg_dqn_set_exchange": ([vp, EXCHANGE_FN, vp, i32, i32], i32),
        "p2pmg_dqn_grad_layout": ([vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res


def lib() -> C.CDLL:
    """Load (building in-tree first if the sources are newer and hipcc exists)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("P2PMG_LIB") or _build.LIB
        if path == _build.LIB and _build.needs_build():
            hipcc = _build.hipcc()
            if os.path.exists(hipcc) or hipcc == "hipcc":
                try:
                    _build.build(verbose=False)
                except Exception as e:  # noqa: BLE001
                    if not os.path.exists(path):
                        raise P2PMGError(f"libp2pmg.so missing and build failed: {e}") from e
        if not os.path.exists(path):
            raise P2PMGError(f"libp2pmg.so not found at {path}; run `python -m p2pmicrogrid_amd._build`")
        _lib = C.CDLL(path)
        _declare(_lib)
        if _lib.p2pmg_abi_version() != ABI_VERSION:
            raise P2PMGError("libp2pmg ABI version mismatch")
        return _lib


def check(status: int, ctx=None, what: str = ""):
    if status != P2PMG_OK:
        msg = ""
        if ctx is not None:
            raw = lib().p2pmg_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise P2PMGError(f"{what}: {STATUS.get(status, status)} {msg}".strip())


def default_config() -> Config:
    cfg = Config()
    check(lib().p2pmg_config_default(C.byref(cfg)), what="config_default")
    return cfg


def device_count() -> int:
    n = C.c_int(0)
    check(lib().p2pmg_device_count(C.byref(n)), what="device_count")
    return int(n.value)


def gpu_available() -> bool:
    """True if a HIP device is visible (asked through libp2pmg itself, not torch)."""
    try:
        return device_count() > 0
    except Exception:  # noqa: BLE001
        return False
