"""ctypes binding of librx.so (include/rx.h).

torch is imported first on purpose: torch ships its own libamdhip64.so.7 and
librx.so links against the same SONAME, so loading librx after torch makes
both share ONE HIP runtime (streams and device pointers are then
interchangeable).  There is no CPU fallback: if the library is missing or the
device is absent, calls fail loudly.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede librx: shared HIP runtime, see above)

from . import _build

ABI_VERSION = 23
RX_EP_SHARDS = 64  # rx_io.ep_stats rows (include/rx.h)
RX_OK, RX_EINVAL, RX_EHIP, RX_ENOMEM, RX_ESTATE = 0, -1, -2, -3, -4
RX_F_CRASHED, RX_F_FINISHED, RX_F_CP25, RX_F_CP50, RX_F_CP75, RX_F_HAS_CRASHED = 1, 2, 4, 8, 16, 32
RX_EF_PENDING_RESET = 1
RX_AUTORESET_NEXT_STEP, RX_AUTORESET_SAME_STEP, RX_AUTORESET_DISABLED = 0, 1, 2
RX_INFO_W = 4
RX_INFO_SPEED, RX_INFO_PROGRESS, RX_INFO_PROGRESS_DELTA, RX_INFO_PLACEMENT = 0, 1, 2, 3

_P = ctypes.c_void_p

EXPORTS = ("rx_last_error", "rx_abi_version", "rx_create", "rx_destroy", "rx_sensor_angles", "rx_upload_tracks",
           "rx_assign", "rx_bind_state", "rx_set_speed_weight", "rx_reset", "rx_step", "rx_step_phases", "rx_gae",
           "rx_gae_scan", "rx_adam_workspace_floats", "rx_adam_clip_step", "rx_ppo_n_params", "rx_ppo_workspace_floats",
           "rx_ppo_workspace_doubles", "rx_ppo_adv_stats", "rx_ppo_minibatch_grad", "rx_policy_act",
           "rx_rollout_supported", "rx_rollout", "rx_ppo_adv_moments", "rx_ppo_adv_finalize", "rx_ppo_minibatch_grad_shard", "rx_ppo_kl_check", "rx_random_permutation",
           "rx_profile", "rx_profile_read", "rx_ppo_update_workspace_floats", "rx_ppo_minibatch_update", "rx_env_order",
           "rx_state_import", "rx_state_export", "rx_schedule",
           "rx_ppo_adv_workspace_doubles", "rx_ppo_adv_stats_ws", "rx_profile_waves", "rx_ray_waves", "rx_ray_tasks", "rx_set_start_draws",
           "rx_rollout_steps", "rx_selfplay_rollout_steps", "rx_steps")
RX_KERNEL_NAMES = ("k_dyn", "k_rays", "k_kin1", "k_step2", "k_step2_reward")
ADAM_MAX_TENSORS = 32
RX_PHASE_DYNAMICS, RX_PHASE_RAYS = 1, 2
RX_PREC_FP32, RX_PREC_BF16 = 0, 1
PRECISION = {"fp32": RX_PREC_FP32, "bf16": RX_PREC_BF16}


class RxConfig(ctypes.Structure):
    _fields_ = [("n_envs", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("n_sensors", ctypes.c_int32),
                ("max_steps", ctypes.c_int32), ("autoreset", ctypes.c_int32), ("device", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("sensor_half_cone", ctypes.c_double), ("speed_weight", ctypes.c_double),
                ("cull_chunk", ctypes.c_int32), ("sort_interval", ctypes.c_int32),
                ("ray_order", ctypes.c_int32), ("cull_super", ctypes.c_int32)] + \
               [(k, ctypes.c_int32) for k in ("split", "wide_n", "dyn_lpe", "ray_lpr", "reward_lpe", "argmin_window",
                                               "seg_filter", "box_quadrants", "ray_dispatch", "ray_tail",
                                               "ray_tail_lpr", "task_sort", "lane_tracks", "reserved0")]


# rx_config launch-schedule fields (ABI v17, v19, v20, v23): 0 = auto, -1 = off / none (include/rx.h).
# Scheduling only: every value gives bit-identical results.
SCHEDULE_W = 18  # rx_schedule: resolved schedule (include/rx.h)
SCHEDULE_KEYS = ("split", "wide", "dyn_lpe", "ray_lpr", "reward_lpe", "argmin_window", "seg_filter", "box_quadrants",
                 "dyn_waves", "ray_waves", "ray_dispatch", "ray_tail", "ray_tail_lpr", "ray_tail_from", "task_sort",
                 "lane_tracks", "dyn_calls", "reserved")
SCHED_FIELDS = ("split", "wide_n", "dyn_lpe", "ray_lpr", "reward_lpe", "argmin_window", "seg_filter", "box_quadrants",
                "ray_dispatch", "ray_tail", "ray_tail_lpr", "task_sort", "lane_tracks")


STATE_FIELDS = ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering", "finished_step", "flags",
                "steps", "track", "env_flags", "ep_return", "ep_length", "speed_weight")


class RxState(ctypes.Structure):
    _fields_ = [(k, _P) for k in STATE_FIELDS]


IO_FIELDS = ("actions", "obs", "reward", "reward64", "terminated", "truncated", "done_f32", "info", "ep_done",
             "ep_stats", "counters")


class RxIO(ctypes.Structure):
    _fields_ = [(k, _P) for k in IO_FIELDS]


# rx_steps (ABI v21): per-step element strides of the io rows
STRIDE_FIELDS = ("actions", "obs", "reward", "reward64", "terminated", "truncated", "done_f32", "info", "ep_done")


class RxIOStrides(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in STRIDE_FIELDS]


class RxAdamConfig(ctypes.Structure):
    _fields_ = [("n_tensors", ctypes.c_int32), ("offsets", ctypes.c_int64 * 33), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("eps", ctypes.c_double), ("max_grad_norm", ctypes.c_double)]


class RxPPOBatch(ctypes.Structure):
    _fields_ = [("obs_dim", ctypes.c_int32), ("mb", ctypes.c_int32), ("n_rows", ctypes.c_int64)] + \
               [(k, _P) for k in ("obs", "actions", "logprobs", "advantages", "returns", "values", "perm", "params",
                                  "log_std", "adv_stats")] + \
               [("clip_coef", ctypes.c_float), ("vf_coef", ctypes.c_float), ("kl_target", ctypes.c_float),
                ("precision", ctypes.c_int32)]


class RxRolloutIO(ctypes.Structure):
    _fields_ = [("T", ctypes.c_int32), ("obs_dim", ctypes.c_int32)] + \
               [(k, _P) for k in ("params", "log_std", "eps", "obs", "actions", "logprobs", "values", "rewards",
                                  "dones", "next_obs", "next_done")]


class RxPolicyIO(ctypes.Structure):
    _fields_ = [("obs_dim", ctypes.c_int32), ("n", ctypes.c_int64)] + \
               [(k, _P) for k in ("obs", "eps", "params", "log_std", "actions", "logprobs", "values")] + \
               [("obs_stride", ctypes.c_int64), ("act_stride", ctypes.c_int64), ("precision", ctypes.c_int32),
                ("actions2", _P), ("act2_stride", ctypes.c_int64)]


class RxSelfplayIO(ctypes.Structure):
    _fields_ = [(k, _P) for k in ("opp_params", "opp_log_std", "opp_eps", "env_actions", "env_obs", "env_reward",
                                  "sink")] + [("agent", ctypes.c_int32), ("opp_precision", ctypes.c_int32)]


class RxError(RuntimeError):
    pass


_lib = None


def lib_path():
    return _build.LIB


def load(build_if_missing=True):
    """Load librx.so (building it with hipcc if it is missing and allowed)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("RX_LIB_PATH") or _build.LIB  # override: profiling builds (tools/dyn_stamps.py)
    if not os.path.exists(path):
        if not build_if_missing:
            raise RxError(f"librx.so not built at {path} (run python -m rx._build)")
        _build.build()
    L = ctypes.CDLL(path)
    L.rx_last_error.restype = ctypes.c_char_p
    L.rx_abi_version.restype = ctypes.c_int
    L.rx_create.argtypes = [ctypes.POINTER(RxConfig), ctypes.POINTER(_P)]
    L.rx_destroy.argtypes = [_P]
    L.rx_sensor_angles.argtypes = [_P, _P]
    L.rx_upload_tracks.argtypes = [_P, ctypes.c_int32, _P, _P, _P, _P, _P]
    L.rx_assign.argtypes = [_P, _P]
    L.rx_bind_state.argtypes = [_P, ctypes.POINTER(RxState)]
    L.rx_set_speed_weight.argtypes = [_P, ctypes.c_double]
    L.rx_reset.argtypes = [_P, _P, ctypes.POINTER(RxIO), _P]
    L.rx_step.argtypes = [_P, ctypes.POINTER(RxIO), _P]
    L.rx_step_phases.argtypes = [_P, ctypes.POINTER(RxIO), ctypes.c_int32, _P]
    L.rx_steps.argtypes = [_P, ctypes.POINTER(RxIO), ctypes.c_int32, ctypes.POINTER(RxIOStrides), _P]
    gae_args = [ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, _P, ctypes.c_double, ctypes.c_double, _P, _P, _P]
    L.rx_gae.argtypes = gae_args
    L.rx_gae_scan.argtypes = gae_args
    L.rx_adam_workspace_floats.argtypes = [ctypes.POINTER(RxAdamConfig)]
    L.rx_adam_workspace_floats.restype = ctypes.c_size_t
    L.rx_adam_clip_step.argtypes = [ctypes.POINTER(RxAdamConfig), _P, _P, _P, _P, _P, _P, _P, _P, _P]
    L.rx_ppo_n_params.argtypes = [ctypes.c_int32]
    L.rx_ppo_workspace_floats.argtypes = [ctypes.c_int32, ctypes.c_int32]
    L.rx_ppo_workspace_floats.restype = ctypes.c_size_t
    L.rx_ppo_workspace_doubles.argtypes = [ctypes.c_int32]
    L.rx_ppo_workspace_doubles.restype = ctypes.c_size_t
    L.rx_ppo_adv_stats.argtypes = [ctypes.POINTER(RxPPOBatch), ctypes.c_int32, _P, _P]
    L.rx_ppo_minibatch_grad.argtypes = [ctypes.POINTER(RxPPOBatch), ctypes.c_int32, _P, _P, _P, _P, _P, _P]
    L.rx_policy_act.argtypes = [ctypes.POINTER(RxPolicyIO), _P]
    L.rx_rollout_supported.argtypes = [_P]
    L.rx_rollout.argtypes = [_P, ctypes.POINTER(RxIO), ctypes.POINTER(RxRolloutIO), _P]
    L.rx_rollout_steps.argtypes = [_P, ctypes.POINTER(RxIO), ctypes.POINTER(RxRolloutIO), ctypes.c_int32, _P]
    L.rx_selfplay_rollout_steps.argtypes = [_P, ctypes.POINTER(RxIO), ctypes.POINTER(RxRolloutIO),
                                            ctypes.POINTER(RxSelfplayIO), ctypes.c_int32, _P]
    L.rx_ppo_adv_moments.argtypes = [ctypes.POINTER(RxPPOBatch), ctypes.c_int32, _P, _P]
    L.rx_ppo_adv_finalize.argtypes = [_P, ctypes.c_int32, ctypes.c_int64, _P, _P]
    L.rx_ppo_minibatch_grad_shard.argtypes = [ctypes.POINTER(RxPPOBatch), ctypes.c_int32, ctypes.c_float, _P, _P, _P,
                                              _P, _P, _P]
    L.rx_ppo_kl_check.argtypes = [_P, ctypes.c_float, _P, _P, _P]
    L.rx_random_permutation.argtypes = [ctypes.c_int64, ctypes.c_uint64, _P, _P]
    L.rx_ppo_update_workspace_floats.argtypes = [ctypes.c_int32, ctypes.POINTER(RxAdamConfig)]
    L.rx_ppo_update_workspace_floats.restype = ctypes.c_size_t
    L.rx_ppo_minibatch_update.argtypes = [ctypes.POINTER(RxPPOBatch), ctypes.c_int32, ctypes.POINTER(RxAdamConfig)] + \
        [_P] * 12
    L.rx_env_order.argtypes = [_P, _P, _P, _P]
    L.rx_state_import.argtypes = [_P, _P]
    L.rx_state_export.argtypes = [_P, _P]
    L.rx_schedule.argtypes = [_P, _P]
    L.rx_ppo_adv_workspace_doubles.argtypes = [ctypes.c_int32, ctypes.c_int32]
    L.rx_ppo_adv_workspace_doubles.restype = ctypes.c_size_t
    L.rx_ppo_adv_stats_ws.argtypes = [ctypes.POINTER(RxPPOBatch), ctypes.c_int32, _P, _P, _P, _P]
    L.rx_profile.argtypes = [_P, ctypes.c_int32]
    L.rx_profile_read.argtypes = [_P, _P, _P]
    L.rx_profile_waves.argtypes = [_P, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P, _P]
    L.rx_ray_waves.argtypes = [_P, _P, ctypes.c_int32, _P]
    L.rx_ray_tasks.argtypes = [_P, _P, ctypes.c_int64, _P, _P]
    L.rx_set_start_draws.argtypes = [_P, _P, ctypes.c_int64, _P]
    for name in EXPORTS:
        if name not in ("rx_last_error", "rx_abi_version", "rx_ppo_workspace_floats", "rx_ppo_workspace_doubles",
                        "rx_ppo_update_workspace_floats", "rx_adam_workspace_floats",
                        "rx_ppo_adv_workspace_doubles"):
            getattr(L, name).restype = ctypes.c_int
    if L.rx_abi_version() != ABI_VERSION:
        raise RxError(f"librx ABI {L.rx_abi_version()} != {ABI_VERSION} (rebuild: python -m rx._build)")
    _lib = L
    return L


def check(rc, what=""):
    if rc != RX_OK:
        msg = _lib.rx_last_error().decode() if _lib is not None else "?"
        raise RxError(f"{what} failed (rc={rc}): {msg}")


def ptr(t):
    """Raw device (or host) pointer of a tensor / ndarray, None for None."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        assert t.is_contiguous(), "tensors handed to librx must be contiguous"
        return _P(t.data_ptr())
    return _P(t.ctypes.data)


def view_ptr(t):
    """Pointer of a strided view whose row stride the caller passes explicitly."""
    return _P(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return _P(s.cuda_stream)
