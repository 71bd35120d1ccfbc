"""ctypes binding of ``libimpala_hip.so`` (C-ABI declared in ``include/impala_hip.h``).

The shared library is built in-tree (``python -m impala_amd.build`` or
``__graft_entry__.build()``) and loaded from ``impala_amd/libimpala_hip.so``.  There is no
fallback: if the library is missing every compute entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IMPALA_HIP_LIB", os.path.join(_HERE, "libimpala_hip.so"))

IMPALA_DTYPE_F32 = 0
IMPALA_DTYPE_BF16 = 1
IMPALA_ALGO_IMPALA = 0
IMPALA_ALGO_PPO = 1
DP_ID_BYTES = 128  # IMPALA_DP_ID_BYTES (ncclUniqueId)
# V-trace gradient semantics (IMPALA_VTRACE_SG_*, include/impala_hip.h):
# what the backward treats as constant.  "sg_advantage" (the default, SURVEY §8(c)'s
# restatement): targets and pg advantages; "sg_targets": rlax's stop_target_gradients=True
# with the advantage learning.py:155 multiplies in left live; "sg_none":
# stop_target_gradients=False.
VTRACE_GRAD_MODES = {"sg_advantage": 0, "sg_targets": 1, "sg_none": 2}
DEFAULT_VTRACE_GRAD_MODE = "sg_advantage"


def vtrace_grad_mode(mode) -> int:
    """A mode name (VTRACE_GRAD_MODES) or its int -> the IMPALA_VTRACE_SG_* value."""
    if mode is None:
        mode = DEFAULT_VTRACE_GRAD_MODE
    if isinstance(mode, str):
        if mode not in VTRACE_GRAD_MODES:
            raise ValueError(f"vtrace grad mode {mode!r}: one of {sorted(VTRACE_GRAD_MODES)}")
        return VTRACE_GRAD_MODES[mode]
    if int(mode) not in VTRACE_GRAD_MODES.values():
        raise ValueError(f"vtrace grad mode {mode!r}: one of {sorted(VTRACE_GRAD_MODES.values())}")
    return int(mode)
ABI_VERSION = 3
NUM_METRICS = 9  # slots 0-6 METRIC_NAMES, 7 step, 8 PPO train/target
METRIC_NAMES = ("train/loss", "train/entropy", "train/td", "train/pg", "train/kl",
                "train/ratio", "train/grad_norm")
# PPOLearner metric keys (losses.py:147-155, agents/ppo/learning.py:136) -> metrics slot
PPO_METRIC_SLOTS = (("train/loss", 0), ("train/entropy", 1), ("train/td", 2), ("train/pg", 3),
                    ("train/target", 8), ("train/kl", 4), ("train/ratio", 5),
                    ("train_step/grad_norm", 6))

# every symbol declared in include/impala_hip.h
EXPORTS = (
    "impala_abi_version", "impala_last_error", "impala_config_default", "impala_param_count",
    "impala_create", "impala_destroy", "impala_bind_state", "impala_refresh_weights",
    "impala_set_step", "impala_set_metrics", "impala_set_metrics_host", "impala_forward",
    "impala_train_step", "impala_compute_grads",
    "impala_apply_update", "impala_compute_grads_part", "impala_grad_bucket_offset",
    "impala_grad_bucket_offset_fc",
    "impala_ppo_train_step", "impala_ppo_loss_head", "impala_vtrace", "impala_loss_head", "impala_kernel_count",
    "impala_kernel_name", "impala_timer_start", "impala_timer_read", "impala_gather_rows",
    "impala_gather_rows_hidx", "impala_train_step_rows",
    "impala_stage_init", "impala_stage", "impala_stage_rows", "impala_stage_rows_async",
    "impala_stage_wait",
    "impala_slot_batch",
    "impala_slot_release", "impala_act", "impala_set_debug_vtrace",
    "impala_timer_read_kernel", "impala_dp_unique_id", "impala_dp_init", "impala_dp_train_step",
    "impala_dp_nranks", "impala_step_clock", "impala_step_clock_end",
)
# every symbol declared in include/sac_hip.h
SAC_EXPORTS = (
    "sac_config_default", "sac_actor_param_count", "sac_critic_param_count", "sac_create",
    "sac_destroy", "sac_bind_state", "sac_refresh_weights", "sac_set_steps", "sac_train_step",
    "sac_act", "sac_policy", "sac_q_forward", "sac_phase_count", "sac_phase_name",
    "sac_timer_start", "sac_timer_read", "sac_sample",
)
SAC_NUM_METRICS = 12
# SACLearner metric keys (agents/sac/learning.py:206,220,243-265) -> metrics slot
SAC_CRITIC_METRICS = (("train/qf1_loss", 0), ("train/qf2_loss", 1), ("train/qf1", 2),
                      ("train/qf2", 3), ("train/qf_loss", 4), ("train/critic_grad_norm", 5))
SAC_ACTOR_METRICS = (("train/actor_loss", 6), ("train/actor_std", 7),
                     ("train/actor_grad_norm", 8))
SAC_ALPHA_METRICS = (("train/alpha_loss", 9), ("train/alpha", 10))


class ImpalaConfig(C.Structure):
    _fields_ = [
        ("batch_size", C.c_int), ("rollout_length", C.c_int), ("num_actions", C.c_int),
        ("dtype", C.c_int), ("lr", C.c_float), ("adam_beta1", C.c_float),
        ("adam_beta2", C.c_float), ("adam_eps", C.c_float), ("max_grad_norm", C.c_float),
        ("entropy_coeff", C.c_float), ("vtrace_lambda", C.c_float),
        ("clip_rho_threshold", C.c_float), ("clip_pg_rho_threshold", C.c_float),
        ("world_size", C.c_int), ("algo", C.c_int), ("ppo_clip", C.c_float),
        ("vtrace_grad_mode", C.c_int),
    ]


class ImpalaBatch(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("actions", C.c_void_p), ("rewards", C.c_void_p),
                ("discounts", C.c_void_p), ("behaviour_logits", C.c_void_p)]


class ImpalaRows(C.Structure):
    """impala_rows: per field, the address of an array of B row pointers (host memory)."""
    _fields_ = [("obs", C.c_void_p), ("actions", C.c_void_p), ("rewards", C.c_void_p),
                ("discounts", C.c_void_p), ("behaviour_logits", C.c_void_p)]


class ImpalaPpoBatch(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("actions", C.c_void_p), ("targets", C.c_void_p),
                ("behaviour_logits", C.c_void_p)]


class SacConfig(C.Structure):
    _fields_ = [
        ("obs_dim", C.c_int), ("act_dim", C.c_int), ("batch_size", C.c_int), ("dtype", C.c_int),
        ("critic_lr", C.c_float), ("actor_lr", C.c_float), ("adam_beta1", C.c_float),
        ("adam_beta2", C.c_float), ("adam_eps", C.c_float), ("max_grad_norm", C.c_float),
        ("tau", C.c_float), ("gamma", C.c_float), ("tune_alpha", C.c_int),
        ("target_entropy", C.c_float), ("prio_exponent", C.c_float), ("seed", C.c_uint64),
    ]


class SacBatch(C.Structure):
    _fields_ = [("s", C.c_void_p), ("a", C.c_void_p), ("r", C.c_void_p), ("s1", C.c_void_p),
                ("done", C.c_void_p), ("probabilities", C.c_void_p), ("noise", C.c_void_p),
                ("priorities", C.c_void_p)]


class SacState(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "actor", "actor_grad", "actor_m", "actor_v", "target_actor", "critic", "critic_grad",
        "critic_m", "critic_v", "target_critic", "log_alpha", "metrics")]


_lib = None
_lock = threading.Lock()
_P = C.c_void_p


def _declare(lib):
    lib.impala_abi_version.restype = C.c_int
    lib.impala_last_error.restype = C.c_char_p
    lib.impala_config_default.argtypes = [C.POINTER(ImpalaConfig)]
    lib.impala_param_count.argtypes = [C.c_int]
    lib.impala_param_count.restype = C.c_size_t
    lib.impala_create.argtypes = [C.POINTER(ImpalaConfig), C.c_int, C.POINTER(_P)]
    lib.impala_destroy.argtypes = [_P]
    lib.impala_bind_state.argtypes = [_P, _P, _P, _P, _P, _P, _P]
    lib.impala_refresh_weights.argtypes = [_P, _P]
    lib.impala_set_step.argtypes = [_P, C.c_int64, _P]
    lib.impala_set_debug_vtrace.argtypes = [_P, _P]
    lib.impala_set_metrics.argtypes = [_P, _P]
    lib.impala_set_metrics_host.argtypes = [_P, _P]
    lib.impala_train_step_rows.argtypes = [_P, C.POINTER(ImpalaBatch), _P, C.c_int, C.c_int64, _P]
    lib.impala_forward.argtypes = [_P, _P, C.c_int, _P, _P, _P]
    lib.impala_act.argtypes = [_P, _P, C.c_int, _P, C.c_int, C.c_uint64, C.c_uint64, _P, _P, _P,
                               _P]
    lib.impala_train_step.argtypes = [_P, C.POINTER(ImpalaBatch), _P]
    lib.impala_compute_grads.argtypes = [_P, C.POINTER(ImpalaBatch), _P]
    lib.impala_apply_update.argtypes = [_P, _P]
    lib.impala_ppo_train_step.argtypes = [_P, C.POINTER(ImpalaPpoBatch), _P]
    lib.impala_ppo_loss_head.argtypes = [_P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_float,
                                         C.c_float, _P, _P, _P, _P]
    lib.impala_compute_grads_part.argtypes = [_P, C.POINTER(ImpalaBatch), C.c_int, _P]
    lib.impala_grad_bucket_offset.argtypes = [_P]
    lib.impala_grad_bucket_offset.restype = C.c_size_t
    lib.impala_grad_bucket_offset_fc.argtypes = [_P]
    lib.impala_grad_bucket_offset_fc.restype = C.c_size_t
    lib.impala_dp_unique_id.argtypes = [_P]
    lib.impala_dp_init.argtypes = [_P, _P, C.c_int, C.c_int]
    lib.impala_dp_train_step.argtypes = [_P, C.POINTER(ImpalaBatch), C.c_int, _P]
    lib.impala_dp_nranks.argtypes = [_P, C.POINTER(C.c_int)]
    lib.impala_vtrace.argtypes = [_P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_float, C.c_float,
                                  C.c_float, _P, _P, _P, _P]
    lib.impala_loss_head.argtypes = [_P, _P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int,
                                     C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, _P, _P,
                                     _P, _P, _P, _P, _P, _P]
    lib.impala_gather_rows.argtypes = [C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_size_t),
                                       C.c_int, _P, C.c_int, _P]
    lib.impala_gather_rows_hidx.argtypes = [C.POINTER(_P), C.POINTER(_P),
                                            C.POINTER(C.c_size_t), C.c_int, _P, C.c_int, _P]
    lib.impala_stage_init.argtypes = [_P, C.c_int]
    lib.impala_stage.argtypes = [_P, C.POINTER(ImpalaBatch), C.c_int]
    lib.impala_stage_rows.argtypes = [_P, C.POINTER(ImpalaRows), C.c_int, C.c_int]
    lib.impala_stage_rows_async.argtypes = [_P, C.POINTER(ImpalaRows), C.c_int, C.c_int]
    lib.impala_stage_wait.argtypes = [_P, C.c_int]
    lib.impala_slot_batch.argtypes = [_P, C.c_int, _P, C.POINTER(ImpalaBatch)]
    lib.impala_slot_release.argtypes = [_P, C.c_int, _P]
    lib.impala_kernel_name.argtypes = [C.c_int]
    lib.impala_kernel_name.restype = C.c_char_p
    lib.impala_timer_start.argtypes = [_P, C.c_int, C.c_int]
    lib.impala_timer_read.argtypes = [_P, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    lib.impala_timer_read_kernel.argtypes = [_P, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    lib.impala_step_clock.argtypes = [_P, _P, C.c_int]
    lib.impala_step_clock_end.argtypes = [_P, _P, C.POINTER(C.c_int)]
    for name in EXPORTS:
        if name not in ("impala_last_error", "impala_param_count", "impala_kernel_name",
                        "impala_grad_bucket_offset", "impala_grad_bucket_offset_fc"):
            getattr(lib, name).restype = C.c_int
    lib.sac_config_default.argtypes = [C.POINTER(SacConfig)]
    lib.sac_actor_param_count.argtypes = [C.c_int, C.c_int]
    lib.sac_critic_param_count.argtypes = [C.c_int, C.c_int]
    lib.sac_create.argtypes = [C.POINTER(SacConfig), C.c_int, C.POINTER(_P)]
    lib.sac_destroy.argtypes = [_P]
    lib.sac_bind_state.argtypes = [_P, C.POINTER(SacState), _P]
    lib.sac_refresh_weights.argtypes = [_P, _P]
    lib.sac_set_steps.argtypes = [_P, C.c_int64, C.c_int64, C.c_int64, _P]
    lib.sac_train_step.argtypes = [_P, C.POINTER(SacBatch), _P]
    lib.sac_act.argtypes = [_P, _P, C.c_int, _P, C.c_float, C.c_float, C.c_float, _P, _P]
    lib.sac_policy.argtypes = [_P, _P, C.c_int, _P, _P, _P, _P, _P, _P, _P]
    lib.sac_q_forward.argtypes = [_P, _P, _P, C.c_int, C.c_int, _P, _P, _P]
    lib.sac_phase_name.argtypes = [C.c_int]
    lib.sac_phase_name.restype = C.c_char_p
    lib.sac_timer_start.argtypes = [_P, C.c_int, C.c_int]
    lib.sac_timer_read.argtypes = [_P, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    lib.sac_sample.argtypes = [C.c_uint64, C.c_uint64, C.c_int64, C.c_int, _P, _P,
                               C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_size_t), C.c_int, _P]
    for name in SAC_EXPORTS:
        if name in ("sac_actor_param_count", "sac_critic_param_count"):
            getattr(lib, name).restype = C.c_size_t
        elif name != "sac_phase_name":
            getattr(lib, name).restype = C.c_int


def lib():
    """Load (once) and return the HIP library; raise if it is not built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"HIP extension not built: {LIB_PATH} is missing "
                    "(run `python -m impala_amd.build`); there is no CPU fallback")
            handle = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            _declare(handle)
            if handle.impala_abi_version() != ABI_VERSION:
                raise RuntimeError(f"{LIB_PATH}: ABI version {handle.impala_abi_version()}, "
                                   f"expected {ABI_VERSION} (rebuild: python -m impala_amd.build)")
            _lib = handle
        return _lib


IMPALA_E_UNSUPPORTED = 1003


class Unsupported(RuntimeError):
    """IMPALA_E_UNSUPPORTED: the handle cannot run this entry point (its caller falls back)."""


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().impala_last_error().decode(errors="replace")
        cls = Unsupported if status == IMPALA_E_UNSUPPORTED else RuntimeError
        raise cls(f"{what or 'impala'} failed (status {status}): {msg}")


def ptr(t) -> int:
    """Device/host pointer of a torch tensor (0 for None)."""
    return 0 if t is None else int(t.data_ptr())


def stream_ptr(stream) -> int:
    """hipStream_t of a torch.cuda.Stream (torch's current stream when None)."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def param_count(num_actions: int = 15) -> int:
    return int(lib().impala_param_count(num_actions))


def default_config() -> ImpalaConfig:
    cfg = ImpalaConfig()
    check(lib().impala_config_default(C.byref(cfg)), "impala_config_default")
    return cfg
