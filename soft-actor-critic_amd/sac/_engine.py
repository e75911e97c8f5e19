"""ctypes binding of ``libsac_engine.so`` (C ABI: include/sac_engine.h).

PyTorch supplies device memory and streams; every compute call goes through the
HIP library.  There is deliberately no fallback: if the library or a GPU is
missing, ``load_library()`` / ``Engine(...)`` raise ``EngineUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch

MAX_LAYERS = 8
PREC_FP32, PREC_BF16 = 0, 1

_LIB_NAME = "libsac_engine.so"
_OPS_NAME = "libsac_torch_ops.so"
_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class EngineUnavailable(RuntimeError):
    """The HIP engine cannot run here (library not built or no MI355X device)."""


class EngineError(RuntimeError):
    pass


class HandoffTimeout(EngineError):
    """A workgroup hand-off inside a phase kernel gave up waiting: the affected
    gradient steps computed on stale inputs and the learner state is invalid."""


c_int32_p = ctypes.POINTER(ctypes.c_int32)


class EngineConfig(ctypes.Structure):
    _fields_ = [
        ("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32), ("batch", ctypes.c_int32),
        ("q_layers", ctypes.c_int32), ("q_dims", ctypes.c_int32 * (MAX_LAYERS + 1)),
        ("q_hidden_act", ctypes.c_int32), ("q_out_act", ctypes.c_int32),
        ("pi_layers", ctypes.c_int32), ("pi_dims", ctypes.c_int32 * (MAX_LAYERS + 1)),
        ("pi_hidden_act", ctypes.c_int32), ("pi_out_act", ctypes.c_int32),
        ("gamma", ctypes.c_float), ("tau", ctypes.c_float),
        ("log_std_min", ctypes.c_float), ("log_std_max", ctypes.c_float), ("action_scale", ctypes.c_float),
        ("actor_lr", ctypes.c_double), ("critic_lr", ctypes.c_double), ("alpha_lr", ctypes.c_double),
        ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("adam_eps", ctypes.c_float),
        ("auto_entropy", ctypes.c_int32), ("target_entropy", ctypes.c_float),
        ("precision", ctypes.c_int32), ("seed", ctypes.c_uint64),
        # kernel layout overrides (0 = the engine's choice; tests and A/B runs only)
        ("layout", ctypes.c_int32), ("stage_path", ctypes.c_int32), ("stage_batch", ctypes.c_int32),
        ("upd_parts", ctypes.c_int32), ("upd_threads", ctypes.c_int32),
    ]


# sac_engine_config.layout (include/sac_engine.h enum sac_layout)
LAYOUTS = {"auto": 0, "roles": 1, "rows": 2, "pairs": 3}
# the overrides a caller may pass to SacEngine(layout={...}), with their C field
LAYOUT_KEYS = ("layout", "stage_path", "stage_batch", "upd_parts", "upd_threads")


class EngineBuffers(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("pi", "q1", "q2", "q1t", "q2t", "pi_m", "pi_v", "q1_m", "q1_v", "q2_m", "q2_v",
                 "alpha_state", "opt_steps", "rng_step", "stats", "workspace")] + [
        ("workspace_bytes", ctypes.c_size_t)]


class ReplayDesc(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("act", ctypes.c_void_p), ("rew", ctypes.c_void_p),
                ("next_obs", ctypes.c_void_p), ("done", ctypes.c_void_p), ("capacity", ctypes.c_int64),
                ("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32), ("state", ctypes.c_void_p),
                ("row_stride", ctypes.c_int64)]


# name -> (restype, argtypes): every symbol include/sac_engine.h declares
SIGNATURES = {
    "sac_last_error": (ctypes.c_char_p, []),
    "sac_version": (ctypes.c_char_p, []),
    "sac_engine_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(EngineConfig)]),
    "sac_engine_create": (ctypes.c_int, [ctypes.POINTER(EngineConfig), ctypes.POINTER(EngineBuffers),
                                         ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "sac_engine_destroy": (None, [ctypes.c_void_p]),
    "sac_engine_sync_params": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "sac_engine_train": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ReplayDesc), ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "sac_engine_train_graph": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ReplayDesc), ctypes.c_int32,
                                              ctypes.c_int32, ctypes.c_void_p]),
    "sac_policy_act": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "sac_replay_push": (ctypes.c_int, [ctypes.POINTER(ReplayDesc), ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]),
    "sac_replay_gather": (ctypes.c_int, [ctypes.POINTER(ReplayDesc), ctypes.c_void_p, ctypes.c_int32]
                          + [ctypes.c_void_p] * 6),
    "sac_replay_sample_indices": (ctypes.c_int, [ctypes.POINTER(ReplayDesc), ctypes.c_int32, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "sac_replay_sample_gather": (ctypes.c_int, [ctypes.POINTER(ReplayDesc), ctypes.c_int32, ctypes.c_uint64,
                                                ctypes.c_uint64] + [ctypes.c_void_p] * 7),
    "sac_engine_read_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "sac_engine_clear_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "sac_engine_time_phases": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ReplayDesc), ctypes.c_int32,
                                              ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]),
    "sac_phase_kernel_name": (ctypes.c_char_p, [ctypes.c_int32]),
    "sac_engine_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "sac_engine_set_alpha_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
}

_lib: Optional[ctypes.CDLL] = None


def library_path() -> str:
    return os.environ.get("SAC_ENGINE_LIB", os.path.join(_PKG_ROOT, _LIB_NAME))


def load_library() -> ctypes.CDLL:
    """Load (once) and type every exported symbol.  Raises EngineUnavailable."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise EngineUnavailable(
            f"{path} not found: build it with `make -C soft-actor-critic_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


_ops_loaded = False


def ops_library_path() -> str:
    return os.path.join(os.path.dirname(library_path()), _OPS_NAME)


def ops():
    """``torch.ops.sac_hip``: the PyTorch custom ops over the C ABI
    (csrc/sac_torch_ops.cpp: replay_push, replay_gather, replay_sample,
    replay_sample_gather, train_step, train_graph, policy_act).  The op library
    dlopens the engine library ctypes loaded (bind_engine_library: the same file,
    so the same instance owns the engine handles).  Raises EngineUnavailable
    when it is not built."""
    global _ops_loaded
    if not _ops_loaded:
        load_library()
        path = ops_library_path()
        if not os.path.exists(path):
            raise EngineUnavailable(
                f"{path} not found: build it with `make -C soft-actor-critic_amd/csrc` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        torch.ops.load_library(path)
        torch.ops.sac_hip.bind_engine_library(os.path.abspath(library_path()))
        _ops_loaded = True
    return torch.ops.sac_hip


def check(rc: int) -> None:
    if rc != 0:
        msg = load_library().sac_last_error().decode()
        if rc == -3:
            raise ValueError(msg)
        raise EngineError(f"libsac_engine error {rc}: {msg}")


def require_gpu(device: torch.device) -> None:
    if device.type != "cuda":
        raise EngineUnavailable(
            f"the SAC engine runs on MI355X (HIP) devices only; got device '{device}'. "
            "Set train.device to 'cuda'.")
    if not torch.cuda.is_available():
        raise EngineUnavailable("no HIP device visible (torch.cuda.is_available() is False)")


def stream_handle(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def net_dims(layers: Sequence[torch.nn.Linear]):
    dims = [layers[0].in_features] + [lin.out_features for lin in layers]
    return len(layers), dims
