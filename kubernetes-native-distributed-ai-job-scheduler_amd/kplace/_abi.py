"""ctypes mirror of include/kplace.h (the C-ABI of libkplace.so).

Only struct layouts, constants and the loader live here. The structs are the
same ones a Go maintainer would bind through cgo; keeping the
Python mirror field-for-field identical lets the tests drive the exact
boundary the Go caller would use.
"""
from __future__ import annotations

import ctypes as C
import os

KP_ABI_VERSION = 8
KP_MAX_DIMS = 8
KP_MAX_CAND = 32
KP_MAX_GANG = 64
KP_MAX_VALUE = 1 << 56

KP_OK = 0
KP_EINVAL = -1
KP_EHIP = -2
KP_ERCCL = -3
KP_ENOMEM = -4
KP_ESTATE = -5
KP_ENODEV = -6

KP_SCORE_MOST_ALLOCATED = 0
KP_SCORE_LEAST_ALLOCATED = 1
KP_TIE_NODE_INDEX = 0
KP_TIE_ROTATED = 1
KP_SCORE_INFEASIBLE = -1
KP_SCORE_NONE = -1
KP_JOB_PLACED = 0
KP_JOB_NO_FIT = 1
KP_JOB_ROUND_LIMIT = 2

_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_u64p = C.POINTER(C.c_uint64)


class Snapshot(C.Structure):
    _fields_ = [
        ("J", C.c_int32), ("N", C.c_int32), ("D", C.c_int32),
        ("req", _i64p), ("cap", _i64p), ("used", _i64p),
        ("prio", _i32p), ("gang_id", _i32p), ("gang_size", _i32p),
        ("topo_domain", _i32p), ("affinity", _i32p),
    ]


class Params(C.Structure):
    _fields_ = [
        ("w_dim", C.c_int32 * KP_MAX_DIMS),
        ("score_mode", C.c_int32),
        ("gpu_dim", C.c_int32),
        ("w_gpu_fit", C.c_int32),
        ("w_spread", C.c_int32),
        ("tie_mode", C.c_int32),
        ("tie_seed", C.c_uint32),
        ("max_rounds", C.c_int32),
        ("n_cand", C.c_int32),
        ("util_scale", C.c_int32),
        ("max_passes", C.c_int32),
        ("w_affinity", C.c_int32),
    ]


class Result(C.Structure):
    _fields_ = [
        ("node_of_job", _i32p), ("score_of_job", _i32p),
        ("status_of_job", _i32p), ("used_out", _i64p),
        ("rounds", C.c_int32), ("passes", C.c_int32), ("placed_jobs", C.c_int32),
        ("unplaced_jobs", C.c_int32), ("units", C.c_int32),
        ("pairs_scored", C.c_int64),
    ]


class Config(C.Structure):
    _fields_ = [
        ("device", C.c_int32), ("world_size", C.c_int32), ("rank", C.c_int32),
        ("nccl_id", C.c_void_p), ("max_pairs_matrix", C.c_int64),
    ]


class Preemption(C.Structure):
    _fields_ = [
        ("node_of_job", _i32p), ("victims_of_job", _i32p), ("cost_of_job", _i64p),
        ("preemptors", C.c_int32), ("nominated", C.c_int32), ("pairs_scored", C.c_int64),
    ]


class Timing(C.Structure):
    _fields_ = [
        ("solve_ms", C.c_double), ("score_ms", C.c_double),
        ("select_ms", C.c_double), ("accept_ms", C.c_double),
        ("score_launches", C.c_int64), ("score_bytes", C.c_int64),
        ("select_bytes", C.c_int64), ("fused", C.c_int32), ("score_form", C.c_int32),
        ("score_classes", C.c_int32), ("rccl_calls", C.c_int32),
        ("cand_ms", C.c_double), ("xchg_ms", C.c_double), ("pass_ms", C.c_double),
    ]


# Documented defaults; kp_params_default() in the library
# must return exactly these (tests/test_abi.py checks it).
DEFAULT_W_DIM = (1, 1, 4, 2, 1, 1, 1, 1)
DEFAULT_TIE_SEED = 0x6B706C61  # "kpla"
DEFAULT_W_AFFINITY = 512


def default_params(**over) -> Params:
    p = Params()
    for d in range(KP_MAX_DIMS):
        p.w_dim[d] = DEFAULT_W_DIM[d]
    p.score_mode = KP_SCORE_MOST_ALLOCATED
    p.gpu_dim = 2
    p.w_gpu_fit = 1024
    p.w_spread = 256
    p.tie_mode = KP_TIE_ROTATED
    p.tie_seed = DEFAULT_TIE_SEED
    p.max_rounds = 0
    p.n_cand = 16
    p.util_scale = 100
    p.max_passes = 16
    p.w_affinity = DEFAULT_W_AFFINITY
    for k, v in over.items():
        if k == "w_dim":
            for d, w in enumerate(v):
                p.w_dim[d] = w
        else:
            setattr(p, k, v)
    return p


def params_dict(p: Params) -> dict:
    return {
        "w_dim": list(p.w_dim), "score_mode": p.score_mode, "gpu_dim": p.gpu_dim,
        "w_gpu_fit": p.w_gpu_fit, "w_spread": p.w_spread, "tie_mode": p.tie_mode,
        "tie_seed": p.tie_seed, "max_rounds": p.max_rounds, "n_cand": p.n_cand,
        "util_scale": p.util_scale, "max_passes": p.max_passes, "w_affinity": p.w_affinity,
    }


PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# KPLACE_LIB: an alternative build of the same library (A/B timing runs only)
_DEFAULT_LIB = os.path.join(os.path.dirname(PKG_DIR), "libkplace.so")
LIB_PATH = os.environ.get("KPLACE_LIB") or _DEFAULT_LIB


# kp_allgather_fn: (user, send, bytes, recv) -> 0 on success
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


def load_library(path: str | None = None) -> C.CDLL:
    """Load libkplace.so and declare every exported signature.

    Fails loudly (OSError) when the library is missing: there is no CPU
    fallback for the product path.
    """
    lib = C.CDLL(path or LIB_PATH)
    vp = C.c_void_p
    sigs = {
        "kp_params_default": (None, [C.POINTER(Params)]),
        "kp_create": (C.c_int, [C.POINTER(vp), C.POINTER(Config)]),
        "kp_create_multi": (C.c_int, [C.POINTER(vp), _i32p, C.c_int32, C.POINTER(Config)]),
        "kp_last_error": (C.c_char_p, [vp]),
        "kp_last_error_r": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
        "kp_destroy": (None, [vp]),
        "kp_strerror": (C.c_char_p, [C.c_int]),
        "kp_abi_version": (C.c_int, []),
        "kp_dist_unique_id": (C.c_int, [vp]),
        "kp_place": (C.c_int, [vp, C.POINTER(Snapshot), C.POINTER(Params), C.POINTER(Result)]),
        "kp_load_nodes": (C.c_int, [vp, C.c_int32, C.c_int32, _i64p, _i64p, _i32p]),
        "kp_load_jobs": (C.c_int, [vp, C.c_int32, _i64p, _i32p, _i32p, _i32p, _i32p]),
        "kp_solve": (C.c_int, [vp, C.POINTER(Params), C.POINTER(Result)]),
        "kp_fetch": (C.c_int, [vp, C.POINTER(Result)]),
        "kp_apply_delta": (C.c_int, [vp, _i32p, _i64p, C.c_int32]),
        "kp_reset_nodes": (C.c_int, [vp]),
        "kp_score": (C.c_int, [vp, C.POINTER(Params), C.c_int32, C.c_int32, _i32p, _u64p]),
        "kp_score_dev": (C.c_int, [vp, C.POINTER(Params), C.c_int32, C.c_int32, vp, vp]),
        "kp_last_timing": (C.c_int, [vp, C.POINTER(Timing)]),
        "kp_last_timing_shards": (C.c_int, [vp, C.POINTER(Timing), C.c_int32]),
        "kp_set_profiling": (C.c_int, [vp, C.c_int]),
        "kp_set_allgather": (C.c_int, [vp, ALLGATHER_FN, vp]),
        "kp_parse_gpu_memory": (C.c_int, [C.c_char_p, _i64p]),
        "kp_load_running": (C.c_int, [vp, C.c_int32, _i32p, _i64p, _i32p]),
        "kp_preempt": (C.c_int, [vp, C.POINTER(Preemption)]),
    }
    for name, (res, args) in sigs.items():
        if (path or LIB_PATH) != _DEFAULT_LIB and not hasattr(lib, name):
            continue  # an explicitly named older build (A/B runs): entry points it lacks stay absent
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


# every symbol include/kplace.h declares (tests check the export table)
EXPORTED = (
    "kp_params_default", "kp_create", "kp_create_multi", "kp_destroy", "kp_strerror",
    "kp_last_error", "kp_last_error_r",
    "kp_abi_version", "kp_dist_unique_id", "kp_place", "kp_load_nodes",
    "kp_load_jobs", "kp_solve", "kp_fetch", "kp_apply_delta", "kp_reset_nodes", "kp_score",
    "kp_last_timing", "kp_last_timing_shards", "kp_set_profiling", "kp_parse_gpu_memory", "kp_load_running",
    "kp_preempt", "kp_set_allgather", "kp_score_dev",
)
