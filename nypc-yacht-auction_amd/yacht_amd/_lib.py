"""ctypes binding of libyacht_hip.so (include/yacht_hip.h).

The product path has no CPU fallback: if the HIP library is missing, or a call fails, an
exception is raised.  Device buffers are passed as raw pointers (torch tensors'
``data_ptr()``); streams as ``hipStream_t`` integers.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
# YK_LIB_PATH: diagnostic builds only (tools/diag_select.py); the product loads the in-tree library
LIB_PATH = os.environ.get("YK_LIB_PATH") or os.path.join(HERE, "libyacht_hip.so")

YK_OK, YK_ERR_ARG, YK_ERR_HIP, YK_ERR_NOMEM, YK_ERR_CAPACITY, YK_ERR_STATE = 0, -1, -2, -3, -4, -5
YK_ERR_RANGE = -6
_ERR_NAMES = {YK_ERR_ARG: "bad argument", YK_ERR_HIP: "HIP error", YK_ERR_NOMEM: "out of device memory",
              YK_ERR_CAPACITY: "engine capacity exceeded", YK_ERR_STATE: "engine state error",
              YK_ERR_RANGE: "a weight outside the fp16 split's range (|w| >= 65520)"}
YK_NET_ERR_SYNC = 1  # yk_net_errors: a value-head wave timed out on the v_head.2 hand-off

# per-element yk_step status -> the reference's exception (YachtGame.py:268-269, 306-307, 372, 508)
ST_OK, ST_VALUE_BID, ST_VALUE_SCORE, ST_RUNTIME, ST_ASSERT, ST_CAPACITY = 0, 1, 2, 3, 4, 5


class YkError(RuntimeError):
    def __init__(self, fn, code):
        hip = _lib.yk_last_hip_error() if _lib is not None else 0
        super().__init__(f"{fn} failed: {_ERR_NAMES.get(code, code)} (code {code}, hip error {hip})")
        self.code = code


class YkEngineConfig(C.Structure):
    _fields_ = [("n_envs", C.c_int), ("sims", C.c_int), ("cpuct", C.c_double), ("temp_threshold", C.c_int),
                ("max_moves", C.c_int), ("prior", C.c_int), ("record_predictions", C.c_int),
                ("max_expansions", C.c_int), ("arena_entries", C.c_int64), ("record_stride", C.c_int),
                ("groups", C.c_int), ("dual_trees", C.c_int)]


# name -> argtypes (restype int unless listed in _RESTYPE)
P = C.c_void_p
I = C.c_int
U64 = C.c_uint64
U32 = C.c_uint32
SIGNATURES = {
    "yk_version": [],
    "yk_last_hip_error": [],
    "yk_rng_draw64": [U64, U32, U64],
    "yk_init_board": [P, P, P, U64, I, P],
    "yk_step": [P, P, P, U64, P, P, P, P, P, I, P],
    "yk_valid_mask": [P, P, P, P, I, P],
    "yk_ended": [P, P, P, P, I, P],
    "yk_canonical": [P, P, P, I, P],
    "yk_score_table": [P, P, P, I, P],
    "yk_score_dice": [P, P, I, P],
    "yk_featurize": [P, P, I, P],
    "yk_key_hash": [P, P, I, P],
    "yk_hash_prior": [P, P, P, I, P],
    "yk_net_create": [C.POINTER(P), I, I, C.POINTER(P), I],
    "yk_net_predict": [P, P, P, P, I, P],
    "yk_net_predict_features": [P, P, P, P, I, P],
    "yk_net_leaf_prior": [P, P, P, P, I, P],
    "yk_net_policy_action": [P, P, P, P, I, P],
    "yk_net_destroy": [P],
    "yk_net_set_precision": [P, I],
    "yk_net_errors": [P, P],
    "yk_engine_create": [C.POINTER(P), C.POINTER(YkEngineConfig), P],
    "yk_engine_destroy": [P],
    "yk_selfplay": [P, U64, U32, P],
    "yk_arena": [P, U64, U32, P, I, I, P],
    "yk_greedy_action": [P, P, I, P],
    "yk_trainer_create": [P, I, I, P, I, P],
    "yk_trainer_destroy": [P],
    "yk_trainer_buffers": [P, P, P, P],
    "yk_trainer_backward": [P, P, P, P, P, I, P],
    "yk_trainer_apply": [P, P],
    "yk_trainer_step": [P, P, P, P, P, I, P],
    "yk_trainer_losses": [P, P],
    "yk_trainer_epoch_loss_begin": [P, C.c_double],
    "yk_trainer_epoch_loss_end": [P, P],
    "yk_trainer_get": [P, I, P],
    "yk_trainer_set": [P, I, P, C.c_int64],
    "yk_trainer_step_count": [P],
    "yk_trainer_set_row_offset": [P, C.c_int64],
    "yk_trainer_amp_state": [P, P],
    "yk_arena_results": [P, P, P, P, P, P, P],
    "yk_engine_set_opponent_net": [P, P],
    "yk_engine_stats": [P, P],
    "yk_engine_counters": [P, P, I],
    "yk_engine_profile": [P, I],
    "yk_engine_kernel_times": [P, P, P],
    "yk_engine_records": [P, P, P, P, P, P, P, P, P, P],
    "yk_engine_predictions": [P, P, P, P, P],
    "yk_engine_record_bytes": [P],
    "yk_engine_pack_records": [P, P, C.c_int64, P],
    "yk_mcts_search": [P, P, U64, P, P, I, P, P],
    "yk_mcts_reset": [P],
    "yk_examples_from_records": [P, I, I, I, I, C.c_int64, C.c_int64, C.c_int64, P, P, P, P, P],
    "yk_examples_policies": [P, I, I, I, I, C.c_int64, C.c_int64, C.c_int64, P, P, P, C.c_int64, P, P, P],
}
_RESTYPE = {"yk_version": C.c_char_p, "yk_rng_draw64": C.c_uint64, "yk_engine_record_bytes": C.c_int64,
            "yk_trainer_step_count": C.c_int64}

_NEWER = {"yk_engine_counters", "yk_net_errors"}  # added in rounds 5-6 (A/B baselines may predate them)
_lib = None


def build() -> str:
    """Compile libyacht_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-C", PKG_ROOT, "-j4"], check=True)
    return LIB_PATH


def lib():
    """Load the HIP library.  Fails loudly: there is no CPU fallback for the product path."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `make -C {PKG_ROOT}` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        lib_ = C.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            if os.environ.get("YK_LIB_PATH") and name in _NEWER and not hasattr(lib_, name):
                continue  # an older diagnostic baseline (A/B): entry points added since are absent
            fn = getattr(lib_, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, C.c_int)
        _lib = lib_
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != YK_OK:
        raise YkError(name, rc)
    return rc


def ptr(t) -> int:
    """device pointer of a torch tensor (must be on the GPU and contiguous)."""
    if not t.is_cuda:
        raise ValueError("yacht_amd kernels take device tensors")
    if not t.is_contiguous():
        raise ValueError("yacht_amd kernels take contiguous tensors")
    return t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
