"""ctypes binding of the C ABI in ``include/drsa_amd.h`` (``lib/libdrsa_amd.so``).

This is the only door between the Python host layer and the HIP kernels.  There is
no CPU fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DRSA_AMD_LIB") or os.path.join(_HERE, "lib", "libdrsa_amd.so")

_lib: Optional[C.CDLL] = None

_vp, _fp, _ip = C.c_void_p, C.c_void_p, C.c_void_p
_i64, _i32, _sz, _f32, _f64 = C.c_int64, C.c_int, C.c_size_t, C.c_float, C.c_double

# name -> (restype, argtypes)
SIGNATURES = {
    "drsa_amd_last_error": (C.c_char_p, []),
    "drsa_amd_version": (_i32, []),
    "drsa_amd_drsa_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "drsa_amd_drsa_slab_floats": (_sz, [_i32, _i32]),
    "drsa_amd_drsa_partial": (_i32, [_fp, _fp, _i64, _i32, _i32, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_drsa_finish": (_i32, [_fp, _i64, _i32, _i32, _fp, _fp, _fp, _i32, _ip, _vp]),
    "drsa_amd_drsa_step": (_i32, [_fp, _fp, _i64, _i32, _i32, _fp, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_drsa_fused_supported": (_i32, [_i32, _i32]),
    "drsa_amd_drsa_fused_step": (_i32, [_fp, _fp, _i64, _i32, _i32, _fp, _i64, _fp, _fp, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_drsa_fused_step_counted": (_i32, [_fp, _fp, _i64, _i32, _i32, _fp, _i64, _fp, _fp, _fp, _ip, _fp, _vp,
                                                _sz, _vp]),
    "drsa_amd_drsa_finish_counted": (_i32, [_fp, _i64, _i32, _i32, _fp, _fp, _fp, _ip, _vp]),
    "drsa_amd_drsa_coop_status": (_i32, [_vp, _i64, _i32, _i32, _ip, _vp]),
    "drsa_amd_debug_coop_spin_budget": (_i32, [C.c_longlong]),
    "drsa_amd_drsa_objective": (_i32, [_fp, _fp, _i64, _i32, _i32, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_drsa_run": (_i32, [_fp, _fp, _i64, _i32, _i32, _fp, _fp, _i32, _fp, _ip, _vp, _sz, _i32, _vp]),
    "drsa_amd_drsa_run_multi": (_i32, [_i32, _vp, _i32, _i32, _vp]),
    "drsa_amd_drsa_run_batched": (_i32, [_i32, _vp, _i32, _i32, _i32, _vp]),
    "drsa_amd_drsa_partial_bf16": (_i32, [_vp, _vp, _i64, _i32, _i32, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_drsa_partial_f16": (_i32, [_vp, _vp, _i64, _i32, _i32, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_polar": (_i32, [_fp, _i32, _fp, _ip, _vp]),
    "drsa_amd_subspace_relevances_workspace_bytes": (_sz, [_i64, _i64, _i32, _i32]),
    "drsa_amd_subspace_relevances": (_i32, [_fp, _fp, _i64, _i64, _i32, _i32, _fp, _fp, _vp, _sz, _vp]),
    "drsa_amd_conv_weight_floats": (_sz, [_i32, _i32, _i32]),
    "drsa_amd_conv_fwd": (_i32, [_fp, _fp, _fp, _fp, _fp, _vp, _fp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "drsa_amd_conv_weight_bf16_elems": (_sz, [_i32, _i32, _i32]),
    "drsa_amd_conv_fwd_has_kernel": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32]),
    "drsa_amd_conv_fwd_bf16": (_i32, [_fp, _vp, _fp, _fp, _fp, _vp, _fp, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                      _vp]),
    "drsa_amd_conv_bwd": (_i32, [_fp, _vp, _fp, _fp, _fp, _fp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                 _i32, _f32, _vp]),
    "drsa_amd_conv_bwd_bf16": (_i32, [_fp, _vp, _vp, _fp, _fp, _fp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                      _i32, _f32, _vp]),
    "drsa_amd_conv_fwd_den_ring": (_i32, [_fp, _fp, _fp, _fp, _fp, _vp, _fp, _i32, _i32, _i32, _i32, _i32, _vp]),
    "drsa_amd_conv_bwd_den_ring": (_i32, [_fp, _vp, _vp, _i32, _fp, _fp, _fp, _fp, _i32, _i32, _i32, _i32, _i32, _i32,
                                          _i32, _i32, _f32, _vp]),
    "drsa_amd_conv_bwd_den_map": (_i32, [_fp, _vp, _i32, _vp, _i32, _fp, _fp, _fp, _i32, _i32, _i32, _i32, _i32, _i32,
                                         _i32, _i32, _f32, _vp]),
    "drsa_amd_conv_bwd_has_kernel_pw": (_i32, [_i32, _i32, _i32, _i32, _i32]),
    "drsa_amd_conv_bwd_has_kernel_bf16_pw": (_i32, [_i32, _i32, _i32, _i32]),
    "drsa_amd_conv_bwd_bf16_pw": (_i32, [_fp, _vp, _i32, _vp, _fp, _fp, _fp, _i32, _i32, _i32, _i32, _i32, _i32,
                                         _i32, _i32, _f32, _vp]),
    "drsa_amd_conv_bwd_has_kernel_bf16": (_i32, [_i32, _i32, _i32, _i32, _i32]),
    "drsa_amd_linear_fwd": (_i32, [_fp, _fp, _fp, _fp, _fp, _i32, _i32, _i32, _vp]),
    "drsa_amd_linear_bwd": (_i32, [_fp, _ip, _i32, _fp, _i32, _i32, _f32, _fp, _fp, _i32, _fp, _i32, _f32, _fp,
                                   _i32, _i32, _i32, _vp]),
    "drsa_amd_projection_residual": (_i32, [_fp, _i32, _fp, _vp]),
    "drsa_amd_projection_fwd": (_i32, [_fp, _fp, _fp, _fp, _fp, _fp, _vp, _i32, _i32, _i32, _i32, _i32, _vp]),
    "drsa_amd_projection_bwd": (_i32, [_fp, _vp, _fp, _fp, _fp, _fp, _fp, _fp, _fp, _i32, _i32, _i32, _i32, _i32,
                                       _f32, _f32, _i32, _vp]),
    "drsa_amd_ab_split": (_i32, [_fp, _fp, _fp, _fp, _fp, _i32, _i32, _i64, _f32, _vp]),
    "drsa_amd_ab_combine": (_i32, [_fp, _fp, _f32, _f32, _fp, _fp, _fp, _i32, _i32, _i64, _i32, _f32, _vp]),
    "drsa_amd_first_layer_bwd": (_i32, [_fp, _vp, _fp, _fp, _i32, _i32, _i32, _i32, _i32, _vp]),
    "drsa_amd_first_layer_den": (_i32, [_fp, _fp, _fp, _i32, _i32, _i32, _i32, _vp]),
    "drsa_amd_heatmap_sort": (_i32, [_fp, _i32, _i32, _i32, _i32, _fp, _fp, _fp, _fp, _vp, _vp]),
    "drsa_amd_maxpool_capture": (_i32, [_fp, _fp, _fp, _vp, _fp, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "drsa_amd_relevance_unpool": (_i32, [_fp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _fp, _vp]),
    "drsa_amd_drsa_vectors": (_i32, [_fp, _fp, _vp, _ip, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _fp, _fp,
                                     _vp]),
    "drsa_amd_normalize_workspace_bytes": (_sz, []),
    "drsa_amd_normalize_vectors": (_i32, [_fp, _i64, _i32, _fp, _vp, _sz, _vp]),
    "drsa_amd_normalize_sumsq": (_i32, [_fp, _i64, _vp, _sz, _fp, _vp]),
    "drsa_amd_normalize_scale": (_i32, [_fp, _i64, _i32, _fp, _i32, _i64, _fp, _vp]),
    "drsa_amd_logmel_smem_bytes": (_i32, [_i32, _i32, _i32, _i32, _i32]),
    "drsa_amd_logmel": (_i32, [_fp, _i64, _i64, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _fp, _ip, _ip, _ip,
                               _fp, _i32, _i32, _i32, _f32, _f32, _fp, _vp]),
}

class DrsaProblem(C.Structure):
    """drsa_amd_problem_t (include/drsa_amd.h)."""
    _fields_ = [("A", _vp), ("C", _vp), ("N", _i64), ("d", _i32), ("K", _i32), ("U_io", _vp), ("U_tmp", _vp),
                ("f_traj", _vp), ("counter", _vp), ("ws", _vp), ("ws_size", _sz), ("dtype", _i32)]


# status codes (include/drsa_amd.h)
DRSA_OK, DRSA_EINVAL, DRSA_EWORKSPACE, DRSA_EUNSUPPORTED, DRSA_ETIMEOUT = 0, -1, -2, -3, -4

XM_NONE, XM_MUL, XM_SPLIT = 0, 1, 2
POST_NONE, POST_DIV, POST_MASK, POST_DIV_RING = 0, 1, 2, 3
POST_DIV_MAP = 4   # host-side plan tag only: POST_DIV on an input-independent map (drsa_amd_conv_bwd_den_map)


class DrsaAmdError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the HIP library (idempotent).  Raises if it is missing — never falls back."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DrsaAmdError(
            f"drsa_amd HIP library not found at {path}; build it with "
            f"`python -m drsa_audio_amd.build` (hipcc, gfx950). There is no CPU fallback.")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib() -> C.CDLL:
    return _lib if _lib is not None else load()


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().drsa_amd_last_error().decode(errors="replace")
        raise DrsaAmdError(f"{what or 'drsa_amd'} failed (rc={rc}): {msg}")


def require_gpu(t: torch.Tensor, name: str, dtype=torch.float32) -> None:
    if not isinstance(t, torch.Tensor):
        raise DrsaAmdError(f"{name}: expected a torch.Tensor on the GPU, got {type(t).__name__}")
    if not t.is_cuda:
        raise DrsaAmdError(f"{name}: tensor must live on the GPU (HIP device); got {t.device}. "
                           "drsa_audio_amd has no CPU path.")
    if dtype is not None and t.dtype != dtype:
        raise DrsaAmdError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise DrsaAmdError(f"{name}: tensor must be contiguous")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream_ptr(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args) -> None:
    fn = getattr(lib(), name)
    check(fn(*args), name)
