"""ctypes binding of the C-ABI library ``libvsrk.so`` (declared in include/vsrk.h).

This module is the only place Python touches the native boundary.  There is
no fallback: if the library is missing or a call fails, a RuntimeError is
raised (the product path never silently drops to a PyTorch/CPU op).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch

from . import build as _build

VSRK_F32 = 0
VSRK_BF16 = 1
VSRK_F16 = 2
PRO_NONE, PRO_RELU, PRO_AFFINE, PRO_AFFINE_RELU = 0, 1, 2, 3
ACT_NONE, ACT_RELU, ACT_PRELU = 0, 1, 2

_DTYPE = {torch.float32: VSRK_F32, torch.bfloat16: VSRK_BF16, torch.float16: VSRK_F16}


class Tensor5(C.Structure):
    _fields_ = [
        ("ptr", C.c_void_p),
        ("n", C.c_int32), ("d", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("c", C.c_int32),
        ("sn", C.c_int64), ("sd", C.c_int64), ("sh", C.c_int64), ("sw", C.c_int64),
        ("shuffle", C.c_int32),
        ("dtype", C.c_int32),
    ]


class ConvDesc(C.Structure):
    _fields_ = [
        ("kd", C.c_int32), ("kh", C.c_int32), ("kw", C.c_int32),
        ("pd", C.c_int32), ("ph", C.c_int32), ("pw", C.c_int32),
        ("prologue", C.c_int32),
        ("act", C.c_int32),
        ("out_scale", C.c_float),
        ("accumulate", C.c_int32),
        ("bias_perm_r", C.c_int32),
        ("act_param", C.c_void_p),
        ("mask_slope", C.c_void_p),
        ("subpixel", C.c_int32),
    ]


class BnContrib(C.Structure):
    """vsrk_bn_contrib (include/vsrk.h)."""
    _fields_ = [
        ("dz", Tensor5), ("d0", C.c_int32),
        ("scale", C.c_void_p), ("shift", C.c_void_p), ("mean", C.c_void_p), ("invstd", C.c_void_p),
        ("gamma", C.c_void_p), ("sum_dy", C.c_void_p), ("sum_dy_xhat", C.c_void_p),
        ("count", C.c_double),
    ]


class PackDesc(C.Structure):
    """vsrk_pack_desc (include/vsrk.h)."""
    _fields_ = [("w", C.c_void_p), ("packed", C.c_void_p),
                ("cout", C.c_int32), ("cin", C.c_int32), ("kd", C.c_int32), ("kh", C.c_int32), ("kw", C.c_int32),
                ("mode", C.c_int32), ("perm_r", C.c_int32), ("reserved", C.c_int32)]


# name -> (restype, argtypes)
_P = C.c_void_p
_T5 = C.POINTER(Tensor5)
_CD = C.POINTER(ConvDesc)
_SIGS = {
    "vsrk_conv_packed_elems": (C.c_size_t, [C.c_int32] * 6),
    "vsrk_conv_pack_weight": (C.c_int, [C.c_int32, _P] + [C.c_int32] * 7 + [_P, _P]),
    "vsrk_conv_pack_weights": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_int64, _P]),
    "vsrk_conv_fwd": (C.c_int, [_CD, _T5, _P, _P, _P, _P, _T5, _T5, _T5, _P]),
    "vsrk_conv_fwd_reduce_workspace": (C.c_size_t, [_CD, _T5]),
    "vsrk_conv_prelu_bwd_workspace": (C.c_size_t, []),
    "vsrk_slope_slot_doubles": (C.c_size_t, []),
    "vsrk_slope_final_sum": (C.c_int, [_P, C.c_int64, _P, _P, C.c_int32, C.c_int32, _P]),
    "vsrk_conv_fwd_prelu_bwd": (C.c_int, [_CD, _T5, _P, _P, _T5, _T5, C.c_int32, _P, C.c_int32, _P, C.c_size_t,
                                          _P]),
    "vsrk_conv_fwd_reduce": (C.c_int, [_CD, _T5, _P, _P, _P, _P, _T5, C.c_int32, _T5, _P, _P, _P, _P, _P, _P, _P,
                                       C.c_size_t, _P]),
    "vsrk_conv_fwd_reduce_bnb": (C.c_int, [_CD, _T5, C.POINTER(BnContrib), _T5, _P, _T5, _T5, _P, _P, _P, _P, _P,
                                           _P, _P, C.c_size_t, _P]),
    "vsrk_conv_wgrad_workspace_size": (C.c_size_t, [_CD, _T5, _T5]),
    "vsrk_conv_wgrad": (C.c_int, [_CD, _T5, _T5, _P, _P, C.c_float, C.c_int32, _P, _P, C.c_int32, _P,
                                  C.c_size_t, _P]),
    "vsrk_ncdhw_to_view": (C.c_int, [_P] + [C.c_int32] * 5 + [_T5, _P]),
    "vsrk_view_to_ncdhw": (C.c_int, [_T5, _P, C.c_int32, _P]),
    "vsrk_relu_bwd": (C.c_int, [_T5, _T5, _T5, _P]),
    "vsrk_add": (C.c_int, [_T5, _T5, _T5, _P]),
    "vsrk_loss_workspace_size": (C.c_size_t, [C.c_int64]),
    "vsrk_loss_fwd": (C.c_int, [C.c_int32, C.c_float, _P, _P, C.c_int64, _P, _P, C.c_size_t, _P]),
    "vsrk_loss_bwd": (C.c_int, [C.c_int32, C.c_float, _P, _P, C.c_int64, _P, _P, C.c_int32, _P]),
    "vsrk_psnr_workspace_size": (C.c_size_t, [C.c_int32, C.c_int64]),
    "vsrk_psnr": (C.c_int, [_P, _P, C.c_int32, C.c_int64, C.c_int32, C.c_float, C.c_float, C.c_float, _P, _P, _P,
                            C.c_size_t, _P]),
    "vsrk_bn_workspace_size": (C.c_size_t, [C.c_int32]),
    "vsrk_bn_stats": (C.c_int, [_T5, _P, _P, _P, C.c_size_t, _P]),
    "vsrk_bn_stats_grouped": (C.c_int, [_T5, C.c_int32, _P, _P, _P, C.c_size_t, _P]),
    "vsrk_peak_mfma_blocks": (C.c_int32, []),
    "vsrk_peak_mfma": (C.c_int, [C.c_int32, _P, _P]),
    "vsrk_peak_copy": (C.c_int, [_P, _P, C.c_int64, _P]),
    "vsrk_gather_windows": (C.c_int, [_P] + [C.c_int32] * 4 + [_P] + [C.c_int32] * 4 + [_P, _P]),
    "vsrk_dcn_im2col": (C.c_int, [_P] * 6),
    "vsrk_dcn_col2im": (C.c_int, [_P] * 6),
    "vsrk_dcn_coord_grad": (C.c_int, [_P] * 8),
    "vsrk_bn_finalize": (C.c_int, [_P, _P, C.c_double, _P, _P, C.c_float, C.c_float, _P, _P, _P, _P, _P, _P,
                                   C.c_int32, _P]),
    "vsrk_bn_finalize_dcount": (C.c_int, [_P, _P, _P, C.c_double, _P, _P, C.c_float, C.c_float, _P, _P, _P, _P,
                                          _P, _P, C.c_int32, _P]),
    "vsrk_bn_fold_running": (C.c_int, [_P, _P, _P, _P, C.c_float, _P, _P, _P, _P, C.c_int32, _P]),
    "vsrk_bn_apply": (C.c_int, [_T5, _P, _P, C.c_int32, _T5, _P]),
    "vsrk_bn_relu_bwd_reduce": (C.c_int, [_T5, _T5, _P, _P, _P, _P, _P, _P, _P, C.c_size_t, _P]),
    "vsrk_bn_relu_bwd_apply": (C.c_int, [_T5, _T5, _P, _P, _P, _P, _P, _P, _P, C.c_double, _T5, C.c_int32, _P]),
    "vsrk_bn_relu_bwd_apply_multi": (C.c_int, [_T5, _T5, C.c_int32, C.c_int32, C.POINTER(BnContrib), _P]),
    "vsrk_duf_dynfilter_fwd": (C.c_int, [_P, _P, _P] + [C.c_int32] * 5 + [_P, _P]),
    "vsrk_duf_dynfilter_bwd": (C.c_int, [_P, _P, _P] + [C.c_int32] * 5 + [_P, _P, C.c_int32, _P]),
    "vsrk_conv_set_algo": (C.c_int, [C.c_int32]),
    "vsrk_conv_set_path": (C.c_int, [C.c_char_p, C.c_int32]),
    "vsrk_conv_set_grid_cap": (C.c_int, [C.c_int32]),
    "vsrk_conv_set_roll_depth": (C.c_int, [C.c_int32]),
    "vsrk_subpixel_conv_weight": (C.c_int, [_P, _P] + [C.c_int32] * 6 + [_P, _P, _P]),
    "vsrk_subpixel_wgrad_fold": (C.c_int, [_P, _P] + [C.c_int32] * 6 + [_P, _P, C.c_int32, _P]),
    "vsrk_prelu_workspace_size": (C.c_size_t, []),
    "vsrk_prelu_wgrad": (C.c_int, [_T5, _T5, _P, _P, C.c_int32, _P, C.c_size_t, _P]),
    "vsrk_prelu_bwd": (C.c_int, [_T5, _T5, _T5, _P, _T5, _P, C.c_int32, _P, C.c_size_t, _P]),
    "vsrk_prelu_bwd_pre": (C.c_int, [_T5, _T5, _T5, _P, _T5, _P, C.c_int32, _P, C.c_size_t, _P]),
    "vsrk_ssim_workspace_size": (C.c_size_t, [C.c_int32] * 4),
    "vsrk_ssim": (C.c_int, [_P, _P] + [C.c_int32] * 5 + [C.c_float] * 3 + [_P, _P, _P, C.c_size_t, _P]),
    "vsrk_ssim3d_workspace_size": (C.c_size_t, [C.c_int32] * 5),
    "vsrk_resize_bicubic": (C.c_int, [_P] + [C.c_int32] * 5 + [_P, C.c_int32, _P]),
    "vsrk_ssim3d": (C.c_int, [_P, _P] + [C.c_int32] * 6 + [C.c_float] * 3 + [_P, _P, _P, C.c_size_t, _P]),
    "vsrk_last_error": (C.c_char_p, []),
    "vsrk_version": (C.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


def lib_path() -> Path:
    # VSRK_LIB: an alternative build of the same ABI (A/B kernel experiments)
    alt = os.environ.get("VSRK_LIB")
    return Path(alt) if alt else _build.LIB


def load(build_if_missing: bool = False):
    """Load libvsrk.so (optionally building it first) and bind signatures."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not path.exists():
            if not build_if_missing:
                raise RuntimeError(
                    f"vsrk native library not found at {path}; run `python -m vsr_amd.build` "
                    "(or __graft_entry__.build()) first — there is no CPU fallback")
            _build.build()
        elif path == _build.LIB and not _build.is_current():
            # a library built from other sources would bind this module's
            # struct layouts and signatures to different kernels
            if not build_if_missing:
                raise RuntimeError(
                    f"vsrk native library {path} is stale (built from different sources than "
                    f"vsr_amd/csrc); rebuild with `python -m vsr_amd.build`")
            _build.build()
        lib = C.CDLL(str(path))
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return _lib


def exported_symbols() -> list[str]:
    return list(_SIGS)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib.vsrk_last_error().decode(errors="replace")
        raise RuntimeError(f"vsrk {what} failed (code {rc}): {msg}")


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _DTYPE[dt]
    except KeyError:
        raise TypeError(f"vsrk supports float32/bfloat16/float16 activations, got {dt}") from None


def t5(t: torch.Tensor, shuffle: int = 1) -> Tensor5:
    """Describe a channels-last (N, D, H, W, C) tensor (any strides, unit
    channel stride).  With shuffle = r the tensor is the PHYSICAL image of a
    sub-pixel view: logical (n, d, h/r, w/r, c*r*r)."""
    if t.dim() != 5:
        raise ValueError(f"expected a 5-D (N,D,H,W,C) tensor, got shape {tuple(t.shape)}")
    if t.stride(4) != 1:
        raise ValueError("channel dimension must be contiguous")
    if not t.is_cuda:
        raise RuntimeError("vsrk ops need device tensors (no CPU fallback)")
    n, d, h, w, c = t.shape
    sn, sd, sh, sw, _ = t.stride()
    if shuffle > 1:
        if h % shuffle or w % shuffle:
            raise ValueError("spatial size not divisible by shuffle factor")
        h //= shuffle
        w //= shuffle
        c *= shuffle * shuffle
    return Tensor5(t.data_ptr(), n, d, h, w, c, sn, sd, sh, sw, shuffle, dtype_code(t.dtype))


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()
