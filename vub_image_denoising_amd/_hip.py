"""ctypes binding of ``librdunet_hip.so`` (the C ABI in ``include/rdunet_hip.h``).

The library is built in-tree (``vub_image_denoising_amd/librdunet_hip.so``) by
``vub_image_denoising_amd.build.build_library`` / ``__graft_entry__.build``.
Nothing here falls back to another implementation: if the library is missing
or a call fails, a ``RuntimeError`` is raised.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RDN_LIB") or os.path.join(HERE, "librdunet_hip.so")

RDN_F32, RDN_BF16 = 0, 1
RDN_G_CONV3, RDN_G_S2, RDN_G_PIX = 0, 1, 2
EPI_BIAS, EPI_STORE_PRE, EPI_PRELU, EPI_RESID, EPI_ACCUM, EPI_SCATTER2, EPI_OUT_NCHW = 1, 2, 4, 8, 16, 32, 64
EPI_GOUT_KEEP = 128
PACK_CONV_FWD, PACK_CONV_DGRAD, PACK_GEMM_T = 0, 1, 2

_vp, _i32, _i64, _f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float


class ConvDesc(C.Structure):
    _fields_ = [
        ("dtype", _i32), ("gather", _i32), ("flags", _i32),
        ("n", _i32), ("h", _i32), ("w", _i32), ("hin", _i32), ("win", _i32), ("cin", _i32),
        ("x", _vp), ("x_ps", _i64), ("x_c0", _i32),
        ("wp", _vp), ("kp", _i32), ("ncols", _i32), ("cout", _i32),
        ("bias", _vp), ("alpha", _vp),
        ("out", _vp), ("out_ps", _i64), ("out_c0", _i32),
        ("pre", _vp), ("pre_ps", _i64),
        ("res", _vp), ("res_ps", _i64), ("res_c0", _i32), ("res_climit", _i32),
        ("out_nchw", _vp), ("res_nchw", _vp),
        ("bm", _i32), ("bn", _i32),
        ("gate", _vp), ("gate_ps", _i64), ("gate_alpha", _vp),
        ("x_pl", _i64), ("out_pl", _i64), ("pre_pl", _i64), ("res_pl", _i64), ("gate_pl", _i64),
        ("gout", _vp), ("gout_ps", _i64), ("gout_pre", _vp), ("gout_pre_ps", _i64),
        ("gout_alpha", _vp), ("gout_part", _vp), ("gout_c0", _i32),
    ]


class WgradDesc(C.Structure):
    _fields_ = [
        ("dtype", _i32), ("gather", _i32), ("n", _i32), ("h", _i32), ("w", _i32), ("hin", _i32), ("win", _i32),
        ("a", _vp), ("a_ps", _i64), ("a_c0", _i32), ("mdim", _i32),
        ("b", _vp), ("b_ps", _i64), ("b_c0", _i32), ("ndim", _i32),
        ("ws", _vp), ("splits", _i32),
        ("a_gate", _vp), ("a_gate_ps", _i64), ("a_gate_alpha", _vp), ("part", _vp),
        ("a_pl", _i64), ("b_pl", _i64), ("a_gate_pl", _i64),
    ]


class Dense3Desc(C.Structure):
    _fields_ = [
        ("n", _i32), ("h", _i32), ("w", _i32),
        ("x", _vp), ("x_pl", _i64),
        ("out", _vp * 3), ("pre", _vp * 3),
        ("wp", _vp * 3), ("kp", _i32 * 3),
        ("bias", _vp * 3), ("alpha", _vp * 3),
        ("x_c", _i32),
    ]


class ReduceJob(C.Structure):
    _fields_ = [("ws", _vp), ("grad", _vp), ("part", _vp), ("dalpha", _vp), ("dbias", _vp),
                ("splits", _i32), ("mdim", _i32), ("ndim", _i32), ("ndim_real", _i32), ("taps", _i32),
                ("gstride", _i32), ("gci0", _i32), ("accumulate", _i32), ("part_splits", _i32),
                ("sl", _i32), ("blocks", _i32), ("pblocks", _i32)]


REDUCE_BATCH_MAX = 8


class PackItem(C.Structure):
    _fields_ = [("w", _vp), ("out", _vp), ("mode", _i32), ("d0", _i32), ("d1", _i32), ("kh", _i32), ("kw", _i32),
                ("pad0", _i32), ("pad1", _i32), ("rows_pad", _i32), ("kp", _i32), ("ck", _i32)]


class SynthItem(C.Structure):
    _fields_ = [("clean_off", _i64), ("noisy_off", _i64), ("seed", C.c_uint64), ("row_stride", _i32),
                ("sigma", _f32), ("flip", _i32), ("rotate", _i32), ("affine", _i32 * 6)]


# name -> (restype, argtypes); every symbol include/rdunet_hip.h declares
SIGNATURES = {
    "rdn_conv_fwd": (_i32, [C.POINTER(ConvDesc), _vp]),
    "rdn_conv_wgrad": (_i32, [C.POINTER(WgradDesc), _vp]),
    "rdn_conv_kernel_name": (_i32, [C.POINTER(ConvDesc), C.c_char_p, _i32]),
    "rdn_conv_gate_rows": (_i32, [C.POINTER(ConvDesc)]),
    "rdn_wgrad_kernel_name": (_i32, [C.POINTER(WgradDesc), C.c_char_p, _i32]),
    "rdn_wgrad_splits": (_i32, [C.POINTER(WgradDesc)]),
    "rdn_conv_dgrad_wgrad": (_i32, [C.POINTER(ConvDesc), C.POINTER(WgradDesc), _vp]),
    "rdn_conv_dgrad_wgrad_splits": (_i32, [C.POINTER(ConvDesc), C.POINTER(WgradDesc)]),
    "rdn_conv_dgrad_wgrad_cols": (_i32, [C.POINTER(ConvDesc), C.POINTER(WgradDesc)]),
    "rdn_conv_dgrad_wgrad_gate_rows": (_i32, [C.POINTER(ConvDesc), C.POINTER(WgradDesc)]),
    "rdn_conv_dgrad_wgrad_kernel_name": (_i32, [C.POINTER(ConvDesc), C.POINTER(WgradDesc), C.c_char_p, _i32]),
    "rdn_wgrad_chunks": (_i32, [C.POINTER(WgradDesc)]),
    "rdn_dense3_fwd": (_i32, [C.POINTER(Dense3Desc), _vp]),
    "rdn_conv_fwd_splits": (_i32, [C.POINTER(ConvDesc)]),
    "rdn_conv_fwd_splitk_workspace_size": (_i64, [C.POINTER(ConvDesc), _i32]),
    "rdn_conv_fwd_splitk": (_i32, [C.POINTER(ConvDesc), _i32, _vp, _vp]),
    "rdn_dense3_kernel_name": (_i32, [C.POINTER(Dense3Desc), C.c_char_p, _i32]),
    "rdn_wgrad_workspace_size": (_i64, [C.POINTER(WgradDesc)]),
    "rdn_wgrad_reduce": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32, _vp, _i32, _vp, _vp, _vp]),
    "rdn_wgrad_reduce_cols": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _vp, _i32, _vp, _vp, _vp]),
    "rdn_wgrad_reduce_batch": (_i32, [C.POINTER(ReduceJob), _i32, _vp]),
    "rdn_prelu_bwd_blocks": (_i32, [_i32, _i64, _i32]),
    "rdn_prelu_bwd": (_i32, [_i32, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _i32, _i64, _vp, _vp, _i64, _vp,
                             _vp, _vp, _vp, _vp, _vp]),
    "rdn_prelu_bwd_workspace_size": (_i64, [_i32, _i64, _i32, _i32]),
    "rdn_interp": (_i32, [_vp, _vp, _vp, _i32, _i64, _vp, _vp]),
    "rdn_pack_input": (_i32, [_i32, _vp, _i32, _i32, _i32, _i32, _vp, _i64, _i64, _i64, _i32, _vp, _i32, _vp]),
    "rdn_pack_weights": (_i32, [_i32, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _vp]),
    "rdn_pack_weights_batched": (_i32, [_vp, _i32, _i32, _vp]),
    "rdn_conv3_chunk": (_i32, [_i32, _i32]),
    "rdn_conv3_packed_k": (_i32, [_i32, _i32]),
    "rdn_conv3_pick_bn": (_i32, [_i32]),
    "rdn_reduce_workspace_size": (_i64, [_i64]),
    "rdn_charbonnier_fwd": (_i32, [_vp, _vp, _i64, _f32, _vp, _vp, _vp]),
    "rdn_charbonnier_bwd": (_i32, [_vp, _vp, _i64, _f32, _f32, _f32, _vp, _vp, _vp]),
    "rdn_sqnorm": (_i32, [_vp, _i64, _f32, _vp, _vp, _vp]),
    "rdn_sqnorm_scaled": (_i32, [_vp, _i64, _f32, _f32, _vp, _vp, _vp]),
    "rdn_clip_scale": (_i32, [_vp, _i64, _vp, _vp]),
    "rdn_adam_step": (_i32, [_vp, _vp, _vp, _vp, _i64, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                             _i32, _i64, _vp, _f32, _vp]),
    "rdn_counter_inc": (_i32, [_vp, _vp]),
    "rdn_stamp": (_i32, [_vp, _i32, _vp]),
    "rdn_wall_clock_khz": (_i64, []),
    "rdn_sampling_combine": (_i32, [_vp, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _vp]),
    "rdn_nchw_to_nhwc": (_i32, [_i32, _vp, _i32, _i32, _i32, _i32, _vp, _i64, _i32, _i64, _i32, _vp]),
    "rdn_nhwc_to_nchw": (_i32, [_i32, _vp, _i64, _i32, _i64, _i32, _i32, _i32, _i32, _vp, _i32, _vp]),
    "rdn_zero_slice": (_i32, [_i32, _vp, _i64, _i64, _i32, _i32, _vp]),
    "rdn_synth_batch": (_i32, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "rdn_image_metrics_workspace_size": (_i64, [_i32, _i32, _i32, _i32]),
    "rdn_image_metrics": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, C.c_float, _vp, _vp, _vp, _vp]),
    "rdn_version": (C.c_char_p, []),
    "rdn_last_error": (C.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load and type the library (no GPU work).  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"librdunet_hip.so not found at {path}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load_library()


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().rdn_last_error().decode(errors="replace")
        raise RuntimeError(f"librdunet_hip {what} failed ({rc}): {msg}")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return RDN_F32
    if dt == torch.bfloat16:
        return RDN_BF16
    raise ValueError(f"unsupported activation dtype {dt}")


def require_device(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda):
            raise RuntimeError("vub_image_denoising_amd runs on the ROCm GPU only (HIP kernels); got a CPU tensor. "
                               "Move the model and inputs to 'cuda'.")
