"""ctypes binding of libvdiff.so (the C-ABI declared in include/vdiff.h).

This is the only place that talks to the native library.  There is no
fallback: if the library or a GPU is missing, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# VDIFF_LIB: alternative build of the same library (kernel A/B experiments, tools/)
LIB_PATH = os.environ.get("VDIFF_LIB") or os.path.join(_HERE, "libvdiff.so")

VD_F32 = 0
VD_BF16 = 1
ABI_VERSION = 1

_vp = C.c_void_p
_i = C.c_int
_i64 = C.c_int64
_u64 = C.c_uint64
_f = C.c_float
_sz = C.c_size_t


class ConvDesc(C.Structure):
    _fields_ = [(n, _i) for n in (
        "B", "Ti", "Hi", "Wi", "Ci", "To", "Ho", "Wo", "Co",
        "kt", "kh", "kw", "st", "sh", "sw", "pt", "ph", "pw",
        "x_cstride", "y_cstride", "dtype")]


class AttnDesc(C.Structure):
    _fields_ = [("nseq", _i), ("seq_len", _i), ("head_dim", _i), ("groups", _i),
                ("batch_stride", _i64), ("group_stride", _i64), ("token_stride", _i64),
                ("o_batch_stride", _i64), ("o_group_stride", _i64), ("o_token_stride", _i64),
                ("scale", _f), ("dtype", _i)]


class XAttnDesc(C.Structure):
    """vd_xattn_desc: queries / output as AttnDesc, K/V rows of their own."""
    _fields_ = [("q", AttnDesc), ("kv_len", _i), ("kv_batch_stride", _i64),
                ("kv_group_stride", _i64), ("kv_token_stride", _i64)]


_SIGS = {
    "vd_version": (_i, []),
    "vd_last_error": (C.c_char_p, []),
    "vd_device_info": (_i, [C.c_char_p, _i]),
    "vd_timestep_embedding": (_i, [_vp, _i, _i, _f, _vp, _vp]),
    "vd_timestep_embedding_tab": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "vd_q_sample": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i, _vp]),
    "vd_p_sample_v1": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i, _vp]),
    "vd_p_sample_v2": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i,
                            _vp]),
    "vd_p_sample_cosine": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i, _vp]),
    "vd_ddim_step": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _i, _i64, _i64, _i, _vp]),
    "vd_set_dropout_counter": (None, [_vp]),
    "vd_groupnorm_set_unroll": (_i, [_i]),
    "vd_groupnorm_workspace_size": (_sz, [_i, _i64, _i, _i]),
    "vd_groupnorm_silu_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i64, _i, _i, _f, _i, _f,
                                   _u64, _i, _vp, _vp]),
    "vd_groupnorm_silu_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i64, _i, _i,
                                   _i, _f, _u64, _i, _vp, _vp]),
    "vd_groupnorm_silu_bwd_add": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i64,
                                       _i, _i, _i, _f, _u64, _i, _vp, _vp]),
    "vd_silu": (_i, [_vp, _vp, _i64, _i, _vp]),
    "vd_silu_bwd": (_i, [_vp, _vp, _vp, _i64, _i, _vp]),
    "vd_cond_concat": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "vd_cond_concat_bwd_workspace_size": (_sz, [_i, _i, _i, _i, _i]),
    "vd_cond_concat_bwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp,
                                _vp]),
    "vd_upsample_nearest_hw": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp]),
    "vd_upsample_nearest_hw_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp]),
    "vd_channel_sums_workspace_size": (_sz, [_i, _i]),
    "vd_channel_sums": (_i, [_vp, _i, _i64, _i, _i, _i, _vp, _vp, _vp]),
    "vd_conv_pack_weight": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "vd_conv_pack_weights": (_i, [_vp, _i, _i64, _i, _vp]),
    "vd_conv_set_wgrad": (_i, [C.c_int]),
    "vd_conv_set_halo": (_i, [_i]),
    "vd_conv3d_fwd": (_i, [C.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "vd_conv3d_bwd_data": (_i, [C.POINTER(ConvDesc), _vp, _vp, _vp, _vp]),
    "vd_conv3d_bwd_weight": (_i, [C.POINTER(ConvDesc), _vp, _vp, _vp, _vp]),
    "vd_conv3d_bwd_weight_workspace_size": (_sz, [C.POINTER(ConvDesc)]),
    "vd_conv3d_bwd_weight_det": (_i, [C.POINTER(ConvDesc), _vp, _vp, _vp, _i, _i, _vp, _sz, _vp]),
    "vd_attention_fwd": (_i, [C.POINTER(AttnDesc), _vp, _vp, _vp, _vp, _vp, _vp]),
    "vd_attention_fwd_workspace_size": (_sz, [C.POINTER(AttnDesc)]),
    "vd_attention_fwd_ws": (_i, [C.POINTER(AttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "vd_attention_bwd_workspace_size": (_sz, [C.POINTER(AttnDesc)]),
    "vd_attention_set_config": (C.c_int, [C.c_int]),
    "vd_attention_bwd": (_i, [C.POINTER(AttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                              _vp, _vp]),
    "vd_attention_bwd_dq": (_i, [C.POINTER(AttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                 _vp]),
    "vd_attention_bwd_dkdv": (_i, [C.POINTER(AttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp]),
    "vd_cross_attention_fwd_workspace_size": (_sz, [C.POINTER(XAttnDesc)]),
    "vd_cross_attention_fwd": (_i, [C.POINTER(XAttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _sz,
                                    _vp]),
    "vd_cross_attention_bwd_workspace_size": (_sz, [C.POINTER(XAttnDesc)]),
    "vd_cross_attention_bwd_dq": (_i, [C.POINTER(XAttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp]),
    "vd_cross_attention_bwd_dkdv": (_i, [C.POINTER(XAttnDesc), _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp, _vp, _vp]),
    "vd_resize_plan": (_i, [_i, _i, _vp, _vp, _i]),
    "vd_frames_resize_normalize": (_i, [_vp, _i64, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _i,
                                        _vp, _vp, _i, _i64, _i, _vp]),
    "vd_audio_window": (_i, [_vp, _i, _i64, _i, C.c_double, _i, _i, _i, _i, _i, _vp]),
    "vd_layernorm_workspace_size": (_sz, [_i, _i]),
    "vd_layernorm_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, C.c_float, _i, _vp]),
    "vd_layernorm_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _sz,
                              _vp]),
    "vd_gelu_tanh": (_i, [_vp, _vp, _i64, _i, _vp]),
    "vd_attention_short_path": (_i, [C.POINTER(AttnDesc)]),
    "vd_attention_bwd_short_path": (_i, [C.POINTER(AttnDesc)] + [C.c_void_p] * 8),
    "vd_attention_set_short": (_i, [_i]),
    "vd_mse_loss_workspace_size": (_sz, [_i64]),
    "vd_mse_loss": (_i, [_vp, _vp, _i64, _i, _vp, _vp, _sz, _vp]),
    "vd_mse_loss_bwd": (_i, [_vp, _vp, _vp, _i64, _i, _vp, _vp]),
    "vd_gelu_tanh_bwd": (_i, [_vp, _vp, _vp, _i64, _i, _vp]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load and type the library (no GPU needed to load)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"libvdiff.so not found at {path}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.vd_version() != ABI_VERSION:
            raise RuntimeError(f"libvdiff ABI {lib.vd_version()} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load()


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().vd_last_error().decode(errors="replace")
        raise RuntimeError(f"libvdiff {what} failed (code {rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
