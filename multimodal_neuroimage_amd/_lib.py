"""ctypes binding of libmmni.so (include/mmni.h).

The product path has no CPU fallback: if the library is missing, or a tensor is not on a
ROCm device, the call raises.  torch is imported before the library is opened so that the
library's libamdhip64.so.7 dependency resolves to the HIP runtime torch already loaded
(one runtime per process; torch's streams are then valid handles for our launches).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# MMNI_LIB selects another in-tree build of the same library (kernel experiments,
# scripts/build_variant.sh); the default is the package's libmmni.so.
LIB_PATH = os.environ.get("MMNI_LIB") or os.path.join(_HERE, "libmmni.so")
ABI_VERSION = 8

_c_int = ctypes.c_int
_c_i32 = ctypes.c_int32
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_vp = ctypes.c_void_p


class WAttnDesc(ctypes.Structure):
    _fields_ = [("B", _c_i32), ("D", _c_i32), ("H", _c_i32), ("W", _c_i32),
                ("C", _c_i32), ("heads", _c_i32),
                ("wd", _c_i32), ("wh", _c_i32), ("ww", _c_i32),
                ("sd", _c_i32), ("sh", _c_i32), ("sw", _c_i32),
                ("kind", _c_i32), ("scale", _c_f),
                ("q_stride", _c_i64), ("k_stride", _c_i64), ("v_stride", _c_i64), ("o_stride", _c_i64)]


class MhaDesc(ctypes.Structure):
    _fields_ = [("Tq", _c_i32), ("Tk", _c_i32), ("B", _c_i32), ("heads", _c_i32), ("head_dim", _c_i32),
                ("causal_diag", _c_i32), ("scale", _c_f),
                ("q_stride", _c_i64), ("k_stride", _c_i64), ("v_stride", _c_i64), ("o_stride", _c_i64),
                ("dropout", _c_f), ("seed", ctypes.c_uint32), ("dtype", ctypes.c_int32)]


class Conv3dDesc(ctypes.Structure):
    _fields_ = [("B", _c_i32), ("D", _c_i32), ("H", _c_i32), ("W", _c_i32), ("Cin", _c_i32),
                ("Cout", _c_i32), ("kd", _c_i32), ("kh", _c_i32), ("kw", _c_i32),
                ("sd", _c_i32), ("sh", _c_i32), ("sw", _c_i32), ("pd", _c_i32), ("ph", _c_i32), ("pw", _c_i32),
                ("Do", _c_i32), ("Ho", _c_i32), ("Wo", _c_i32), ("slope", _c_f)]


class TLinDesc(ctypes.Structure):
    _fields_ = [("rows", _c_i64), ("K", _c_i32), ("N", _c_i32), ("epi", _c_i32), ("K2", _c_i32),
                ("ldx", _c_i64), ("ldy", _c_i64), ("ldaux", _c_i64), ("w_sn", _c_i64), ("w_sk", _c_i64)]


class MlpDesc(ctypes.Structure):
    _fields_ = [("rows", _c_i64), ("C", _c_i32), ("H", _c_i32), ("ldx", _c_i64), ("ldy", _c_i64)]


class TokDesc(ctypes.Structure):
    _fields_ = [("rows", _c_i64), ("C", _c_i32), ("N", _c_i32), ("eps", _c_f)]


class BandSplitDesc(ctypes.Structure):
    _fields_ = [("B", _c_i32), ("R", _c_i32), ("Lmax", _c_i32), ("seq", _c_i32), ("ntaps", _c_i32)]


class RowGemmDesc(ctypes.Structure):
    _fields_ = [("rows", _c_i64), ("K", _c_i32), ("N", _c_i32), ("ldx", _c_i64), ("ldy", _c_i64),
                ("ldres", _c_i64), ("ldaux", _c_i64), ("w_sn", _c_i64), ("w_sk", _c_i64), ("ln", _c_i32),
                ("eps", _c_f), ("relu", _c_i32)]


# symbol -> (restype, argtypes); every symbol include/mmni.h declares
SIGNATURES = {
    "mmni_version": (_c_int, []),
    "mmni_rowgemm": (_c_int, [ctypes.POINTER(RowGemmDesc)] + [_vp] * 11),
    "mmni_rowgemm_dw_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(RowGemmDesc)]),
    "mmni_rowgemm_dw": (_c_int, [ctypes.POINTER(RowGemmDesc)] + [_vp] * 10),
    "mmni_row_layernorm_fwd": (_c_int, [_c_i64, _c_int, _vp, _c_i64, _vp, _vp, ctypes.c_float, _vp, _c_i64, _vp, _vp,
                                        _vp]),
    "mmni_row_layernorm_bwd_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_int]),
    "mmni_row_layernorm_fwd_t": (_c_int, [_c_i64, _c_int, _vp, _c_i64, _vp, _vp, ctypes.c_float, _vp, _c_int, _c_i64,
                                          _vp, _vp, _vp]),
    "mmni_row_layernorm_bwd_t": (_c_int, [_c_i64, _c_int, _vp, _c_int, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp, _c_i64,
                                          _vp, _c_i64, _vp, _vp, _vp, _vp]),
    "mmni_cpb_fwd": (_c_int, [_c_i64, _c_int, _c_int, _c_int] + [_vp] * 6),
    "mmni_cpb_bwd_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_int, _c_int, _c_int]),
    "mmni_cpb_bwd": (_c_int, [_c_i64, _c_int, _c_int, _c_int] + [_vp] * 11),
    "mmni_row_layernorm_bwd": (_c_int, [_c_i64, _c_int, _vp, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp, _c_i64, _vp,
                                        _c_i64, _vp, _vp, _vp, _vp]),
    "mmni_cast_bf16_multi": (_c_int, [_c_int, _vp, _vp, _vp, _vp]),
    "mmni_splitk_reduce_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_int]),
    "mmni_splitk_reduce": (_c_int, [_c_int, _c_i64, _vp, _c_i64, _c_int, _vp, _c_i64, _c_int, _vp, _vp, _vp, _vp]),
    "mmni_last_error": (ctypes.c_char_p, []),
    "mmni_wattn_fwd": (_c_int, [ctypes.POINTER(WAttnDesc)] + [_vp] * 9),
    "mmni_wattn_bwd": (_c_int, [ctypes.POINTER(WAttnDesc)] + [_vp] * 16),
    "mmni_wattn_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(WAttnDesc)]),
    "mmni_window_rows": (_c_int, [ctypes.POINTER(WAttnDesc), _vp, _vp]),
    "mmni_window_mask": (_c_int, [ctypes.POINTER(WAttnDesc), _vp, _vp]),
    "mmni_relative_index": (_c_int, [ctypes.POINTER(WAttnDesc), _vp, _vp]),
    "mmni_mha_fwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(MhaDesc)]),
    "mmni_mha_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(MhaDesc)]),
    "mmni_mha_fwd": (_c_int, [ctypes.POINTER(MhaDesc)] + [_vp] * 7),
    "mmni_mha_bwd": (_c_int, [ctypes.POINTER(MhaDesc)] + [_vp] * 11),
    "mmni_mha_mean_probs": (_c_int, [ctypes.POINTER(MhaDesc), _vp, _vp, _vp, _vp, _vp]),
    "mmni_mha_dropout_mask": (_c_int, [ctypes.POINTER(MhaDesc), _vp, _vp]),
    "mmni_conv3d_fwd": (_c_int, [ctypes.POINTER(Conv3dDesc), _vp, _vp, _vp, _vp, _vp]),
    "mmni_conv3d_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(Conv3dDesc)]),
    "mmni_conv3d_bwd": (_c_int, [ctypes.POINTER(Conv3dDesc)] + [_vp] * 9),
    "mmni_layernorm_fwd": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _c_f, _vp, _vp, _vp, _vp]),
    "mmni_layernorm_bwd_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_int]),
    "mmni_layernorm_bwd": (_c_int, [_c_i64, _c_int] + [_vp] * 10),
    "mmni_linear_dw_workspace_bytes": (ctypes.c_size_t, [_c_int, _c_int]),
    "mmni_linear_dw": (_c_int, [_c_i64, _c_int, _c_int, _vp, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp]),
    "mmni_token_linear": (_c_int, [ctypes.POINTER(TLinDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmni_token_linear_supported": (_c_int, [_c_int, _c_int, _c_int, _c_int]),
    "mmni_mlp_supported": (_c_int, [_c_int, _c_int]),
    "mmni_mlp_fwd": (_c_int, [ctypes.POINTER(MlpDesc)] + [_vp] * 8),
    "mmni_mlp_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(MlpDesc)]),
    "mmni_mlp_bwd": (_c_int, [ctypes.POINTER(MlpDesc)] + [_vp] * 12),
    "mmni_ln_mlp_fwd": (_c_int, [ctypes.POINTER(MlpDesc), _c_f] + [_vp] * 7 + [_c_int, _vp, _vp]),
    "mmni_ln_mlp_skip_fwd": (_c_int, [ctypes.POINTER(MlpDesc), _c_f] + [_vp] * 7 + [_c_int, _vp, _vp, _vp]),
    "mmni_ln_mlp_bwd": (_c_int, [ctypes.POINTER(MlpDesc), _c_f] + [_vp] * 7 + [_c_int] + [_vp] * 9),
    "mmni_zscore_workspace_bytes": (ctypes.c_size_t, [_c_i64]),
    "mmni_zscore": (_c_int, [_c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp]),
    "mmni_fir_highpass_taps": (_c_int, [_c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]),
    "mmni_fmri_band_split": (_c_int, [ctypes.POINTER(BandSplitDesc)] + [_vp] * 7),
    "mmni_ln_linear_fwd": (_c_int, [ctypes.POINTER(TokDesc)] + [_vp] * 9),
    "mmni_tok_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(TokDesc)]),
    "mmni_ln_linear_bwd": (_c_int, [ctypes.POINTER(TokDesc)] + [_vp] * 15),
    "mmni_ln_linear_bwd2": (_c_int, [ctypes.POINTER(TokDesc)] + [_vp] * 16),
    "mmni_linear_bwd": (_c_int, [ctypes.POINTER(TokDesc)] + [_vp] * 8),
}

_lib = None


def load():
    """Open libmmni.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                           "(there is no CPU fallback for the HIP hot path)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.mmni_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"libmmni.so ABI version {v} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().mmni_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def stream_handle(device=None):
    return _vp(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return _vp(t.data_ptr()) if t is not None else _vp(0)


def require_device(*tensors, what="mmni", dtypes=(torch.float32,)):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f"{what}: tensors must live on a ROCm device (got {t.device}); "
                               "the HIP hot path has no CPU fallback")
        if t.dtype not in dtypes:
            raise RuntimeError(f"{what}: expected {' or '.join(str(d) for d in dtypes)} tensors, got {t.dtype}")