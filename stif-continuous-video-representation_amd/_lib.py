"""ctypes binding of libstif_hip.so (the C ABI declared in include/stif.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``).  There is
no fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os

# STIF_HIP_LIB overrides the in-tree library (kernel experiments); the default is the in-tree build
LIB_PATH = os.environ.get("STIF_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libstif_hip.so")

MAXG = 8
EPI_NONE, EPI_LRELU, EPI_RELU, EPI_RES, EPI_OFFMASK, EPI_LSTM = range(6)
PACK_PLAIN, PACK_OFFMASK, PACK_LSTM, PACK_WINO, PACK_WINO_OFFMASK, PACK_WINO_LSTM, PACK_DCNSEP, PACK_DCNPAIR = range(8)
PACK_F16X3 = 16          # OR'ed into a PACK_WINO* mode (stif.h STIF_PACK_F16X3)
CONV_F16X3 = 1           # stif_conv_args.flags
CONV_DYNAMIC = 2         # stif_conv_args.flags: dynamic tile schedule (sched counters)
DEC_REVOLUTIONS = 2      # stif_pack_dec_proj_ex lr_image bit (stif.h STIF_DEC_REVOLUTIONS)

_P = C.c_void_p
_PA = _P * MAXG


class ConvArgs(C.Structure):
    _fields_ = [
        ("in0", _PA), ("in1", _PA), ("w", _PA), ("bias", _PA), ("out", _PA), ("res", _PA), ("out2", _PA),
        ("in0_item", C.c_longlong), ("in1_item", C.c_longlong), ("out_item", C.c_longlong),
        ("res_item", C.c_longlong), ("out2_item", C.c_longlong),
        ("ngroups", C.c_int), ("nitems", C.c_int),
        ("H", C.c_int), ("W", C.c_int), ("C0", C.c_int),
        ("C1", C.c_int), ("in1_mode", C.c_int), ("in1_scale", C.c_float),
        ("Ho", C.c_int), ("Wo", C.c_int), ("cout", C.c_int), ("ks", C.c_int), ("stride", C.c_int),
        ("epi", C.c_int), ("flags", C.c_int), ("status", _P), ("sched", _P),
    ]


class DcnArgs(C.Structure):
    _fields_ = [
        ("inp", _PA), ("offmask", _PA), ("w", _PA), ("bias", _PA), ("out", _PA),
        ("in_item", C.c_longlong), ("om_item", C.c_longlong), ("out_item", C.c_longlong),
        ("ngroups", C.c_int), ("nitems", C.c_int), ("H", C.c_int), ("W", C.c_int), ("epi", C.c_int),
        ("flags", C.c_int), ("status", _P),
    ]


class DcnSepArgs(C.Structure):
    _fields_ = [
        ("fea", _PA), ("inp", _PA), ("w_om", _PA), ("b_om", _PA), ("w", _PA), ("bias", _PA), ("out", _PA),
        ("fea_item", C.c_longlong), ("in_item", C.c_longlong), ("out_item", C.c_longlong),
        ("ngroups", C.c_int), ("nitems", C.c_int), ("H", C.c_int), ("W", C.c_int), ("epi", C.c_int),
        ("flags", C.c_int), ("status", _P),
    ]


class DecTables(C.Structure):
    _fields_ = [(n, _P) for n in ("near_y", "rel_y", "by0", "by1", "wy0", "wy1", "lin_y",
                                  "near_x", "rel_x", "bx0", "bx1", "wx0", "wx1", "lin_x", "hr_y", "hr_x")]


class DecImage(C.Structure):
    _fields_ = [("img", _P), ("ih", C.c_int), ("iw", C.c_int)] + [
        (n, _P) for n in ("by0", "by1", "wy0", "wy1", "bx0", "bx1", "wx0", "wx1")]


EXPORTS = {
    # name: (restype, argtypes)
    "stif_conv2d_nhwc": (C.c_int, [C.POINTER(ConvArgs), _P]),
    "stif_conv3x3_wino": (C.c_int, [C.POINTER(ConvArgs), _P]),
    "stif_upsample2x_nhwc": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_longlong,
                                       C.c_longlong, _P]),
    "stif_conv_first": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, C.c_int, _P]),
    "stif_dcn_nhwc": (C.c_int, [C.POINTER(DcnArgs), _P]),
    "stif_dcn_sep_nhwc": (C.c_int, [C.POINTER(DcnSepArgs), _P]),
    "stif_dcn_v2_workspace_size": (C.c_size_t, [C.c_int] * 14),
    "stif_dcn_v2_forward": (C.c_int, [_P] * 6 + [C.c_int] * 14 + [_P, C.c_size_t, _P]),
    "stif_dcn_v2_backward_workspace_size": (C.c_size_t, [C.c_int] * 14),
    "stif_dcn_v2_backward": (C.c_int, [_P] * 11 + [C.c_int] * 14 + [_P, C.c_size_t, _P]),
    "stif_dec_pack_lr": (C.c_int, [_P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int, _P]),
    "stif_dec_stage1": (C.c_int, [_P, _P, C.POINTER(DecTables), C.POINTER(DecImage), _P, _P, _P] + [C.c_int] * 5
                        + [_P]),
    "stif_dec_stage2": (C.c_int, [_P, _P, _P, _P, C.POINTER(DecTables), C.POINTER(DecImage), _P, _P]
                        + [C.c_int] * 5 + [_P]),
    "stif_dec_stage1_ex": (C.c_int, [_P, _P, C.POINTER(DecTables), C.POINTER(DecImage), _P, _P, _P]
                           + [C.c_int] * 6 + [_P, _P]),
    "stif_dec_stage2_ex": (C.c_int, [_P, _P, _P, _P, C.POINTER(DecTables), C.POINTER(DecImage), _P, _P]
                           + [C.c_int] * 6 + [_P, _P]),
    "stif_dec_blend4": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, _P]),
    "stif_upsample_image": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    "stif_resize_frames": (C.c_int, [_P, _P] + [C.c_int] * 5 + [_P, _P, C.c_int, C.c_int, _P, _P, C.c_int, C.c_int,
                                                                 _P]),
    "stif_frames_to_u8": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, _P]),
    "stif_pack_dec_proj_ex": (C.c_int, [_P, _P, _P, _P, C.c_int, _P, _P]),
    "stif_conv_weight_floats": (C.c_size_t, [C.c_int, C.c_int, C.c_int, C.c_int]),
    "stif_conv_bias_floats": (C.c_size_t, [C.c_int, C.c_int]),
    "stif_pack_conv_weight": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P]),
    "stif_dec_proj_floats": (C.c_size_t, []),
    "stif_pack_dec_proj": (C.c_int, [_P] * 6),
    "stif_dec_mlp_floats": (C.c_size_t, []),
    "stif_pack_dec_mlp": (C.c_int, [C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), _P]),
    "stif_pack_dec_mlp_ex": (C.c_int, [C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), _P, C.c_int]),
    "stif_last_error": (C.c_char_p, []),
    "stif_version": (C.c_char_p, []),
}

_lib = None


E_INVALID, E_LAUNCH, E_WORKSPACE, E_RANGE = 1, 2, 3, 4   # stif.h STIF_E_*


class StifError(RuntimeError):
    """Raised for any non-zero status of the C ABI (the reference surfaces AT_ERROR as RuntimeError)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise StifError(f"{LIB_PATH} not built; run `make` (or __graft_entry__.build())")
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().stif_last_error().decode(errors="replace")
        raise StifError(f"{what} failed (code {rc}): {msg}", rc)
