"""Thin torch-facing wrappers over the C ABI.

Torch tensors are only device buffers here: every op passes ``data_ptr()``s,
sizes and the current HIP stream to libstif_hip.so.  Feature maps are NHWC
``[items, H, W, C]`` fp32 tensors (any item stride; rows/pixels contiguous).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib as L
from .coords import TABLE_ORDER, dec_tables

# Optional launch tracer (bench.py sets it to time the dominant kernel with HIP events on
# the launch stream): an object with begin(kind: tuple, flops: float) and end().
TRACE = None

# Dynamic tile scheduling of the persistent Winograd conv (stif_conv_args.sched): one block of counters
# per (device, stream), zeroed once and kept for the process (the library tracks each block's running
# totals) -- launches on one stream run in issue order, launches on different streams never share one.
# Default off: at C0 the dynamic schedule measured 0.1-0.3 ms per step slower than the static one alone,
# and equal to it with the PCD DCN branch on a second stream (profiles/r05_dynamic_tiles_ab.log).
DYNAMIC_TILES = False
_SCHED = {}


def _sched_buf():
    if not DYNAMIC_TILES or torch.cuda.is_current_stream_capturing():
        return None
    s = torch.cuda.current_stream()
    key = (s.device.index, s.cuda_stream)
    b = _SCHED.get(key)
    if b is None:
        b = _SCHED[key] = torch.zeros(16, dtype=torch.int32, device=s.device)   # stream-ordered before use
    return b


def _vp(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _item_stride(ts: Sequence[Optional[torch.Tensor]], what: str) -> int:
    strides = {t.stride(0) for t in ts if t is not None}
    if len(strides) > 1:
        raise ValueError(f"{what}: groups must share the item stride, got {strides}")
    for t in ts:
        if t is None:
            continue
        if t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"{what}: expected float32 CUDA tensors")
        _, h, w, c = t.shape
        # strides of size-1 dims never address anything
        if (c > 1 and t.stride(3) != 1) or (w > 1 and t.stride(2) != c) or (h > 1 and t.stride(1) != w * c):
            raise ValueError(f"{what}: pixels of an item must be contiguous NHWC")
    return strides.pop() if strides else 0


@dataclass
class PackedConv:
    """A conv layer repacked for stif_conv2d_nhwc (see stif_pack_conv_weight)."""
    w: torch.Tensor
    b: torch.Tensor
    cout: int
    cin: int
    ks: int
    mode: int


def pack_conv(weight: np.ndarray, bias: np.ndarray, mode: int = L.PACK_PLAIN, device="cuda",
              range_fallback: bool = True) -> PackedConv:
    """Pack one conv layer.  A STIF_PACK_F16X3 packing whose weights leave the split-fp16 range
    (stif_pack_conv_weight -> STIF_E_RANGE) is re-packed in fp32 (same kernel family, fp32 MFMA)
    when ``range_fallback``; otherwise the StifError propagates."""
    weight = np.ascontiguousarray(weight, np.float32)
    bias = np.ascontiguousarray(bias, np.float32)
    cout, cin, ks, _ = weight.shape
    lib = L.lib()
    wd = np.empty(lib.stif_conv_weight_floats(cout, cin, ks, mode), np.float32)
    bd = np.empty(lib.stif_conv_bias_floats(cout, mode), np.float32)
    try:
        L.check(lib.stif_pack_conv_weight(weight.ctypes.data, bias.ctypes.data, cout, cin, ks, mode,
                                          wd.ctypes.data, bd.ctypes.data), "stif_pack_conv_weight")
    except L.StifError as e:
        if e.code != L.E_RANGE or not range_fallback or not mode & L.PACK_F16X3:
            raise
        return pack_conv(weight, bias, mode & ~L.PACK_F16X3, device, False)
    return PackedConv(torch.from_numpy(wd).to(device), torch.from_numpy(bd).to(device), cout, cin, ks, mode)


def _split_by_mode(groups, key):
    """Launch groups by operand mode: layers that fell back to fp32 packing run in their own launch."""
    f16 = [g for g in groups if g[key].mode & L.PACK_F16X3]
    return [f16, [g for g in groups if not g[key].mode & L.PACK_F16X3]] if 0 < len(f16) < len(groups) else None


def conv2d(groups, *, epi=L.EPI_NONE, in1_mode=0, in1_scale=1.0, stride=None, status=None):
    """groups: list of dicts {layer: PackedConv, in0, [in1], out, [res], [out2]} with tensors
    [nitems, H, W, C].  All groups share shapes and item strides.  status: optional int32 device
    word that f16x3 kernels set on a non-finite output (operand out of the split range)."""
    if not 1 <= len(groups) <= L.MAXG:
        raise ValueError("conv2d: 1..8 groups")
    parts = _split_by_mode(groups, "layer")
    if parts:
        for part in parts:
            conv2d(part, epi=epi, in1_mode=in1_mode, in1_scale=in1_scale, stride=stride, status=status)
        return
    g0 = groups[0]
    lay: PackedConv = g0["layer"]
    in0 = g0["in0"]
    nitems, H, W, C0 = in0.shape
    C1 = g0["in1"].shape[3] if in1_mode else 0
    ks = lay.ks
    if stride is None:
        stride = 1
    pad = ks // 2
    Ho = (H + 2 * pad - ks) // stride + 1
    Wo = (W + 2 * pad - ks) // stride + 1
    a = L.ConvArgs()
    for i, g in enumerate(groups):
        if g["layer"].cin != C0 + C1 or g["layer"].ks != ks:
            raise ValueError("conv2d: layer shape mismatch")
        a.in0[i] = _vp(g["in0"])
        a.in1[i] = _vp(g.get("in1"))
        a.w[i] = _vp(g["layer"].w)
        a.bias[i] = _vp(g["layer"].b)
        a.out[i] = _vp(g["out"])
        a.res[i] = _vp(g.get("res"))
        a.out2[i] = _vp(g.get("out2"))
        if tuple(g["out"].shape[:3]) != (nitems, Ho, Wo):
            raise ValueError(f"conv2d: output shape {tuple(g['out'].shape)} != {(nitems, Ho, Wo)}")
    a.in0_item = _item_stride([g["in0"] for g in groups], "in0")
    a.in1_item = _item_stride([g.get("in1") for g in groups], "in1") if in1_mode else 0
    a.out_item = _item_stride([g["out"] for g in groups], "out")
    a.res_item = _item_stride([g.get("res") for g in groups], "res")
    a.out2_item = _item_stride([g.get("out2") for g in groups], "out2")
    a.ngroups, a.nitems = len(groups), nitems
    a.H, a.W, a.C0, a.C1 = H, W, C0, C1
    a.in1_mode, a.in1_scale = in1_mode, in1_scale
    a.Ho, a.Wo, a.cout, a.ks, a.stride, a.epi = Ho, Wo, lay.cout, ks, stride, epi
    wmodes = (L.PACK_WINO, L.PACK_WINO_OFFMASK, L.PACK_WINO_LSTM)
    wino = (lay.mode & ~L.PACK_F16X3) in wmodes
    if any(((g["layer"].mode & ~L.PACK_F16X3) in wmodes) != wino or (g["layer"].mode ^ lay.mode) & L.PACK_F16X3
           for g in groups):
        raise ValueError("conv2d: groups mix Winograd / direct or f32 / f16x3 packings")
    a.flags = L.CONV_F16X3 if lay.mode & L.PACK_F16X3 else 0
    a.status = _vp(status)
    sched = _sched_buf() if wino else None
    a.sched = _vp(sched)
    if sched is not None:
        a.flags |= L.CONV_DYNAMIC
    tr = TRACE
    if tr is not None:
        # algorithmic (direct-convolution) FLOPs, whichever algorithm runs
        # algorithmic HBM bytes: every input read once, every output written once
        px_in, px_out = H * W * nitems * len(groups), Ho * Wo * nitems * len(groups)
        c_in = C0 + (C1 if in1_mode == 1 else C1 / 4.0 if in1_mode == 2 else 0)
        c_out = 128 if epi == L.EPI_LSTM else lay.cout
        c_res = 64 if epi in (L.EPI_RES, L.EPI_LSTM) else 0
        tr.begin(("wino" if wino else "conv", ks, stride, epi, in1_mode, lay.cout),
                 2.0 * lay.cout * (C0 + C1) * ks * ks * Ho * Wo * nitems * len(groups),
                 4.0 * (c_in * px_in + (c_out + c_res) * px_out))
    if wino:
        L.check(L.lib().stif_conv3x3_wino(C.byref(a), _stream()), "stif_conv3x3_wino")
    else:
        L.check(L.lib().stif_conv2d_nhwc(C.byref(a), _stream()), "stif_conv2d_nhwc")
    if tr is not None:
        tr.end()


def upsample2x(x: torch.Tensor, out: torch.Tensor, scale: float = 1.0):
    """out = scale * bilinear x2 upsample (align_corners=False) of NHWC x [n, h, w, c] (items may be
    strided; pixels contiguous) into out [n, 2h, 2w, c]."""
    n, h, w, c = x.shape
    if tuple(out.shape) != (n, 2 * h, 2 * w, c):
        raise ValueError(f"upsample2x: out shape {tuple(out.shape)} != {(n, 2 * h, 2 * w, c)}")
    for t in (x, out):
        # strides of size-1 dims never address anything, so they are not checked
        _, th, tw, _ = t.shape
        if (c > 1 and t.stride(3) != 1) or (tw > 1 and t.stride(2) != c) or (th > 1 and t.stride(1) != tw * c):
            raise ValueError("upsample2x: pixels must be contiguous")
    tr = TRACE
    if tr is not None:
        tr.begin(("up2",), 0.0)
    L.check(L.lib().stif_upsample2x_nhwc(_vp(x), _vp(out), n, h, w, c, float(scale),
                                         x.stride(0) if n > 1 else h * w * c,
                                         out.stride(0) if n > 1 else 4 * h * w * c, _stream()),
            "stif_upsample2x_nhwc")
    if tr is not None:
        tr.end()


def conv_first(x_nchw: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: torch.Tensor):
    n, c, h, wd = x_nchw.shape
    assert c == 3 and x_nchw.is_contiguous() and out.is_contiguous()
    L.check(L.lib().stif_conv_first(_vp(x_nchw), _vp(w), _vp(b), _vp(out), n, h, wd, _stream()), "stif_conv_first")


def dcn(groups, *, epi=L.EPI_NONE, status=None):
    """Fused DCN_sep core. groups: list of {layer: PackedConv (64->64 3x3), inp, offmask, out}."""
    parts = _split_by_mode(groups, "layer")
    if parts:
        for part in parts:
            dcn(part, epi=epi, status=status)
        return
    g0 = groups[0]
    nitems, H, W, Cc = g0["inp"].shape
    assert Cc == 64
    a = L.DcnArgs()
    for i, g in enumerate(groups):
        a.inp[i] = _vp(g["inp"])
        a.offmask[i] = _vp(g["offmask"])
        a.w[i] = _vp(g["layer"].w)
        a.bias[i] = _vp(g["layer"].b)
        a.out[i] = _vp(g["out"])
    a.in_item = _item_stride([g["inp"] for g in groups], "dcn in")
    a.om_item = _item_stride([g["offmask"] for g in groups], "dcn offmask")
    a.out_item = _item_stride([g["out"] for g in groups], "dcn out")
    a.ngroups, a.nitems, a.H, a.W, a.epi = len(groups), nitems, H, W, epi
    f16 = g0["layer"].mode & L.PACK_F16X3
    a.flags = L.CONV_F16X3 if f16 else 0
    a.status = _vp(status)
    tr = TRACE
    if tr is not None:
        tr.begin(("dcn", epi), 2.0 * 64 * 576 * H * W * nitems * len(groups),
                 4.0 * (64 + 216 + 64) * H * W * nitems * len(groups))
    L.check(L.lib().stif_dcn_nhwc(C.byref(a), _stream()), "stif_dcn_nhwc")
    if tr is not None:
        tr.end()


def dcn_sep_fusable(om_layer: PackedConv, layer: PackedConv) -> bool:
    """Both layers of a DCN_sep packed for the fused kernel (stif_dcn_sep_nhwc)."""
    return om_layer.mode == (L.PACK_DCNSEP | L.PACK_F16X3) and layer.mode == (L.PACK_DCNPAIR | L.PACK_F16X3)


def dcn_sep(groups, *, epi=L.EPI_NONE, status=None):
    """Fused DCN_sep (dcn_v2.py:127-140): offset/mask conv + sigmoid + deformable conv in one launch.
    groups: list of {om_layer: PackedConv (STIF_PACK_DCNSEP | F16X3), layer: PackedConv (64->64 3x3,
    STIF_PACK_DCNPAIR | F16X3), fea, inp, out} with NHWC [nitems, H, W, 64] tensors."""
    if not 1 <= len(groups) <= L.MAXG:
        raise ValueError("dcn_sep: 1..8 groups")
    g0 = groups[0]
    nitems, H, W, Cc = g0["inp"].shape
    a = L.DcnSepArgs()
    for i, g in enumerate(groups):
        if not dcn_sep_fusable(g["om_layer"], g["layer"]):
            raise ValueError("dcn_sep: layers not packed for the fused kernel")
        for k in ("fea", "inp", "out"):
            if tuple(g[k].shape) != (nitems, H, W, 64):
                raise ValueError(f"dcn_sep: {k} shape {tuple(g[k].shape)} != {(nitems, H, W, 64)}")
        a.fea[i] = _vp(g["fea"])
        a.inp[i] = _vp(g["inp"])
        a.w_om[i] = _vp(g["om_layer"].w)
        a.b_om[i] = _vp(g["om_layer"].b)
        a.w[i] = _vp(g["layer"].w)
        a.bias[i] = _vp(g["layer"].b)
        a.out[i] = _vp(g["out"])
    a.fea_item = _item_stride([g["fea"] for g in groups], "dcn_sep fea")
    a.in_item = _item_stride([g["inp"] for g in groups], "dcn_sep in")
    a.out_item = _item_stride([g["out"] for g in groups], "dcn_sep out")
    a.ngroups, a.nitems, a.H, a.W, a.epi = len(groups), nitems, H, W, epi
    a.flags = L.CONV_F16X3
    a.status = _vp(status)
    tr = TRACE
    if tr is not None:
        px = H * W * nitems * len(groups)
        # algorithmic: the offset/mask conv (216 x 576 MACs) + the deformable conv (64 x 576) per pixel;
        # HBM bytes: the offset feature, the DCN input and the output read / written once (768 B / px)
        tr.begin(("dcnsep", epi), 2.0 * (216 + 64) * 576 * px, 4.0 * 3 * 64 * px)
    L.check(L.lib().stif_dcn_sep_nhwc(C.byref(a), _stream()), "stif_dcn_sep_nhwc")
    if tr is not None:
        tr.end()


def dcn_v2_forward(input, weight, bias, offset, mask, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                   dilation_h, dilation_w, deformable_group):
    """Drop-in for ``_ext.dcn_v2_forward`` (DCNv2/src/dcn_v2.h:9-23): NCHW in, new NCHW tensor out."""
    for t in (input, weight, bias, offset, mask):
        if not (t.is_cuda and t.dtype == torch.float32):
            raise RuntimeError("dcn_v2_forward: tensors must be float32 on the GPU")
    input, weight, bias, offset, mask = (t.contiguous() for t in (input, weight, bias, offset, mask))
    b, c, h, w = input.shape
    co, ci, kh, kw = weight.shape
    if (kh, kw) != (kernel_h, kernel_w):
        raise RuntimeError(f"Input shape and kernel shape wont match: ({kernel_h} x {kernel_w} vs {kh} x {kw}).")
    if ci != c:
        raise RuntimeError(f"Input shape and kernel channels wont match: ({c} vs {ci}).")
    ho = (h + 2 * pad_h - (dilation_h * (kernel_h - 1) + 1)) // stride_h + 1
    wo = (w + 2 * pad_w - (dilation_w * (kernel_w - 1) + 1)) // stride_w + 1
    out = torch.empty(b, co, ho, wo, device=input.device, dtype=torch.float32)
    lib = L.lib()
    dims = (b, c, h, w, co, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
            deformable_group)
    nbytes = lib.stif_dcn_v2_workspace_size(*dims)
    ws = torch.empty(max(nbytes // 4, 1), device=input.device, dtype=torch.float32)
    L.check(lib.stif_dcn_v2_forward(_vp(input), _vp(weight), _vp(bias), _vp(offset), _vp(mask), _vp(out), *dims,
                                    _vp(ws), nbytes, _stream()), "dcn_v2_forward")
    return out


def dcn_v2_backward(input, weight, bias, offset, mask, grad_output, kernel_h, kernel_w, stride_h, stride_w, pad_h,
                    pad_w, dilation_h, dilation_w, deformable_group):
    """Drop-in for ``_ext.dcn_v2_backward`` (DCNv2/src/dcn_v2.h:39-52): returns new tensors
    (grad_input, grad_offset, grad_mask, grad_weight, grad_bias) in that order, as
    ``_DCNv2.backward`` (DCNv2/dcn_v2.py:31-45) unpacks them."""
    ts = (input, weight, bias, offset, mask, grad_output)
    for t in ts:
        if not (t.is_cuda and t.dtype == torch.float32):
            raise RuntimeError("dcn_v2_backward: tensors must be float32 on the GPU")
    input, weight, bias, offset, mask, grad_output = (t.contiguous() for t in ts)
    b, c, h, w = input.shape
    co, ci, kh, kw = weight.shape
    if (kh, kw) != (kernel_h, kernel_w):
        raise RuntimeError(f"Input shape and kernel shape wont match: ({kernel_h} x {kernel_w} vs {kh} x {kw}).")
    if ci != c:
        raise RuntimeError(f"Input shape and kernel channels wont match: ({c} vs {ci}).")
    grads = [torch.empty_like(t) for t in (input, offset, mask, weight, bias)]
    lib = L.lib()
    dims = (b, c, h, w, co, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
            deformable_group)
    nbytes = lib.stif_dcn_v2_backward_workspace_size(*dims)
    ws = torch.empty(max(nbytes // 4, 1), device=input.device, dtype=torch.float32)
    L.check(lib.stif_dcn_v2_backward(*[_vp(t) for t in (input, weight, bias, offset, mask, grad_output)],
                                     *[_vp(g) for g in grads], *dims, _vp(ws), nbytes, _stream()), "dcn_v2_backward")
    return tuple(grads)


class DecTablesDev:
    """Device copies of coords.dec_tables(h, w, HH, WW[, shift]) + the C struct pointing at them.
    With a shift (local ensemble) the HR remap tables are set too."""

    def __init__(self, h, w, HH, WW, device="cuda", shift=None):
        tab = dec_tables(h, w, HH, WW, shift)
        keys = TABLE_ORDER + (["hr_y", "hr_x"] if shift is not None else [])
        self._t = {k: torch.from_numpy(np.ascontiguousarray(tab[k])).to(device) for k in keys}
        self.c = L.DecTables(*[self._t[k].data_ptr() for k in keys])
        self.shape = (h, w, HH, WW)


class DecImageDev:
    """decoding_test's HRinp: the x`s` bilinear upsample of the frame pair ([n, s*h, s*w, 8] NHWC on
    the device, stif_upsample_image) and its bilinear tables at the HR query grid (HH, WW)."""

    def __init__(self, x_nchw, s, HH, WW):
        n, _, _, h, w = x_nchw.shape
        self.img = torch.empty(n, s * h, s * w, 8, device=x_nchw.device, dtype=torch.float32)
        L.check(L.lib().stif_upsample_image(_vp(x_nchw), _vp(self.img), n, h, w, s, _stream()), "stif_upsample_image")
        t = dec_tables(s * h, s * w, HH, WW)
        keys = ["b0_y", "b1_y", "w0_y", "w1_y", "b0_x", "b1_x", "w0_x", "w1_x"]
        self._t = {k: torch.from_numpy(np.ascontiguousarray(t[k])).to(x_nchw.device) for k in keys}
        self.c = L.DecImage(self.img.data_ptr(), s * h, s * w, *[self._t[k].data_ptr() for k in keys])


def dec_blend4(preds, weights, out):
    """out = sum_k preds[k] * weights[k] (per HR pixel), the local ensemble's area blend."""
    n, _, HH, WW = out.shape
    pp = (C.c_void_p * 4)(*[_vp(p) for p in preds])
    ww = (C.c_void_p * 4)(*[_vp(w_) for w_ in weights])
    L.check(L.lib().stif_dec_blend4(pp, ww, _vp(out), n, HH, WW, _stream()), "stif_dec_blend4")


def dec_pack_lr(f0, f1, f2, x, out):
    n, h, w, _ = f0.shape
    L.check(L.lib().stif_dec_pack_lr(_vp(f0), _vp(f1), _vp(f2), _vp(x), _vp(out), n, h, w, _stream()),
            "stif_dec_pack_lr")


def dec_stage1(proj, mlp, tables: DecTablesDev, t, hrfeat, flow, image: "DecImageDev" = None, flags=0, status=None):
    n, h, w, _ = proj.shape
    HH, WW = hrfeat.shape[1:3]
    tr = TRACE
    if tr is not None:   # per HR px: feat_imnet layers 1-3 (36,864 MAC) + flow_imnet HRfeat/1-3 (25,600 MAC)
        tr.begin(("dec1",), 2.0 * 62464 * n * HH * WW)
    L.check(L.lib().stif_dec_stage1_ex(_vp(proj), _vp(mlp), C.byref(tables.c), C.byref(image.c) if image else None,
                                       _vp(t), _vp(hrfeat), _vp(flow), n, h, w, HH, WW, flags, _vp(status), _stream()),
            "stif_dec_stage1")
    if tr is not None:
        tr.end()


def dec_stage2(proj, mlp, hrfeat, flow, tables: DecTablesDev, t, out, image: "DecImageDev" = None, flags=0,
               status=None):
    n, h, w, _ = proj.shape
    HH, WW = hrfeat.shape[1:3]
    tr = TRACE
    if tr is not None:   # per HR px: encode_imnet HRfeat part + layers 1-4 (94,976 MAC)
        tr.begin(("dec2",), 2.0 * 94976 * n * HH * WW)
    L.check(L.lib().stif_dec_stage2_ex(_vp(proj), _vp(mlp), _vp(hrfeat), _vp(flow), C.byref(tables.c),
                                       C.byref(image.c) if image else None, _vp(t), _vp(out), n, h, w, HH, WW, flags,
                                       _vp(status), _stream()), "stif_dec_stage2")
    if tr is not None:
        tr.end()
