"""custom_video_test-style driver (codes/custom_video_test.py:41-110) on the engine.

``single_forward`` keeps the harness's behaviour: zero-pad H, W up to a multiple
of 4 on the bottom/right (:44-48), query the eight times i/8 (:50), return the
uncropped [1,3,4h_n,4w_n] outputs.  ``run_sequence`` is the harness's pair loop
(:81-97) as one batched window: every adjacent pair of a frame sequence, with the
per-frame encoder shared between the two pairs that use a frame.

The harness's data formats either side of the model run on the GPU too:
``resize_frames`` = ``data.util.imresize_np(frame, 1/2, True)`` on cv2-style uint8 BGR frames
+ ``/255`` + BGR->RGB + NCHW (:88-93), ``frames_to_u8`` = ``(clamp(0,1)*255).astype(uint8)`` HWC
(:101-102); ``run_folder`` is the whole script (LR / HR / bicubic outputs, PIL file I/O).
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib as L

HARNESS_TIMES = [i / 8 for i in range(8)]


def pad_to_4(imgs: torch.Tensor) -> torch.Tensor:
    """imgs [..., h, w] -> zero-padded to multiples of 4 (custom_video_test.py:44-48)."""
    h, w = imgs.shape[-2:]
    hn, wn = int(4 * math.ceil(h / 4)), int(4 * math.ceil(w / 4))
    if (hn, wn) == (h, w):
        return imgs
    out = imgs.new_zeros(*imgs.shape[:-2], hn, wn)
    out[..., :h, :w] = imgs
    return out


def single_forward(model, imgs_in: torch.Tensor, times=None):
    """imgs_in [1,2,3,h,w] RGB in [0,1] -> list over times of [1,3,4h_n,4w_n]."""
    with torch.no_grad():
        x = pad_to_4(imgs_in)
        ts = HARNESS_TIMES if times is None else times
        return model(x, [torch.tensor([t])[None] for t in ts])


def run_sequence(model, frames: torch.Tensor, times=None, scale=None):
    """frames [F,3,h,w] -> list over the F-1 pairs of lists over times of [3,HH,WW]."""
    with torch.no_grad():
        fr = pad_to_4(frames)
        model.gen_feat_window(fr)
        ts = HARNESS_TIMES if times is None else times
        preds = model.decoding([torch.tensor([t])[None] for t in ts], scale)
    return [[p[i] for p in preds] for i in range(frames.shape[0] - 1)]


# ----------------------------------------------------------------------------- harness I/O
F32 = np.float32


def _cubic(x):
    ax = np.abs(x).astype(F32)
    ax2 = (ax * ax).astype(F32)
    ax3 = (ax2 * ax).astype(F32)
    a = ((F32(1.5) * ax3 - F32(2.5) * ax2 + F32(1)) * (ax <= 1)).astype(F32)
    b = ((F32(-0.5) * ax3 + F32(2.5) * ax2 - F32(4) * ax + F32(2)) * ((ax > 1) & (ax <= 2))).astype(F32)
    return (a + b).astype(F32)


def resize_tables(in_len: int, out_len: int, scale: float, antialias: bool = True):
    """calculate_weights_indices (data/util.py:248-300) in fp32 -> (weights [out, P], first
    symmetric-padded index per output [out], top/left padding sym_len_s)."""
    kw = 4.0 / scale if (scale < 1 and antialias) else 4.0
    x = np.linspace(1, out_len, out_len, dtype=np.float64).astype(F32)
    u = (x / F32(scale) + F32(0.5 * (1 - 1 / scale))).astype(F32)
    left = np.floor(u - F32(kw / 2)).astype(F32)
    P = int(math.ceil(kw)) + 2
    ind = (left[:, None] + np.arange(P, dtype=F32)[None, :]).astype(F32)
    dist = (u[:, None] - ind).astype(F32)
    w = (F32(scale) * _cubic((dist * F32(scale)).astype(F32))).astype(F32) if (scale < 1 and antialias) else _cubic(dist)
    w = (w / w.sum(1, dtype=F32)[:, None]).astype(F32)
    zeros = (w == 0).sum(0)                     # counted before either narrow (:286-291)
    if zeros[0] != 0:
        ind, w = ind[:, 1:P - 1], w[:, 1:P - 1]
    if zeros[-1] != 0:
        ind, w = ind[:, :P - 2], w[:, :P - 2]
    s0 = int(-ind.min() + 1)
    return np.ascontiguousarray(w, F32), (ind[:, 0] + s0 - 1).astype(np.int32), s0


_RESIZE_CACHE = {}


def resize_frames(frames_bgr_u8, scale: float = 0.5, device="cuda") -> torch.Tensor:
    """imresize_np(frame, scale, True).astype(float32) / 255, BGR -> RGB, HWC -> CHW for a stack of
    cv2-style uint8 BGR frames [n, H, W, 3] (numpy or torch) -> device float [n, 3, oH, oW]."""
    fr = torch.as_tensor(frames_bgr_u8).to(device=device, dtype=torch.uint8).contiguous()
    n, H, W, c = fr.shape
    if c != 3:
        raise ValueError("frames must be [n, H, W, 3] uint8 (BGR, as cv2.imread)")
    oH, oW = int(math.ceil(H * scale)), int(math.ceil(W * scale))
    key = (H, W, scale, str(device))
    if key not in _RESIZE_CACHE:
        wH, iH, sH = resize_tables(H, oH, scale)
        wW, iW, sW = resize_tables(W, oW, scale)
        dev = [torch.from_numpy(a).to(device) for a in (wH, iH, wW, iW)]
        _RESIZE_CACHE[key] = (dev, wH.shape[1], sH, wW.shape[1], sW)
    (twH, tiH, twW, tiW), PH, sH, PW, sW = _RESIZE_CACHE[key]
    out = torch.empty(n, 3, oH, oW, device=device, dtype=torch.float32)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(L.lib().stif_resize_frames(fr.data_ptr(), out.data_ptr(), n, H, W, oH, oW, twH.data_ptr(), tiH.data_ptr(),
                                       PH, sH, twW.data_ptr(), tiW.data_ptr(), PW, sW, st), "stif_resize_frames")
    return out


def frames_to_u8(frames: torch.Tensor) -> torch.Tensor:
    """(clamp(frames, 0, 1) * 255).astype(uint8), NCHW float -> HWC uint8 [n, H, W, 3] on the device."""
    f = frames.contiguous()
    n, c, H, W = f.shape
    if c != 3:
        raise ValueError("frames must be [n, 3, H, W]")
    out = torch.empty(n, H, W, 3, device=f.device, dtype=torch.uint8)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(L.lib().stif_frames_to_u8(f.data_ptr(), out.data_ptr(), n, H, W, st), "stif_frames_to_u8")
    return out


def run_folder(model, in_dir: str, out_dir: str, times=None):
    """custom_video_test.py:60-110 for one folder of frames: every adjacent pair is resized by 1/2
    (imresize_np), run at the eight harness times, and written as JPGs under out_dir/HR; the LR
    frames go to out_dir/LR and the PIL-bicubic x4 baseline to out_dir/bicubic.  Frames are read with
    PIL and flipped to BGR so the data path matches cv2.imread's."""
    from PIL import Image

    names = sorted(os.listdir(in_dir))
    for sub in ("HR", "bicubic", "LR"):
        os.makedirs(os.path.join(out_dir, sub), exist_ok=True)
    idx_hr = idx_bic = 0
    for i in range(len(names) - 1):
        bgr = np.stack([np.asarray(Image.open(os.path.join(in_dir, names[i + k])).convert("RGB"))[:, :, ::-1]
                        for k in range(2)])
        lr = resize_frames(bgr)                                           # [2,3,h,w] RGB
        lr_u8 = frames_to_u8(lr).cpu().numpy()
        Image.fromarray(lr_u8[0]).save(os.path.join(out_dir, "LR", names[i]))
        outs = single_forward(model, lr[None], times)
        hr = frames_to_u8(torch.cat(outs, 0)).cpu().numpy()
        for k in range(hr.shape[0]):
            Image.fromarray(hr[k]).save(os.path.join(out_dir, "HR", f"{idx_hr}.jpg"))
            idx_hr += 1
        h, w = lr_u8.shape[1:3]
        for _ in range(len(outs)):
            Image.fromarray(lr_u8[0]).resize((4 * w, 4 * h), Image.BICUBIC).save(
                os.path.join(out_dir, "bicubic", f"{idx_bic}.jpg"))
            idx_bic += 1
