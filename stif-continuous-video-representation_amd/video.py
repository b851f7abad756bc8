"""custom_video_test-style driver (codes/custom_video_test.py:41-110) on the engine.

``single_forward`` keeps the harness's behaviour: zero-pad H, W up to a multiple
of 4 on the bottom/right (:44-48), query the eight times i/8 (:50), return the
uncropped [1,3,4h_n,4w_n] outputs.  ``run_sequence`` is the harness's pair loop
(:81-97) as one batched window: every adjacent pair of a frame sequence, with the
per-frame encoder shared between the two pairs that use a frame.
"""
from __future__ import annotations

import math

import torch

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
