"""Host-side query-grid tables of the implicit decoder, in the reference's fp32.

``LunaTokis.decoding`` (Sakuya_arch_test.py:364-459) samples the LR maps at
``coord_highres = make_coord((HH, WW)).clamp(-1+1e-6, 1-1e-6)`` (:373): a
separable meshgrid, so every discrete decision (nearest index with
round-half-to-even, bilinear corners) and every coordinate-derived value
(``rel_coord``, the ``warpgrid`` linspace base) depends on the HR row or column
only.  They are computed here once per (h, w, HH, WW) in float32 with the same
operation order as the reference (make_coord :1233-1248, grid_sample's
``((x + 1) * size - 1) / 2`` unnormalisation, torch.linspace), then uploaded;
the kernels only look them up.  This is what makes non-integer scales (2.5x,
where nearest-rounding ties occur) match the reference exactly.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
LO = F32(-1 + 1e-6)
HI = F32(1 - 1e-6)


def make_coord_1d(n: int) -> np.ndarray:
    """One axis of make_coord: fp32(-1 + r) + fp32(2r) * arange(n).float(), r = 1/n."""
    r = 2.0 / (2 * n)
    return (F32(2 * r) * np.arange(n, dtype=F32)).astype(F32) + F32(-1 + r)


def linspace_f32(n: int) -> np.ndarray:
    """torch.linspace(-1, 1, n) in fp32 (the warpgrid base grid, warplayer.py:27-31)."""
    if n == 1:
        return np.array([-1.0], F32)
    step = F32(2.0 / (n - 1))
    i = np.arange(n)
    lo = (F32(-1.0) + step * i.astype(F32)).astype(F32)
    hi = (F32(1.0) - step * (n - 1 - i).astype(F32)).astype(F32)
    return np.where(i < n // 2, lo, hi).astype(F32)


def _unnorm(c: np.ndarray, size: int) -> np.ndarray:
    return ((c + F32(1)) * F32(size) - F32(1)) / F32(2)


def axis_table(n_lr: int, n_hr: int, shift: float = 0.0) -> dict:
    """Per-HR-index sampling data along one axis (rows: n = H, HH; cols: n = W, WW).
    shift: the local ensemble's query offset v * (2 / n_lr / 2) + 1e-6 (Sakuya_arch_test.py:
    994-998), added in fp32 and re-clamped; rel_coord keeps the unshifted query (:1000-1002) and
    ``hr`` is the HR pixel nearest to the shifted query (grid_sample nearest of HRfeat, :1022)."""
    c = np.clip(make_coord_1d(n_hr), LO, HI)
    s = c if shift == 0.0 else np.clip((c + F32(shift)).astype(F32), LO, HI)
    lr_c = make_coord_1d(n_lr)
    src = _unnorm(s, n_lr)
    near = np.clip(np.rint(src), 0, n_lr - 1).astype(np.int32)      # nearest (round half even)
    rel = ((c - lr_c[near]) * F32(n_lr)).astype(F32)                  # rel_coord (:394-396)
    f0 = np.floor(src)
    i0 = f0.astype(np.int64)
    i1 = i0 + 1
    w1 = (src - f0).astype(F32)
    w0 = ((f0 + F32(1)) - src).astype(F32)
    v0 = (i0 >= 0) & (i0 < n_lr)
    v1 = (i1 >= 0) & (i1 < n_lr)
    return dict(
        near=near, rel=rel,
        b0=np.clip(i0, 0, n_lr - 1).astype(np.int32), b1=np.clip(i1, 0, n_lr - 1).astype(np.int32),
        w0=np.where(v0, w0, F32(0)).astype(F32), w1=np.where(v1, w1, F32(0)).astype(F32),
        lin=linspace_f32(n_hr),
        hr=np.clip(np.rint(_unnorm(s, n_hr)), 0, n_hr - 1).astype(np.int32),
    )


def dec_tables(h: int, w: int, HH: int, WW: int, shift=None) -> dict:
    """Tables of one decode; shift = (vx, vy) of the local ensemble (rows move by vx/h, cols by vy/w)."""
    sy, sx = (0.0, 0.0) if shift is None else (shift[0] * (2 / h / 2) + 1e-6, shift[1] * (2 / w / 2) + 1e-6)
    ty = axis_table(h, HH, sy)
    tx = axis_table(w, WW, sx)
    out = {}
    for k, v in ty.items():
        out[("near" if k == "near" else k) + "_y"] = v
    for k, v in tx.items():
        out[k + "_x"] = v
    return out


TABLE_ORDER = ["near_y", "rel_y", "b0_y", "b1_y", "w0_y", "w1_y", "lin_y",
               "near_x", "rel_x", "b0_x", "b1_x", "w0_x", "w1_x", "lin_x"]


def ensemble_weights(h: int, w: int, HH: int, WW: int) -> list:
    """Per-HR-pixel blend weights of decoding_localensemble (:1003-1004, 1075-1084), in fp32 and the
    reference's order: area_k = |rel_y rel_x| + 1e-9 for shifts (vx, vy) in (-1,-1), (-1,1), (1,-1),
    (1,1); tot = sum of the four; decode k is weighted by the diagonally opposite area / tot."""
    areas = []
    for vx in (-1, 1):
        for vy in (-1, 1):
            t = dec_tables(h, w, HH, WW, (vx, vy))
            areas.append((np.abs(np.outer(t["rel_y"], t["rel_x"]).astype(F32)) + F32(1e-9)).astype(F32))
    tot = (((areas[0] + areas[1]).astype(F32) + areas[2]).astype(F32) + areas[3]).astype(F32)
    return [(areas[3 - k] / tot).astype(F32) for k in range(4)]
