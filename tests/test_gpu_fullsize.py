"""Full-size decodes pinned to the oracle at sampled pixels (BASELINE configs C2, C3 and C4).

The engine's latent at 540x960 (C2, 4x, 3 t) and 1080x1920 (C4, 2.5x -> 2700x4800, 4 t) is decoded
on the GPU over the whole frame; the oracle's pixel-subset decoder (``decoding_at``: the reference
decoder, Sakuya_arch_test.py:364-459 with warplayer.py:25-39, evaluated only where asked) decodes
the same latent at ~4,096 HR pixels: random ones, the first and last row and column (where outward
flows clamp the warped grid), and -- at 2.5x -- the rows and columns whose nearest LR index is a
round-half-even tie.  Elementwise |gpu - oracle| <= 1e-4 |oracle| + 1e-6 (north star rtol 1e-4), so
the full-size decoder is pinned to the reference arithmetic, not only to the other operand mode.
C3 decodes a whole 9-frame 720p window (8 pairs) and pins its LAST pair: item 7's HRfeat starts
7 x 2880 x 5120 x 64 x 4 B = 26 GB into the buffer, beyond 2^32 bytes, so the decoder's 64-bit item
offsets are checked against the oracle too (missing 4).
The encoder at these sizes is covered by test_gpu_configs (f16x3 vs fp32) and, at sizes the oracle
runs in seconds, by the reference fixtures.
"""
import numpy as np
import pytest
import torch

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-4, 1e-6


def synth(first, count, H, W):
    out = torch.empty(count, 3, H, W)
    for i in range(count):
        out[i] = torch.rand(3, H, W, generator=torch.Generator().manual_seed(1234 + first + i))
    return out.cuda()


def tie_indices(n_hr, n_lr):
    """HR rows/columns whose grid_sample-nearest source index ((c + 1) n - 1) / 2 is an exact .5 tie"""
    c = np.clip(O.make_coord_1d(n_hr), np.float32(-1 + 1e-6), np.float32(1 - 1e-6))
    src = ((c + np.float32(1)) * np.float32(n_lr) - np.float32(1)) / np.float32(2)
    return np.nonzero(src - np.floor(src) == np.float32(0.5))[0]


def pick_pixels(HH, WW, H, W, n=4096, seed=0):
    rng = np.random.default_rng(seed)
    ys, xs = [], []

    def add(y, x):
        ys.append(np.asarray(y, np.int64))
        xs.append(np.asarray(x, np.int64))
    k = n // 16
    add([0, 0, HH - 1, HH - 1], [0, WW - 1, 0, WW - 1])                                  # corners
    add(np.full(k, HH - 1), rng.integers(0, WW, k))                                      # last row
    add(rng.integers(0, HH, k), np.full(k, WW - 1))                                      # last column
    add(np.zeros(k, np.int64), rng.integers(0, WW, k))                                   # first row
    add(rng.integers(0, HH, k), np.zeros(k, np.int64))                                   # first column
    ty, tx = tie_indices(HH, H), tie_indices(WW, W)
    if len(ty):
        add(rng.choice(ty, 2 * k), rng.integers(0, WW, 2 * k))                           # tie rows
        add(rng.choice(ty, k), rng.choice(tx, k) if len(tx) else rng.integers(0, WW, k))  # tie x tie
    if len(tx):
        add(rng.integers(0, HH, 2 * k), rng.choice(tx, 2 * k))                           # tie columns
    m = n - sum(len(y) for y in ys)
    add(rng.integers(0, HH, m), rng.integers(0, WW, m))                                  # anywhere
    return np.concatenate(ys), np.concatenate(xs), len(ty), len(tx)


CASES = {
    # frames, H, W, output size (None = 4x), times
    "C2": (3, 540, 960, None, [0.25, 0.5, 0.75]),
    "C3": (9, 720, 1280, None, [0.0, 0.5]),
    "C4": (2, 1080, 1920, (2700, 4800), [0.0, 0.25, 0.5, 0.75]),
}


@pytest.mark.parametrize("cfg", sorted(CASES))
def test_full_size_decode_matches_oracle_at_pixels(stif, sd, cfg):
    F_, H, W, size, times = CASES[cfg]
    HH, WW = size or (4 * H, 4 * W)
    m = stif.LunaTokis(64, 6, 8, 5, 40)
    m.load_state_dict(sd, strict=True)
    if cfg == "C3":
        # one decode pass over all 8 items (the default dec_chunk_px would split them 2 per pass), so the
        # HRfeat / flow scratch holds the whole window and item 7 sits 26 GB (> 2^32 B) into it
        m.dec_chunk_px = (F_ - 1) * HH * WW
        assert (F_ - 2) * HH * WW * 64 * 4 > 2 ** 32
    fr = synth(0, F_, H, W)
    with torch.no_grad():
        m.gen_feat_window(fr)
        outs = m.decoding([torch.tensor([[t]]) for t in times], size)
    py, px, nty, ntx = pick_pixels(HH, WW, H, W)
    if size is not None:
        assert nty > 0 and ntx > 0          # 1080 -> 2700 and 1920 -> 4800 both have ties
    b = F_ - 2                              # the last pair of the window (C3: item 7, past 2^32 bytes of HRfeat)
    feat = m.feat[b:b + 1].cpu().numpy()    # [1,3,64,H,W], a strided view of the NHWC latent
    x = m.inp[b:b + 1].cpu().numpy()
    st = {}
    ref = O.decoding_at(feat, x, times, sd, HH, WW, py, px, stats=st)
    assert st["clamped"] > 0                # some warped samples leave the frame
    iy, ix = torch.from_numpy(py).cuda(), torch.from_numpy(px).cuda()
    for t, o, r in zip(times, outs, ref):
        assert tuple(o.shape) == (F_ - 1, 3, HH, WW)
        got = o[b][:, iy, ix].double().cpu().numpy()
        d = np.abs(got - r[0])
        lim = RTOL * np.abs(r[0]) + ATOL
        assert (d <= lim).all(), (cfg, t, float((d / lim).max()), float(d.max()))
