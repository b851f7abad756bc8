"""The decoder LR projection (200 -> 256) and the 1x1 cat convs (fusion / conv_1x1, (64 | 64) -> 64): direct fp32-MFMA kernel
(k_conv) vs k_conv1x1 (split-fp16), HIP-event time per launch and algorithmic GB/s."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
rng = np.random.default_rng(0)
# the decoder's LR projection 200 -> 256 at C0 (6 pairs at 128 x 128)
xs = torch.randn(6, 128, 128, 200, device="cuda")
wp = (rng.standard_normal((256, 200, 1, 1)) * 0.05).astype(np.float32)
bp = rng.standard_normal(256).astype(np.float32)
op = torch.empty(6, 128, 128, 256, device="cuda")
for name, mode in (("direct f32", L.PACK_PLAIN), ("k_conv1x1 f16x3", L.PACK_PLAIN | L.PACK_F16X3)):
    lay = ops.pack_conv(wp, bp, mode)
    for _ in range(3):
        ops.conv2d([dict(layer=lay, in0=xs, out=op)])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        ops.conv2d([dict(layer=lay, in0=xs, out=op)])
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"LR projection 6x128x128 200->256 {name:16s} {us:8.1f} us  {6 * 128 * 128 * (800 + 1024) / us / 1e3:7.1f} GB/s",
          flush=True)
for G, N, H, W in ((4, 6, 128, 128), (1, 6, 128, 128), (1, 18, 256, 256)):
    x0 = torch.randn(N, H, W, 64, device="cuda")
    x1 = torch.randn(N, H, W, 64, device="cuda")
    w = (rng.standard_normal((64, 128, 1, 1)) * 0.05).astype(np.float32)
    b = rng.standard_normal(64).astype(np.float32)
    out = torch.empty(G, N, H, W, 64, device="cuda")
    for name, mode in (("direct f32", L.PACK_PLAIN), ("k_conv1x1 f16x3", L.PACK_PLAIN | L.PACK_F16X3)):
        lay = ops.pack_conv(w, b, mode)
        grp = [dict(layer=lay, in0=x0, in1=x1, out=out[g]) for g in range(G)]
        for _ in range(3):
            ops.conv2d(grp, in1_mode=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.conv2d(grp, in1_mode=1)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        nb = G * N * H * W * (512 + 256)
        print(f"G={G} N={N} {H}x{W} {name:16s} {us:8.1f} us  {nb / us / 1e3:7.1f} GB/s algorithmic", flush=True)
