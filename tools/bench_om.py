"""Time the offset/mask conv (64 -> 216, EPI_OFFMASK) on C1-like launch shapes, f16x3 Winograd."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
rng = np.random.default_rng(0)
for (G, N, H, W) in ((2, 6, 256, 256), (8, 6, 256, 256), (2, 6, 128, 128), (8, 6, 64, 64)):
    ws = [(rng.standard_normal((216, 64, 3, 3)) * 0.05).astype(np.float32) for _ in range(G)]
    bs = [rng.standard_normal(216).astype(np.float32) for _ in range(G)]
    lays = [ops.pack_conv(w, b, L.PACK_WINO_OFFMASK | L.PACK_F16X3) for w, b in zip(ws, bs)]
    x = torch.randn(G, N, H, W, 64, device="cuda")
    out = torch.empty(G, N, H, W, 216, device="cuda")
    flop = 2.0 * 216 * 64 * 9 * G * N * H * W

    def run():
        ops.conv2d([dict(layer=lays[g], in0=x[g], out=out[g]) for g in range(G)], epi=L.EPI_OFFMASK)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"offmask G={G} N={N} {H}x{W}: {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TFLOP/s direct-equiv "
          f"({flop / ms / 1e9 / 1875:.3f} of the f16x3 Winograd peak)")
