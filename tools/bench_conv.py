"""Time the direct and Winograd 3x3 conv kernels on the C1 trunk shape (18 x 256 x 256 x 64)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
N, H, W = int(os.environ.get("N", 18)), int(os.environ.get("HW", 256)), int(os.environ.get("HW", 256))
rng = np.random.default_rng(0)
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32)
x = torch.randn(N, H, W, 64, device="cuda")
r = torch.randn(N, H, W, 64, device="cuda")
flop = 2.0 * 64 * 64 * 9 * N * H * W
ONLY = os.environ.get("ONLY")
for name, mode in (("direct", L.PACK_PLAIN), ("wino", L.PACK_WINO), ("wino16", L.PACK_WINO | L.PACK_F16X3)):
    if ONLY and name != ONLY:
        continue
    lay = ops.pack_conv(w, b, mode)
    out = torch.empty(N, H, W, 64, device="cuda")
    for epi in (L.EPI_RES, L.EPI_RELU):
        def run():
            ops.conv2d([dict(layer=lay, in0=x, out=out, res=r)], epi=epi)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"{name:7s} epi={epi} {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TFLOP/s (direct-equivalent)")
lw = ops.pack_conv(w, b, L.PACK_WINO)
ld = ops.pack_conv(w, b)
o1, o2 = torch.empty(N, H, W, 64, device="cuda"), torch.empty(N, H, W, 64, device="cuda")
ops.conv2d([dict(layer=lw, in0=x, out=o1, res=r)], epi=L.EPI_RES)
ops.conv2d([dict(layer=ld, in0=x, out=o2, res=r)], epi=L.EPI_RES)
print("max |wino - direct| / max|direct|:", float((o1 - o2).abs().max() / o2.abs().max()))
