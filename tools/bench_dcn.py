"""Time the fused DCN kernel (stif_dcn_nhwc) on the C1 PCD L1 shape (12 x 256 x 256 x 64, offsets of
a few pixels)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
N, H, W = int(os.environ.get("N", 12)), 256, 256
rng = np.random.default_rng(0)
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32)
x = torch.randn(N, H, W, 64, device="cuda")
om = torch.randn(N, H, W, 216, device="cuda") * 2.0
om.view(N, H, W, 72, 3)[..., 2].sigmoid_()
lay = ops.pack_conv(w, b)
out = torch.empty(N, H, W, 64, device="cuda")
flop = 2.0 * 64 * 64 * 9 * N * H * W
for _ in range(3):
    ops.dcn([dict(layer=lay, inp=x, offmask=om, out=out)])
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    ops.dcn([dict(layer=lay, inp=x, offmask=om, out=out)])
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(f"dcn {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TFLOP/s")
