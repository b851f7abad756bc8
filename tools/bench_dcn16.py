"""Time the fused DCN core (k_dcn) in both operand modes on the C1 L1 shape (8 x 256 x 256)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
N, H, W = int(os.environ.get("N", 8)), int(os.environ.get("HW", 256)), int(os.environ.get("HW", 256))
rng = np.random.default_rng(0)
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32)
x = torch.randn(N, H, W, 64, device="cuda")
om = torch.randn(N, H, W, 216, device="cuda") * 2
om.view(N, H, W, 72, 3)[..., 2] = torch.rand(N, H, W, 72, device="cuda")
flop = 2.0 * 64 * 576 * N * H * W
outs = {}
for name, mode in (("f32", L.PACK_PLAIN), ("f16x3", L.PACK_PLAIN | L.PACK_F16X3)):
    lay = ops.pack_conv(w, b, mode)
    out = torch.empty(N, H, W, 64, device="cuda")
    def run():
        ops.dcn([dict(layer=lay, inp=x, offmask=om, out=out)], epi=L.EPI_LRELU)
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
    outs[name] = out
    print(f"dcn {name:6s} {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TFLOP/s")
print("max |f16x3 - f32| / max|f32|:", float((outs["f16x3"] - outs["f32"]).abs().max() / outs["f32"].abs().max()))
