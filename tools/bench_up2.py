"""Time stif_upsample2x_nhwc (x2 bilinear, 64 ch NHWC) on the C1 PCD shapes; STIF_HIP_LIB picks the build."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
for n, h, w in ((48, 128, 128), (48, 64, 64)):
    x = torch.randn(n, h, w, 64, device="cuda")
    out = torch.empty(n, 2 * h, 2 * w, 64, device="cuda")
    for _ in range(3):
        stif.ops.upsample2x(x, out, 2.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        stif.ops.upsample2x(x, out, 2.0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ref = torch.nn.functional.interpolate(x.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                                          align_corners=False).permute(0, 2, 3, 1) * 2.0
    err = float((out - ref).abs().max())
    gbs = 5 * x.numel() * 4 / ms / 1e6
    print(f"up2 {n}x{h}x{w}: {ms * 1e3:7.1f} us  {gbs:7.1f} GB/s  max|out - torch| {err:.2e}")
