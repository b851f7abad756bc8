"""Debug aid: error pattern of the Winograd conv against the oracle (GPU box)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402
from oracle import stif_oracle as O  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
H, W = 8, 32
rng = np.random.default_rng(0)
x = rng.standard_normal((1, 64, H, W)).astype(np.float32)
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = np.zeros(64, np.float32)
ref = O.conv2d(x, w, b)[0].transpose(1, 2, 0)          # [H,W,C]
out = torch.zeros(1, H, W, 64, device="cuda")
ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_WINO), in0=torch.from_numpy(x.transpose(0, 2, 3, 1).copy()).cuda(),
                 out=out)])
o = out[0].cpu().numpy()
err = np.abs(o - ref)
print("max err", err.max(), "max ref", np.abs(ref).max())
print("err per row", err.max(axis=(1, 2)).round(3))
print("err per col", err.max(axis=(0, 2)).round(3))
print("err per ch", err.max(axis=(0, 1)).round(3))
print("zeros in out", int((o == 0).sum()), "of", o.size)
# is the output a permutation? try to find, for a few wrong outputs, the matching ref location
for (yy, xx, cc) in [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (3, 5, 7)]:
    v = o[yy, xx, cc]
    idx = np.argwhere(np.abs(ref - v) < 1e-4)
    print((yy, xx, cc), "out", v, "ref", ref[yy, xx, cc], "matches at", idx[:4].tolist())
