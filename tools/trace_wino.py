"""Per-wave s_memtime trace of the Winograd conv (kernel-experiment build with -DWINO_EXP_TRACE):
average cycles of each segment between trace points, per wave role.  STIF_HIP_LIB must point at
the trace build.  Tags: 1 tile start, 6 before a phase barrier, 2 after it, 3 after the exchange
barrier, 4 after the second epilogue barrier, 5 end of the tile's stores."""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
N, H, W = int(os.environ.get("N", 18)), 256, 256
EPI = int(os.environ.get("EPI", L.EPI_RELU))
rng = np.random.default_rng(0)
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32)
x = torch.randn(N, H, W, 64, device="cuda")
r = torch.randn(N, H, W, 64, device="cuda")
lay = ops.pack_conv(w, b, L.PACK_WINO)
out = torch.empty(N, H, W, 64, device="cuda")
for _ in range(3):
    ops.conv2d([dict(layer=lay, in0=x, out=out, res=r)], epi=EPI)
torch.cuda.synchronize()
buf = np.zeros(512 * 4 * 128, dtype=np.uint64)
lib = L.lib()
lib.stif_exp_wino_trace.argtypes = [C.c_void_p]
assert lib.stif_exp_wino_trace(buf.ctypes.data) == 0
tr = buf.reshape(512, 4, 128)
seg = defaultdict(list)
for blk in range(512):
    for wv in range(4):
        ev = [(int(v) >> 8, int(v) & 0xFF) for v in tr[blk, wv] if v]
        for (t0, a), (t1, bb) in zip(ev, ev[1:]):
            seg[(wv, a, bb)].append(t1 - t0)
names = {1: "start", 6: "pre-bar", 2: "post-bar", 3: "xchg", 4: "comb", 5: "stored"}
tot = defaultdict(float)
for k in sorted(seg):
    v = np.array(seg[k])
    print(f"wave {k[0]} {names[k[1]]:>8s} -> {names[k[2]]:<8s} n={len(v):5d} avg {v.mean():8.0f} med {np.median(v):8.0f} cyc")
# per-tile period
for wv in range(4):
    st = [int(v) >> 8 for v in tr[:, wv].reshape(-1) if v and (int(v) & 0xFF) == 1]
print("MFMA cycles per tile per wave at peak: 256 x 64 =", 256 * 64)
