"""s_memtime trace of the warp-specialised Winograd conv (build with -DWINO_EXP_TRACE): average
cycles between trace points for MFMA wave 0 and helper wave 4.  Tags: 1 tile start, 6 before a phase
barrier, 2 after it, 3 before the P barrier, 4 after it."""
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
names = {1: "start", 6: "pre-bar", 2: "post-bar", 3: "pre-P", 4: "post-P", 7: "epi-done", 8: "dma-issued"}
for role, blocks in (("mfma", range(0, 256)), ("helper", range(256, 512))):
    seg = defaultdict(list)
    for blk in blocks:
        ev = [(int(v) >> 8, int(v) & 0xFF) for v in tr[blk, 0, :127] if v]
        for (t0, a), (t1, bb) in zip(ev, ev[1:]):
            seg[(a, bb)].append(t1 - t0)
    for k in sorted(seg):
        v = np.array(seg[k])
        print(f"{role:6s} {names[k[0]]:>8s} -> {names[k[1]]:<8s} n={len(v):5d} avg {v.mean():8.0f} med {np.median(v):8.0f}")
