"""Per-wave s_memtime trace of the f16x3 Winograd conv (tools/exp_trace.so, built by
tools/experiments/make_wino_trace.py): average cycles of each segment between trace points per wave,
and for the two waves that share a SIMD, how much of the time at least one of them is inside a phase
(MFMA stream).  Tags: 1 tile start, 6 before a phase's wait+barrier, 2 after it, 3 after an exchange
barrier, 5 before the closing barrier, 4 after it, 7 tile setup done.  Env: N, HW (trunk shape N x HW x HW x 64), EPI."""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("STIF_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tools", "exp_trace.so"))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
N, H = int(os.environ.get("N", 18)), int(os.environ.get("HW", 128))
W = H
EPI = int(os.environ.get("EPI", L.EPI_RELU))
rng = np.random.default_rng(0)
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32)
x = torch.randn(N, H, W, 64, device="cuda")
r = torch.randn(N, H, W, 64, device="cuda")
lay = ops.pack_conv(w, b, L.PACK_WINO | L.PACK_F16X3)
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
simd = defaultdict(list)   # placement -> list of (block, wave)
for blk in range(512):
    for wv in range(4):
        ev = [(int(v) >> 8, int(v) & 0xFF) for v in tr[blk, wv, :127] if v]
        for (t0, a), (t1, bb) in zip(ev, ev[1:]):
            seg[(wv, a, bb)].append(t1 - t0)
        hw = int(tr[blk, wv, 127])
        xcc, hid = hw >> 32, hw & 0xFFFFFFFF
        simd[(xcc & 0xF, (hid >> 8) & 0xF, (hid >> 12) & 1, (hid >> 13) & 7, (hid >> 4) & 3)].append((blk, wv))
names = {1: "start", 6: "pre-bar", 2: "post-bar", 3: "xchg", 4: "end-bar", 5: "stored", 7: "setup", 8: "sp0", 9: "sp1"}
for k in sorted(seg):
    v = np.array(seg[k])
    print(f"wave {k[0]} {names[k[1]]:>8s} -> {names[k[2]]:<8s} n={len(v):5d} avg {v.mean():8.0f} med {np.median(v):8.0f} cyc")
print("MFMA cycles per tile per wave at peak (C0 = 64 -> 64):", 96 * 32)


def phase_intervals(blk, wv):
    """[start, end) intervals in which the wave runs a phase: tag 1 or 2 -> next tag 6"""
    ev = [(int(v) >> 8, int(v) & 0xFF) for v in tr[blk, wv, :127] if v]
    iv = []
    for (t0, a), (t1, bb) in zip(ev, ev[1:]):
        if a in (7, 2) and bb == 8:
            iv.append((t0, t1))
    return iv, (ev[0][0], ev[-1][0]) if ev else (0, 0)


sizes = defaultdict(int)
both_idle = tot = 0.0
for key, members in simd.items():
    sizes[len(members)] += 1
    if len(members) != 2:
        continue
    (i1, s1), (i2, s2) = [phase_intervals(*m) for m in members]
    lo, hi = max(s1[0], s2[0]), min(s1[1], s2[1])
    if hi <= lo:
        continue
    grid = np.zeros(int(hi - lo) // 16 + 1, bool)
    for iv in (i1, i2):
        for a0, a1 in iv:
            a0, a1 = max(a0, lo), min(a1, hi)
            if a1 > a0:
                grid[int(a0 - lo) // 16:int(a1 - lo) // 16] = True
    both_idle += (~grid).sum()
    tot += grid.size
print("waves per SIMD histogram:", dict(sizes))
print(f"fraction of the common window with NEITHER wave of a SIMD inside a phase: {both_idle / max(tot, 1):.3f}")
