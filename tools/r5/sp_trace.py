"""Per-step s_memtime trace of k_wino_sp (build with -DWINO_SP_TRACE=1, STIF_HIP_LIB): trunk RELU shape,
workgroups 0-7, every wave; prints per-role step durations (stamp after the barrier -> stamp before the
next barrier) and the barrier waits."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
os.environ["STIF_WINO_SP"] = "1"
TR = 96
buf = torch.zeros(8 * 8 * 2 * TR * 64, dtype=torch.int64, device="cuda")
lib = ctypes.CDLL(os.environ["STIF_HIP_LIB"])
lib.stif_wino_sp_trace.argtypes = [ctypes.c_void_p]
assert lib.stif_wino_sp_trace(ctypes.c_void_p(buf.data_ptr())) == 0
rng = np.random.default_rng(0)
N, H, W = 18, 128, 128
x = torch.randn(N, H, W, 64, device="cuda")
lay = ops.pack_conv((rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32),
                    rng.standard_normal(64).astype(np.float32), L.PACK_WINO | L.PACK_F16X3)
out = torch.empty(N, H, W, 64, device="cuda")
epi = getattr(L, os.environ.get("EPI", "EPI_RELU"))
for _ in range(5):
    ops.conv2d([dict(layer=lay, in0=x, out=out, res=x)], epi=epi)
torch.cuda.synchronize()
t = buf.view(8, 8, 2 * TR, 64)[:, :, :, 0].cpu().numpy().astype(np.int64)
nsteps = 38
for wg in range(2):
    base = t[wg, :, 0].min()
    print(f"WG {wg}: per step [T start..end | M start..end] relative cycles (wave 0 = T row 0, wave 4 = M row 0)")
    for n in range(nsteps):
        ts, te = t[wg, 0, 2 * n] - base, t[wg, 0, 2 * n + 1] - base
        ms, me = t[wg, 4, 2 * n] - base, t[wg, 4, 2 * n + 1] - base
        print(f"  step {n:2d}: T {ts:7d}..{te:7d} ({te - ts:5d})  M {ms:7d}..{me:7d} ({me - ms:5d})")
# aggregate over workgroups 0-7: step duration per role, barrier wait = next start - this end
dT = (t[:, :4, 1:2 * nsteps:2] - t[:, :4, 0:2 * nsteps:2]).reshape(-1)
dM = (t[:, 4:, 1:2 * nsteps:2] - t[:, 4:, 0:2 * nsteps:2]).reshape(-1)
step = (t[:, :, 2:2 * nsteps:2] - t[:, :, 0:2 * nsteps - 2:2]).reshape(-1)
print("median T step work", int(np.median(dT)), "M step work", int(np.median(dM)), "step period", int(np.median(step)))
for q in range(4):
    sel = slice(2 * q, 2 * nsteps, 8)
    dq = (t[:, 4:, 2 * q + 1:2 * nsteps:8] - t[:, 4:, 2 * q:2 * nsteps:8]).reshape(-1)
    tq = (t[:, :4, 2 * q + 1:2 * nsteps:8] - t[:, :4, 2 * q:2 * nsteps:8]).reshape(-1)
    print(f"  q={q}: median T {int(np.median(tq))}  M {int(np.median(dq))}")
