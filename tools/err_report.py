"""Accuracy report of the two Winograd operand modes (f32 MFMA vs f16x3 split) on the GPU:
per-conv relative error against the fp64 oracle and end-to-end error against the golden
fixtures (reference model output) and the oracle.  Prints one line per check."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import stif_pkg  # noqa: E402
from oracle import stif_oracle as O  # noqa: E402

S = stif_pkg.load()
L, ops = S._lib, S.ops
rng = np.random.default_rng(0)


def nhwc(x):
    return torch.from_numpy(np.ascontiguousarray(x.transpose(0, 2, 3, 1))).cuda()


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / np.abs(b).max())


x = rng.standard_normal((2, 64, 32, 64)).astype(np.float32) * 0.5
w = (rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32) * 0.1
ref = O.conv2d(x.astype(np.float64), w.astype(np.float64), b.astype(np.float64))
for name, pf in (("f32", 0), ("f16x3", L.PACK_F16X3)):
    for sc in (1.0, 1e-2, 1e2):
        o = torch.empty(2, 32, 64, 64, device="cuda")
        ops.conv2d([dict(layer=ops.pack_conv(w, b * sc, L.PACK_WINO | pf), in0=nhwc(x * sc), out=o)])
        print(f"conv 64->64 {name:6s} input scale {sc:g}: rel err {rel(o.cpu().numpy().transpose(0, 3, 1, 2), ref * sc):.3e}")
o = torch.empty(2, 32, 64, 64, device="cuda")
ops.conv2d([dict(layer=ops.pack_conv(w, b), in0=nhwc(x), out=o)])
print(f"conv 64->64 direct f32: rel err {rel(o.cpu().numpy().transpose(0, 3, 1, 2), ref):.3e}")

sd = S.weights.make_state_dict(seed=0)
g = np.load(os.path.join(REPO, "tests", "golden", "model_16x20.npz"))
xr = rng.random((1, 2, 3, 32, 48)).astype(np.float32)
oref = O.forward(xr, [0.3], sd)[0]
for mode in ("f32", "f16x3"):
    m = S.LunaTokis(64, 6, 8, 5, 40, mfma=mode)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    with torch.no_grad():
        outs = m(torch.from_numpy(g["x"]).cuda(), [torch.tensor([[float(t)]]) for t in g["times"]])
        feat = m.feat.cpu().numpy()[0]
        o2 = m(torch.from_numpy(xr).cuda(), [0.3])[0].cpu().numpy()
    errs = [np.abs(o.cpu().numpy()[0] - g["out"][i]).max() / np.abs(g["out"][i]).max() for i, o in enumerate(outs)]
    print(f"model {mode:6s} 16x20 feat rel {rel(feat, g['feat']):.3e}  outputs rel max {max(errs):.3e} "
          f"(bar 1e-4)  32x48 vs oracle rel {rel(o2, oref):.3e}")
