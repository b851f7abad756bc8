"""k_wino vs k_wino_sp (STIF_WINO_SP) on the C0 trunk shape (18 x 128 x 128 x 64, RES / RELU) and the PCD cat
shape (2 groups x 6 x 128 x 128, 64 | 64 -> 64, LRELU), alternating in one process; HIP-event times per launch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
rng = np.random.default_rng(0)
REPS = int(os.environ.get("REPS", 3))


def case_trunk(epi):
    N, H, W = 18, 128, 128
    x = torch.randn(N, H, W, 64, device="cuda")
    r = torch.randn(N, H, W, 64, device="cuda")
    lay = ops.pack_conv((rng.standard_normal((64, 64, 3, 3)) * 0.05).astype(np.float32),
                        rng.standard_normal(64).astype(np.float32), L.PACK_WINO | L.PACK_F16X3)
    out = torch.empty(N, H, W, 64, device="cuda")
    return lambda: ops.conv2d([dict(layer=lay, in0=x, out=out, res=r)], epi=epi), out


def case_cat():
    N, H, W = 6, 128, 128
    ents = []
    for g in range(2):
        lay = ops.pack_conv((rng.standard_normal((64, 128, 3, 3)) * 0.03).astype(np.float32),
                            rng.standard_normal(64).astype(np.float32), L.PACK_WINO | L.PACK_F16X3)
        ents.append(dict(layer=lay, in0=torch.randn(N, H, W, 64, device="cuda"),
                         in1=torch.randn(N, H, W, 64, device="cuda"), out=torch.empty(N, H, W, 64, device="cuda")))
    return lambda: ops.conv2d(ents, epi=L.EPI_LRELU, in1_mode=1), ents[0]["out"]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


cases = {"trunk_res": case_trunk(L.EPI_RES), "trunk_relu": case_trunk(L.EPI_RELU), "cat_lrelu": case_cat()}
for name, (fn, out) in cases.items():
    res = {}
    for rep in range(REPS):
        for sp in ("0", "1"):
            os.environ["STIF_WINO_SP"] = sp
            res.setdefault(sp, []).append(timeit(fn))
    os.environ["STIF_WINO_SP"] = "0"
    fn()
    a = out.clone()
    os.environ["STIF_WINO_SP"] = "1"
    fn()
    same = bool(torch.equal(a, out))
    print(f"{name:12s} k_wino {' '.join(f'{v:7.1f}' for v in res['0'])} us | k_wino_sp "
          f"{' '.join(f'{v:7.1f}' for v in res['1'])} us | bit-identical {same}", flush=True)
