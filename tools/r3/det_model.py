"""Diagnose the window-vs-pair mismatch: re-run every fused dcn_sep launch of a C0 window into fresh
buffers and compare bit for bit (kernel race vs launch-level aliasing)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
sd = stif.weights.make_state_dict(seed=0)
fr = torch.empty(7, 3, 128, 128)
for i in range(7):
    fr[i] = torch.rand(3, 128, 128, generator=torch.Generator().manual_seed(1234 + i))
fr = fr.cuda()
ops = stif.ops
orig = ops.dcn_sep
n = [0]
nd = []


def traced(groups, epi=0, status=None):
    orig(groups, epi=epi, status=status)
    outs = [g["out"].clone() for g in groups]
    ptrs = {k: [g[k].data_ptr() for g in groups] for k in ("fea", "inp", "out")}
    alias = any(p in ptrs["out"] for p in ptrs["fea"] + ptrs["inp"])
    for rep in range(3):
        g2 = [dict(g, out=torch.full_like(g["out"], float("nan"))) for g in groups]
        orig(g2, epi=epi, status=None)
        torch.cuda.synchronize()
        same = [torch.equal(a["out"], b) for a, b in zip(g2, outs)]
        if not all(same):
            d = [float((a["out"] - b).abs().max()) for a, b in zip(g2, outs)]
            bad = [(a["out"] != b) for a, b in zip(g2, outs)]
            where = [tuple(int(x) for x in b.nonzero()[0].tolist()) if b.any() else None for b in bad]
            nd.append(n[0])
            if False: print(f"launch {n[0]} rep {rep}: {len(groups)} groups {tuple(groups[0]['out'].shape)} epi {epi} "
                  f"alias {alias} NONDET max|d| {d} first {where} count {[int(b.sum()) for b in bad]}", flush=True)
    n[0] += 1


ops.dcn_sep = traced
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3", fused_dcn=True)
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
m.eval()
with torch.no_grad():
    m.gen_feat_window(fr)
print(os.environ.get("STIF_HIP_LIB", "in-tree"), "launches", n[0], "nondeterministic (launch per rep)", nd, flush=True)
