"""Debug aid: decoder stage 1 / stage 2 against the oracle's intermediates (GPU box)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402
from oracle import stif_oracle as O  # noqa: E402

stif = stif_pkg.load()
ops = stif.ops
g = dict(np.load("tests/golden/model_16x20.npz"))
sd = stif.weights.make_state_dict(0)
m = stif.LunaTokis(64, 6, 8, 5, 40)
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
x = torch.from_numpy(g["x"]).cuda()
m.gen_feat(x)
feat = m.feat.detach().cpu().numpy()
cap = {}
ref = O.decoding(feat, g["x"], [0.5], sd, capture=cap)
hr_ref, fl_ref = cap["hrfeat"][0], cap["flow"][0]
feats, xin = m._feat, m.inp
_, B, H, Wd, _ = feats.shape
HH, WW = 4 * H, 4 * Wd
tab = ops.DecTablesDev(H, Wd, HH, WW, m.device)
src = m._empty(B, H, Wd, 200)
ops.dec_pack_lr(feats[0], feats[1], feats[2], xin, src)
proj = m._empty(B, H, Wd, 256)
ops.conv2d([dict(layer=m.layers["dec.proj"], in0=src, out=proj)])
mlp = m.layers["dec.mlp"]
hrf = m._empty(B, HH, WW, 64)
flow = m._empty(B, HH, WW, 4)
t = m._time_vec(torch.tensor([[0.5]]), B)
ops.dec_stage1(proj, mlp, tab, t, hrf, flow)
torch.cuda.synchronize()
h = hrf.cpu().numpy().reshape(B, -1, 64)
f = flow.cpu().numpy().reshape(B, -1, 4)
print("hrfeat err", np.abs(h - hr_ref).max(), "max", np.abs(hr_ref).max())
e = np.abs(h - hr_ref).max(-1)[0].reshape(HH, WW)
print("hrfeat bad pixels", int((e > 1e-3).sum()), "of", e.size, "first", np.argwhere(e > 1e-3)[:5].tolist())
ec = np.abs(h - hr_ref)[0].max(0)
print("hrfeat bad channels", np.nonzero(ec > 1e-3)[0].tolist())
print("flow err", np.abs(f - fl_ref).max(), "max", np.abs(fl_ref).max())
ef = np.abs(f - fl_ref)[0].max(0)
print("flow err per comp", ef.tolist())
# stage 2 from the oracle intermediates
hrf.copy_(torch.from_numpy(hr_ref.astype(np.float32).reshape(hrf.shape)))
flow.copy_(torch.from_numpy(fl_ref.astype(np.float32).reshape(flow.shape)))
out = m._empty(B, 3, HH, WW)
ops.dec_stage2(proj, mlp, hrf, flow, tab, t, out)
torch.cuda.synchronize()
o = out.cpu().numpy()
print("out err (oracle intermediates)", np.abs(o - ref[0]).max(), "max", np.abs(ref[0]).max())
