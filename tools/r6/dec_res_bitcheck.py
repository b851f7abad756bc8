"""Decode the C0 window's first pair with the library STIF_HIP_LIB names and save HRfeat-dependent outputs, or compare
with a saved run: the resident-weight stage 1 (DEC1_RES) must be bit-identical to the streamed k_dec1."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
sd = {k: torch.from_numpy(v) for k, v in stif.weights.make_state_dict(0).items()}
fr = torch.empty(7, 3, 128, 128)
for i in range(7):
    fr[i] = torch.rand(3, 128, 128, generator=torch.Generator().manual_seed(1234 + i))
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3")
m.load_state_dict(sd, strict=True)
m.eval()
with torch.no_grad():
    m.gen_feat_window(fr.cuda())
    outs = [o.cpu().numpy() for o in m.decoding([torch.tensor([[0.5]]), torch.tensor([[0.25]])])]
path = sys.argv[2]
if sys.argv[1] == "save":
    np.savez(path, *outs)
    print("saved", [o.shape for o in outs])
else:
    ref = np.load(path)
    for i, o in enumerate(outs):
        r = ref[f"arr_{i}"]
        print(f"time {i}: bit-identical {np.array_equal(o, r)}  max|d| {np.abs(o - r).max():.3e}")
