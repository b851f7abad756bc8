"""Run the C0 window through the engine rooted at ROOT (default: this repo; e.g. tools/base_tree for the round-4
tree) and save every decoded output to gpurun_out/r5/out_<TAG>.npy; with CMP=<tag>, compare bit for bit."""
import os
import sys

import numpy as np
import torch

here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
root = os.path.abspath(os.environ.get("ROOT", here))
sys.path.insert(0, root)
import stif_pkg  # noqa: E402
import bench  # noqa: E402

tag, cmp = os.environ.get("TAG", "in-tree"), os.environ.get("CMP")
stif = stif_pkg.load()
dev = torch.device("cuda", 0)
nframes, H, W, scale, times, _ = bench.CONFIGS[os.environ.get("CFG", "c0")]
model = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
model.load_state_dict(stif.weights.make_state_dict(seed=0), strict=True)
frames = bench.synth_frames(0, nframes, H, W, dev)
tq = [torch.tensor([[t]], device=dev) for t in times]
with torch.no_grad():
    for _ in range(2):                      # the second call runs on the constants cached by the first
        model.gen_feat_window(frames)
        outs = model.decoding(tq, None)
    torch.cuda.synchronize()
a = np.stack([o.float().cpu().numpy() for o in outs])
lat = model._feat.float().cpu().numpy()
os.makedirs(os.path.join(here, "gpurun_out/r5"), exist_ok=True)
np.savez(os.path.join(here, f"gpurun_out/r5/out_{tag}.npz"), out=a, feat=lat)
if cmp:
    b = np.load(os.path.join(here, f"gpurun_out/r5/out_{cmp}.npz"))
    print(f"{tag} vs {cmp}: outputs identical={np.array_equal(a, b['out'])} max|d|={float(np.abs(a - b['out']).max()):.3e}; "
          f"latents identical={np.array_equal(lat, b['feat'])}")
