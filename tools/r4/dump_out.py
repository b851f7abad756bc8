"""Round-4 A/B aid: run the bench's C0 window (or CFG) once through the library STIF_HIP_LIB names (default:
in-tree) and save every decoded output to gpurun_out/r4/out_<TAG>.npy; with CMP=<tag>, compare against that
saved run bit for bit and print the max abs difference."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402
import bench  # noqa: E402

cfg, tag, cmp = os.environ.get("CFG", "c0"), os.environ.get("TAG", "in-tree"), os.environ.get("CMP")
stif = stif_pkg.load()
dev = torch.device("cuda", 0)
nframes, H, W, scale, times, _ = bench.CONFIGS[cfg]
model = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
model.load_state_dict(stif.weights.make_state_dict(seed=0), strict=True)
frames = bench.synth_frames(0, nframes, H, W, dev)
tq = [torch.tensor([[t]], device=dev) for t in times]
with torch.no_grad():
    model.gen_feat_window(frames)
    outs = model.decoding(tq, None)
    torch.cuda.synchronize()
a = np.stack([o.float().cpu().numpy() for o in outs])
os.makedirs("gpurun_out/r4", exist_ok=True)
np.save(f"gpurun_out/r4/out_{tag.replace('/', '_')}.npy", a)
if cmp:
    b = np.load(f"gpurun_out/r4/out_{cmp}.npy")
    print(f"{tag} vs {cmp}: identical={np.array_equal(a, b)} max|d|={float(np.abs(a - b).max()):.3e} "
          f"max|ref|={float(np.abs(b).max()):.3e}")
