"""Per-wave s_memtime trace of k_dec2 (tools/exp_dectrace.so, built by tools/r4/make_dec_trace.py): the C0 (CFG)
window's latents once, then model.decoding; prints the average cycles of every segment between trace tags
(tags: see make_dec_trace.py) over the traced waves, the layer-2/3 steps pooled."""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("STIF_HIP_LIB", os.path.join(R, "tools", "exp_dectrace.so"))
import stif_pkg  # noqa: E402
import bench  # noqa: E402

cfg = os.environ.get("CFG", "c0")
stif = stif_pkg.load()
dev = torch.device("cuda", 0)
nframes, H, W, scale, times, _ = bench.CONFIGS[cfg]
model = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
model.load_state_dict(stif.weights.make_state_dict(seed=0), strict=True)
frames = bench.synth_frames(0, nframes, H, W, dev)
tq = [torch.tensor([[t]], device=dev) for t in times[:1]]
with torch.no_grad():
    model.gen_feat_window(frames)
    for _ in range(3):
        model.decoding(tq, None)
    torch.cuda.synchronize()
buf = np.zeros(4096 * 4 * 64, dtype=np.uint64)
lib = stif._lib.lib()
lib.stif_exp_dec_trace.argtypes = [C.c_void_p]
assert lib.stif_exp_dec_trace(buf.ctypes.data) == 0
tr = buf.reshape(4096, 4, 64)
names = {0: "start", 1: "P3", 2: "P4+lr", 3: "HRF1", 4: "bar0", 5: "mma0a", 6: "HRF2", 7: "l0", 8: "bar1", 9: "l1",
         10: "st", 11: "st.bar", 12: "st.l2", 13: "st.l3", 14: "bar4", 15: "l4", 16: "end"}
seg = defaultdict(list)
life = []
for blk in range(4096):
    for wv in range(4):
        ev = [(int(v) >> 8, int(v) & 0xFF) for v in tr[blk, wv] if v]
        if len(ev) < 2:
            continue
        life.append(ev[-1][0] - ev[0][0])
        for (t0, a), (t1, b) in zip(ev, ev[1:]):
            seg[(a, b)].append(t1 - t0)
tot = np.mean(life)
print(f"{cfg}: {len(life)} traced waves, lifetime avg {tot:.0f} med {np.median(life):.0f} cycles")
for k in sorted(seg, key=lambda k: (k[0], k[1])):
    v = np.array(seg[k])
    per_wave = v.sum() / len(life)
    print(f"  {names[k[0]]:>7s} -> {names[k[1]]:<7s} n={len(v):6d} avg {v.mean():8.0f} med {np.median(v):8.0f} "
          f"per wave {per_wave:8.0f} ({per_wave / tot * 100:4.1f} %)")
