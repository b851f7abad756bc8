"""Decoder-only microbenchmark: C0 latents computed once, then REPS x model.decoding (k_pack_lr, the
LR projection, k_dec1, k_dec2) with HIP-event times per decoder kernel kind."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402
import bench  # noqa: E402

cfg = os.environ.get("CFG", "c0")
reps = int(os.environ.get("REPS", "5"))
stif = stif_pkg.load()
sd = stif.weights.make_state_dict(seed=0)
dev = torch.device("cuda", 0)
nframes, H, W, scale, times, _ = bench.CONFIGS[cfg]
model = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
model.load_state_dict(sd, strict=True)
frames = bench.synth_frames(0, nframes, H, W, dev)
tq = [torch.tensor([[t]], device=dev) for t in times]
with torch.no_grad():
    model.gen_feat_window(frames)
    model.decoding(tq, None)
    torch.cuda.synchronize()
    probe = bench.KernelTimer(None)
    stif.ops.TRACE = probe
    for _ in range(reps):
        model.decoding(tq, None)
    torch.cuda.synchronize()
    stif.ops.TRACE = None
for k, (nl, ms, fl, nb) in sorted(probe.per_kind().items(), key=lambda kv: -kv[1][1]):
    print(f"{str(k):50s} {nl:4d} x {ms / nl * 1e3:9.1f} us  {fl / (ms * 1e-3) / 1e12:7.1f} TFLOP/s", flush=True)
