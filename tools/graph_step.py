"""Eager vs hipGraph-replayed C0 step (torch.cuda.CUDAGraph over the ctypes launches): wall time per
step and bit-exactness of the output."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402
import bench  # noqa: E402

cfg = os.environ.get("CFG", "c0")
steps = int(os.environ.get("STEPS", "20"))
stif = stif_pkg.load()
sd = stif.weights.make_state_dict(seed=0)
dev = torch.device("cuda", 0)
nframes, H, W, scale, times, _ = bench.CONFIGS[cfg]
model = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
model.load_state_dict(sd, strict=True)
frames = bench.synth_frames(0, nframes, H, W, dev)
tq = [torch.tensor([[t]], device=dev) for t in times]


def step():
    model.gen_feat_window(frames)
    return model.decoding(tq, None)


def timeit(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


with torch.no_grad():
    for _ in range(2):
        ref = step()
    torch.cuda.synchronize()
    ref = [r.clone() for r in ref]
    e1 = timeit(step, steps)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gout = step()
    g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(gout, ref))
    print("graph output bit-identical:", same, "status", int(model._range_status.item()), flush=True)
    g1 = timeit(g.replay, steps)
    e2 = timeit(step, steps)
    g2 = timeit(g.replay, steps)
    print(f"{cfg}: eager {e1:.3f} / {e2:.3f} ms, graph {g1:.3f} / {g2:.3f} ms per step", flush=True)
