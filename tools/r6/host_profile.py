"""Host-side cost of one C0 bench step (gen_feat_window + decoding): wall time of the step without a final sync
(host issue time) vs with it, and a cProfile of 5 steps (top functions by own time)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
sd = {k: torch.from_numpy(v) for k, v in stif.weights.make_state_dict(0).items()}
fr = torch.empty(7, 3, 128, 128)
for i in range(7):
    fr[i] = torch.rand(3, 128, 128, generator=torch.Generator().manual_seed(1234 + i))
fr = fr.cuda()
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3")
m.load_state_dict(sd, strict=True)
m.eval()
tq = [torch.tensor([[0.5]], device="cuda")]


def step():
    m.gen_feat_window(fr)
    return m.decoding(tq)


with torch.no_grad():
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for rc in ("rerun", "off"):
        m.range_check = rc
        t0 = time.perf_counter()
        for _ in range(10):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"range_check={rc}: host issue {(t1 - t0) / 10 * 1e3:.2f} ms/step, wall {(t2 - t0) / 10 * 1e3:.2f} ms/step")
    m.range_check = "rerun"
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
