"""Host issue time vs GPU time of one C0 step: is the step bound by Python-side launch issue?
range_check 'off' (no status read between gen_feat and decoding) vs 'rerun' (the default: one
status read after each public call)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
dev = torch.device("cuda", 0)
sd = stif.weights.make_state_dict(seed=0)
frames = bench.synth_frames(0, 7, 128, 128, dev)
tq = [torch.tensor([[0.5]], device=dev)]
for rc in ("off", "rerun", "off", "rerun"):
    m = stif.LunaTokis(64, 6, 8, 5, 40, device=dev, range_check=rc)
    m.load_state_dict(sd, strict=True)
    with torch.no_grad():
        for _ in range(3):
            m.gen_feat_window(frames)
            m.decoding(tq)
        torch.cuda.synchronize()
        iss, tot = [], []
        for _ in range(10):
            t0 = time.perf_counter()
            m.gen_feat_window(frames)
            t1 = time.perf_counter()
            m.decoding(tq)
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            iss.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
            tot.append((t3 - t0) * 1e3)
        g = sorted(i[0] for i in iss)[5]
        d = sorted(i[1] for i in iss)[5]
        print(f"range_check={rc:5s}: host gen_feat call {g:7.3f} ms, decoding call {d:6.3f} ms, step {sorted(tot)[5]:7.3f} ms "
              f"(medians of 10)", flush=True)
