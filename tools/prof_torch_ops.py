"""Which torch ops (fills, copies) run inside one C0 bench step, with their Python call sites."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402
import bench  # noqa: E402

stif = stif_pkg.load()
sd = stif.weights.make_state_dict(seed=0)
dev = torch.device("cuda", 0)
model = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
model.load_state_dict(sd, strict=True)
frames = bench.synth_frames(0, 7, 128, 128, dev)
tq = [torch.tensor([[0.5]], device=dev)]
shards = stif.parallel.pair_shards(7, 1)
with torch.no_grad():
    for _ in range(2):
        stif.parallel.gen_feat_shard(model, frames, 0, 1, shards=shards, exchange=True)
        model.decoding(tq, None)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
        stif.parallel.gen_feat_shard(model, frames, 0, 1, shards=shards, exchange=True)
        model.decoding(tq, None)
        torch.cuda.synchronize()
c = Counter()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::to", "aten::cat", "aten::stack",
                   "aten::contiguous", "aten::item", "aten::_local_scalar_dense", "aten::clone"):
        st = [f for f in (ev.stack or []) if "stif-continuous" in f or "bench" in f or "parallel" in f]
        c[(ev.name, st[0] if st else "?")] += 1
for (n, s), k in sorted(c.items(), key=lambda kv: -kv[1]):
    print(f"{k:4d}  {n:24s} {s}")
