"""Frame-pair sharding of a video over ranks (one process per GPU).

A sequence of F frames is F-1 independent pairs (custom_video_test.py:81; the
ConvLSTM state is re-zeroed for every pair, convlstm.py:60-63), so the temporal
axis shards with no data-path collective: rank r owns a contiguous run of pairs
and the frames they touch.  Neighbouring shards share one boundary frame (the
temporal halo).  By default each rank recomputes that frame's per-frame encoder
(≈1 frame of conv_first + 5 residual blocks + pyramid); ``halo_exchange``
instead ships the encoder features of the boundary frame from rank r+1 to rank
r with point-to-point send/recv (RCCL over xGMI on the GPU, gloo on CPU).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def pair_shards(num_frames: int, world: int) -> List[Tuple[int, int]]:
    """Frame ranges [start, stop) per rank; consecutive ranges overlap by one frame.
    Pairs are split as evenly as possible (the first `rem` ranks take one more)."""
    pairs = num_frames - 1
    if pairs < 1 or world < 1:
        raise ValueError("need >= 2 frames and >= 1 rank")
    base, rem = divmod(pairs, world)
    out = []
    p0 = 0
    for r in range(world):
        n = base + (1 if r < rem else 0)
        out.append((p0, p0 + n + 1) if n else (p0, p0))
        p0 += n
    return out


def shard_for_rank(num_frames: int, world: int, rank: int) -> Tuple[int, int]:
    return pair_shards(num_frames, world)[rank]


def halo_exchange(first_frame_feats: Sequence[torch.Tensor], rank: int, world: int, group=None):
    """Send this rank's first-frame features to rank-1 and receive rank+1's (which is this
    rank's last frame).  Returns the received tensors (None on the last rank)."""
    reqs = []
    recv = None
    if rank + 1 < world:
        recv = [torch.empty_like(t) for t in first_frame_feats]
        reqs += [dist.irecv(t, src=rank + 1, group=group) for t in recv]
    if rank > 0:
        reqs += [dist.isend(t.contiguous(), dst=rank - 1, group=group) for t in first_frame_feats]
    for q in reqs:
        q.wait()
    return recv
