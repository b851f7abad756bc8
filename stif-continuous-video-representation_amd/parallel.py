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
    Pairs are split as evenly as possible (the first `rem` ranks take one more); with more ranks
    than pairs the surplus ranks get an empty range (start == stop)."""
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


# process-group objects already warmed.  Held by reference and compared by identity: a group destroyed and
# re-created (destroy_process_group + init_process_group) is a new object and is warmed again, and an id()
# cannot be reused by a later group while its object is held here.
_WARM: list = []


def _group_object(group):
    return group if group is not None else dist.distributed_c10d._get_default_group()


def warm_group(group=None):
    """One ``dist.barrier(group)`` per process group, the first time a shard step runs: every rank --
    also one whose shard is empty and that never enters the exchange -- takes part, so a lazily
    initialised NCCL communicator exists before the first ``batch_isend_irecv`` whatever the caller's
    ``init_process_group`` did (no ``device_id`` needed)."""
    if not dist.is_initialized():
        return
    g = _group_object(group)
    if any(w is g for w in _WARM):
        return
    dist.barrier(group)
    _WARM.append(g)


def halo_exchange(first_frame_feats: Sequence[torch.Tensor], rank: int, world: int, group=None,
                  shards: Sequence[Tuple[int, int]] = None):
    """Send this rank's first-frame features to rank-1 and receive rank+1's (which is this rank's
    last frame): one neighbour exchange per rank, issued as one batched P2P group (RCCL over xGMI
    with the nccl backend, gloo on CPU).  Returns the received tensors (on the device of the sent
    ones), or None when this rank has no right neighbour with frames.  ``shards`` (pair_shards) lets
    ranks whose shard is empty -- more ranks than pairs -- drop out of the exchange instead of
    waiting on a peer that sends nothing.

    With the gloo backend device tensors are staged through host memory (gloo's send/recv move CPU
    tensors), so several ranks can share one GPU (the multi-rank GPU test).  With nccl the group's
    communicator must exist before the first exchange: ranks with an empty shard (or no neighbour)
    never enter ``batch_isend_irecv``, and a lazily created NCCL communicator needs every rank of the
    group in its first collective -- ``gen_feat_shard`` calls ``warm_group`` (one barrier) first."""
    def has(r):
        return 0 <= r < world and (shards is None or shards[r][1] > shards[r][0])

    if not has(rank):
        return None
    stage = dist.get_backend(group) == "gloo"
    ops = []
    recv = None
    if has(rank + 1):
        recv = [torch.empty_like(t, device="cpu" if stage else t.device) for t in first_frame_feats]
        ops += [dist.P2POp(dist.irecv, t, rank + 1, group) for t in recv]
    if has(rank - 1):
        ops += [dist.P2POp(dist.isend, (t.cpu() if stage else t).contiguous(), rank - 1, group)
                for t in first_frame_feats]
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    if recv is not None and stage:
        recv = [r.to(t.device) for r, t in zip(recv, first_frame_feats)]
    return recv


def gen_feat_shard(model, frames, rank: int, world: int, group=None, shards=None,
                   exchange: bool = True):
    """Encoder of this rank's shard of one sequence.  ``frames``: the shard's frames [a, b) (its
    pairs' frames, boundary frame included), or None for an empty shard (more ranks than pairs: the
    rank only joins the first call's ``warm_group`` barrier).  With ``exchange``, the boundary frame's
    per-frame features (L1/L2/L3 of conv_first + feature_extraction + pyramid, 336 B per LR pixel)
    come from rank r+1 by ``halo_exchange`` instead of being recomputed; ``exchange=False`` recomputes
    them.  Every rank of the group calls it (collectively, the first time).  Leaves the latents of the
    shard's pairs in ``model.feat``."""
    if exchange and world > 1:
        warm_group(group)
    if frames is None:
        return
    if not exchange or world == 1:
        model.gen_feat_window(frames)
        return
    has_right = rank + 1 < world and (shards is None or shards[rank + 1][1] > shards[rank + 1][0])
    own = model.frame_features(frames[:-1] if has_right else frames)
    recv = halo_exchange([t[:1] for t in own], rank, world, group, shards)
    feats = own if recv is None else tuple(torch.cat([a, b]) for a, b in zip(own, recv))
    model.gen_feat_window(frames, frame_feats=feats)
