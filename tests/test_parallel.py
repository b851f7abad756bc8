"""Multi-process (gloo, CPU) coverage of the frame-pair sharding and the
optional boundary-frame halo exchange (stif_amd.parallel), with the oracle as compute."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import stif_oracle as O


def test_pair_shards_cover_every_pair_once(stif):
    P = stif.parallel
    for F in (2, 3, 7, 9, 64, 65):
        for world in (1, 2, 3, 8):
            shards = P.pair_shards(F, world)
            pairs = [p for (a, b) in shards for p in range(a, max(a, b - 1))]
            assert pairs == list(range(F - 1)), (F, world, shards)
            for (a, b), (c, d) in zip(shards, shards[1:]):
                if b > a and d > c:
                    assert c == b - 1          # one shared boundary frame
    assert P.pair_shards(64, 8)[0] == (0, 9)    # C3: 63 pairs over 8 ranks = 8,8,...,7


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import stif_pkg
    stif = stif_pkg.load()
    sd = stif.weights.make_state_dict(0)
    a, b = stif.parallel.shard_for_rank(frames.shape[0], world, rank)
    mine = frames[a:b]
    own = O.frame_features(mine[:-1] if rank + 1 < world else mine, sd)
    first = [torch.from_numpy(np.ascontiguousarray(t[:1])) for t in own]
    halo = stif.parallel.halo_exchange(first, rank, world)
    if halo is not None:
        own = [np.concatenate([t, h.numpy()]) for t, h in zip(own, halo)]
    fea1 = [t[:-1] for t in own]
    fea2 = [t[1:] for t in own]
    feat = O.gen_feat_levels(fea1, fea2, sd, back_RBs=40)
    x = np.stack([mine[:-1], mine[1:]], axis=1)
    out = O.decoding(feat, x, [0.5], sd)[0]
    np.save(os.path.join(outdir, f"r{rank}.npy"), out)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_window_equals_single_process(sd):
    rng = np.random.default_rng(5)
    frames = rng.random((5, 3, 8, 8))
    ref = O.forward(np.stack([frames[:-1], frames[1:]], 1), [0.5], sd)[0]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), frames, d), nprocs=2, join=True)
        got = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(2)])
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-9 * np.abs(ref).max()


def _halo_worker(rank, world, port, nframes, outdir):
    """Rank r's shard of an nframes sequence; its 'features' are tagged with the global frame index,
    so the received halo must be the right neighbour's first frame."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import stif_pkg
    P = stif_pkg.load().parallel
    shards = P.pair_shards(nframes, world)
    a, b = shards[rank]
    got = None
    if b > a:
        first = [torch.full((1, 2, 3, 4 * (lv + 1)), float(a * 10 + lv)) for lv in range(3)]
        recv = P.halo_exchange(first, rank, world, shards=shards)
        got = None if recv is None else [float(t.flatten()[0]) for t in recv]
    np.save(os.path.join(outdir, f"h{rank}.npy"), np.array(got if got is not None else [-1.0]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nframes,world", [(3, 4), (7, 3), (9, 4)], ids=["empty_shards", "uneven", "even"])
def test_halo_exchange_neighbours(nframes, world):
    """Rehearsal of the N-rank halo exchange (gloo): every rank with frames receives its last frame's
    L1/L2/L3 features from the next rank with frames; ranks past the last pair (more ranks than pairs)
    take no part and nobody waits on them."""
    import stif_pkg
    P = stif_pkg.load().parallel
    shards = P.pair_shards(nframes, world)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_halo_worker, args=(world, _free_port(), nframes, d), nprocs=world, join=True)
        got = [np.load(os.path.join(d, f"h{r}.npy")).tolist() for r in range(world)]
    for r, (a, b) in enumerate(shards):
        nxt = shards[r + 1] if r + 1 < world else (0, 0)
        if b > a and nxt[1] > nxt[0]:
            assert nxt[0] == b - 1                                   # the shared boundary frame
            assert got[r] == [nxt[0] * 10 + lv for lv in range(3)], (r, got[r])
        else:
            assert got[r] == [-1.0], (r, got[r])


@pytest.mark.parametrize("nframes,world", [(64, 8), (9, 8)], ids=["c3_plan", "c4_plan"])
def test_halo_exchange_world8_plans(nframes, world):
    """The exact shard plans of the 8-GPU configs (BASELINE configs[3] / [4]): C3 = 64 frames -> 63 pairs as
    8,8,8,8,8,8,8,7; C4 = 9 frames -> one pair per rank.  Every rank receives its last frame's features
    from its right neighbour (whose first frame it is), rank 7 receives nothing."""
    import stif_pkg
    P = stif_pkg.load().parallel
    shards = P.pair_shards(nframes, world)
    sizes = [b - a - 1 for a, b in shards]
    assert sizes == ([8] * 7 + [7] if nframes == 64 else [1] * 8), sizes
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_halo_worker, args=(world, _free_port(), nframes, d), nprocs=world, join=True)
        got = [np.load(os.path.join(d, f"h{r}.npy")).tolist() for r in range(world)]
    for r in range(world - 1):
        assert got[r] == [shards[r + 1][0] * 10 + lv for lv in range(3)], (r, got[r])
        assert shards[r + 1][0] == shards[r][1] - 1
    assert got[world - 1] == [-1.0]


class _FakeModel:
    """Stands in for LunaTokis in gen_feat_shard: per-frame 'features' tagged with the global frame index."""

    def __init__(self, a):
        self.a = a
        self.window = None

    def frame_features(self, frames):
        idx = frames[:, 0, 0, 0]
        return tuple(idx.view(-1, 1, 1, 1).repeat(1, 2, 2, 3) * 10 + lv for lv in range(3))

    def gen_feat_window(self, frames, frame_feats=None):
        self.window = (frames[:, 0, 0, 0].tolist(), None if frame_feats is None else
                       [t[:, 0, 0, 0].tolist() for t in frame_feats])


def _shard_worker(rank, world, port, nframes, outdir):
    """gen_feat_shard on every rank, empty shards included (frames=None): the first call's warm_group
    barrier is collective, then the halo exchange runs among the ranks with frames."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import stif_pkg
    P = stif_pkg.load().parallel
    shards = P.pair_shards(nframes, world)
    a, b = shards[rank]
    frames = torch.arange(a, b, dtype=torch.float32).view(-1, 1, 1, 1).repeat(1, 3, 2, 2) if b > a else None
    m = _FakeModel(a)
    for _ in range(2):                                   # the barrier runs once per group
        P.gen_feat_shard(m, frames, rank, world, shards=shards, exchange=True)
    np.save(os.path.join(outdir, f"s{rank}.npy"), np.array(m.window, dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def _reinit_worker(rank, world, ports, nframes, outdir):
    """init -> gen_feat_shard -> destroy -> init again -> gen_feat_shard, every rank incl. an empty shard:
    the re-created default group is a new group and must get its own warm-up barrier."""
    import stif_pkg
    P = stif_pkg.load().parallel
    shards = P.pair_shards(nframes, world)
    a, b = shards[rank]
    frames = torch.arange(a, b, dtype=torch.float32).view(-1, 1, 1, 1).repeat(1, 3, 2, 2) if b > a else None
    calls = []
    real_barrier = dist.barrier

    def counting_barrier(group=None, **kw):
        calls.append(1)
        return real_barrier(group, **kw)

    dist.barrier = counting_barrier
    try:
        for port in ports:                 # a fresh rendezvous port per cycle (rank 0's store is torn down)
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            dist.init_process_group("gloo", rank=rank, world_size=world)
            n0 = len(calls)
            P.gen_feat_shard(_FakeModel(a), frames, rank, world, shards=shards, exchange=True)
            P.gen_feat_shard(_FakeModel(a), frames, rank, world, shards=shards, exchange=True)
            np.save(os.path.join(outdir, f"b{rank}_{len(P._WARM)}.npy"), np.array([len(calls) - n0]))
            real_barrier()
            dist.destroy_process_group()
    finally:
        dist.barrier = real_barrier


def test_warm_group_after_reinit():
    """warm_group's cache must not treat a re-initialised default group as warmed (an empty-shard
    rank would then skip the barrier that creates a lazy NCCL communicator, and the first exchange could
    hang).  Each of the two init/destroy cycles runs exactly one warm-up barrier per rank."""
    world, nframes = 3, 3      # rank 2 has an empty shard
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_reinit_worker, args=(world, (_free_port(), _free_port()), nframes, d), nprocs=world, join=True)
        for r in range(world):
            for k in (1, 2):
                assert np.load(os.path.join(d, f"b{r}_{k}.npy")).tolist() == [1], (r, k)


@pytest.mark.parametrize("nframes,world", [(3, 4), (9, 8)], ids=["empty_shards", "c4_plan"])
def test_gen_feat_shard_all_ranks(nframes, world):
    """gen_feat_shard called by every rank (bench.py's step): ranks with frames get their window's
    features with the boundary frame's from the right neighbour; empty-shard ranks return after the
    one-time barrier and nobody hangs."""
    import stif_pkg
    P = stif_pkg.load().parallel
    shards = P.pair_shards(nframes, world)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_shard_worker, args=(world, _free_port(), nframes, d), nprocs=world, join=True)
        got = [np.load(os.path.join(d, f"s{r}.npy"), allow_pickle=True) for r in range(world)]
    for r, (a, b) in enumerate(shards):
        if b <= a:
            assert got[r].tolist() is None or got[r].size == 0 or got[r].tolist() == [None, None], got[r]
            continue
        frames_seen, feats = got[r].tolist()
        assert frames_seen == list(range(a, b))
        assert feats is not None and feats[0] == [10.0 * f for f in range(a, b)], (r, feats)


class _FakeWork:
    def wait(self):
        return True


class _FakeP2POp:
    """dist.P2POp's fields (the real one needs an initialised default group to be constructed)"""

    def __init__(self, op, tensor, peer, group=None):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


@pytest.mark.parametrize("rank,world,shards", [(0, 2, None), (1, 3, None), (2, 3, None), (7, 8, [(0, 9)] * 8),
                                               (1, 3, [(0, 2), (1, 3), (3, 3)])])
def test_nccl_branch_sends_the_shard_features_unstaged(stif, monkeypatch, rank, world, shards):
    """halo_exchange's nccl branch (the one only the driver's multi-GPU run executes, round-5 review item 7):
    with dist.get_backend monkeypatched to "nccl" and batch_isend_irecv captured, the P2P list holds exactly
    the L1/L2/L3 first-frame features gen_feat_shard passes (shapes [1,H,W,64] / [1,H/2,W/2,64] /
    [1,H/4,W/4,64], float32, contiguous) -- sent as the caller's tensors (no host staging: no copy, same
    device) to rank-1 and received into same-shape, same-device, contiguous buffers from rank+1 -- and the
    received tensors are what gen_feat_shard concatenates.  Empty neighbours are left out."""
    P = stif.parallel
    sent = []
    monkeypatch.setattr(P.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(P.dist, "P2POp", _FakeP2POp)

    def fake_batch(ops):
        sent.extend(ops)
        for op in ops:
            if op.op is P.dist.irecv:
                op.tensor.fill_(float(op.peer))
        return [_FakeWork() for _ in ops]

    monkeypatch.setattr(P.dist, "batch_isend_irecv", fake_batch)
    H, W = 16, 24
    own = [torch.randn(3, H >> k, W >> k, 64) for k in range(3)]   # frame_features of a 3-frame shard
    first = [t[:1] for t in own]                                      # as gen_feat_shard slices them
    recv = P.halo_exchange(first, rank, world, None, shards)
    has = lambda r: 0 <= r < world and (shards is None or shards[r][1] > shards[r][0])   # noqa: E731
    sends = [op for op in sent if op.op is P.dist.isend]
    recvs = [op for op in sent if op.op is P.dist.irecv]
    if has(rank - 1):
        assert [op.peer for op in sends] == [rank - 1] * 3
        for op, t in zip(sends, first):
            assert op.tensor.data_ptr() == t.data_ptr() and op.tensor.device == t.device   # unstaged, no copy
            assert op.tensor.is_contiguous() and op.tensor.dtype == torch.float32
            assert tuple(op.tensor.shape) == tuple(t.shape) == (1, t.shape[1], t.shape[2], 64)
    else:
        assert not sends
    if has(rank + 1):
        assert [op.peer for op in recvs] == [rank + 1] * 3 and recv is not None
        for op, t, r in zip(recvs, first, recv):
            assert op.tensor is r and r.is_contiguous() and r.device == t.device and r.shape == t.shape
            assert r.dtype == torch.float32 and bool((r == rank + 1).all())
        assert [tuple(r.shape[1:3]) for r in recv] == [(H, W), (H // 2, W // 2), (H // 4, W // 4)]
    else:
        assert recv is None and not recvs
