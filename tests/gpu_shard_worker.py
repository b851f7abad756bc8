"""One rank of the multi-rank GPU test (tests/test_gpu_parallel.py), started by torch.distributed.run:
gloo process group, every rank on cuda:0 (one GPU box), the HIP engine as compute.  Rank r encodes
its pair shard of an F-frame sequence with parallel.gen_feat_shard (boundary-frame features from
rank r+1 by halo_exchange, staged through host memory for gloo), decodes it and saves the latents and
outputs to <outdir>/r<rank>.pt."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    nframes, H, W, outdir = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    import stif_pkg
    stif = stif_pkg.load()
    P = stif.parallel
    torch.cuda.set_device(0)
    m = stif.LunaTokis(64, 6, 8, 5, 40, device="cuda:0")
    m.load_state_dict(stif.weights.make_state_dict(0), strict=True)
    shards = P.pair_shards(nframes, world)
    a, b = shards[rank]
    res = {"shard": (a, b)}
    fr = None
    if b > a:
        fr = torch.empty(b - a, 3, H, W)
        for i in range(b - a):
            fr[i] = torch.rand(3, H, W, generator=torch.Generator().manual_seed(1234 + a + i))
        fr = fr.cuda()
    with torch.no_grad():
        # every rank calls it, an empty shard too (frames=None: it only joins the first call's barrier)
        P.gen_feat_shard(m, fr, rank, world, shards=shards, exchange=True)
        if fr is not None:
            res["feat"] = m.feat.cpu().clone()
            res["out"] = m.decoding([torch.tensor([[0.5]])])[0].cpu()
    torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
