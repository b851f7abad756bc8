"""The multi-rank path with the HIP engine as compute, on the one GPU of a test box: several
processes (gloo, all on cuda:0) run parallel.gen_feat_shard -- pair shards, the boundary frame's
encoder features handed over by halo_exchange -- and bench.py's distributed timing.  The sharded
latents and outputs must equal a single-process window bit for bit (every kernel computes each pair
independently of the batch it is launched in), also when a rank's shard is empty."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(world, args, timeout=240):
    """torch.distributed.run with `world` local ranks (a child process; the launcher itself never
    touches the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + args
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("nframes,world", [(9, 2), (3, 3)], ids=["2ranks", "3ranks_one_empty"])
def test_sharded_hip_window_equals_single_process(stif, sd, nframes, world):
    H, W = 32, 48
    with tempfile.TemporaryDirectory() as d:
        _launch(world, ["tests/gpu_shard_worker.py", str(nframes), str(H), str(W), d])
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    shards = stif.parallel.pair_shards(nframes, world)
    assert [tuple(r["shard"]) for r in res] == [tuple(s) for s in shards]
    live = [r for r in res if "feat" in r]
    assert len(live) == min(world, nframes - 1)
    m = stif.LunaTokis(64, 6, 8, 5, 40)
    m.load_state_dict(sd, strict=True)
    fr = torch.empty(nframes, 3, H, W)
    for i in range(nframes):
        fr[i] = torch.rand(3, H, W, generator=torch.Generator().manual_seed(1234 + i))
    with torch.no_grad():
        m.gen_feat_window(fr.cuda())
        ref_feat = m.feat.cpu()
        ref_out = m.decoding([torch.tensor([[0.5]])])[0].cpu()
    assert torch.equal(torch.cat([r["feat"] for r in live]), ref_feat)
    assert torch.equal(torch.cat([r["out"] for r in live]), ref_out)


def test_bench_two_ranks_gloo():
    """bench.py's N>1 path (barrier + synchronize around the timed steps, max over ranks, the halo
    exchange inside the step, one JSON line from rank 0) with 2 ranks sharing the GPU over gloo."""
    out = _launch(2, ["bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--backend", "gloo",
                      "--no-cpu-baseline"], timeout=400)
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["scaling"] == "weak"
    assert "halo" in line["config"]["parallelism"].lower()
