"""End-to-end parity of the MI355X LunaTokis against the reference's own outputs
(golden fixtures) and the CPU oracle, plus the size-independent checks used at
full benchmark sizes."""
import numpy as np
import pytest
import torch

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu

# north_star: outputs within rtol 1e-4 (fp32) and PSNR within 1e-3 dB of the reference.
# Elementwise: |gpu - ref| <= 1e-4 * max|ref| + 1e-6.
RTOL = 1e-4
ATOL = 1e-6


def close(a, b, rtol=RTOL, atol=ATOL):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b).max()
    return err <= rtol * np.abs(b).max() + atol, float(err), float(np.abs(b).max())


def psnr(a, gt):
    mse = float(np.mean((np.asarray(a, np.float64) - gt) ** 2))
    return 10 * np.log10(1.0 / mse)


@pytest.fixture(scope="module")
def model(stif, sd):
    m = stif.LunaTokis(64, 6, 8, 5, 40)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return m.eval()


@pytest.fixture(scope="module")
def run16(model, golden):
    g = golden["model_16x20"]
    x = torch.from_numpy(g["x"]).cuda()
    times = [torch.tensor([[float(t)]]) for t in g["times"]]
    with torch.no_grad():
        outs = model(x, times)
        feat = model.feat.detach().cpu().numpy()
        out25 = model.decoding([torch.tensor([[0.5]])], scale=(40, 50))[0]
    torch.cuda.synchronize()
    return g, outs, feat, out25


def test_gen_feat_matches_reference(run16):
    g, _, feat, _ = run16
    ok, err, mx = close(feat[0], g["feat"])
    assert ok, (err, mx)


def test_outputs_match_reference(run16):
    g, outs, _, _ = run16
    for i, o in enumerate(outs):
        assert tuple(o.shape) == (1, 3, 64, 80)
        ok, err, mx = close(o[0], g["out"][i])
        assert ok, (i, err, mx)


def test_arbitrary_scale_matches_reference(run16):
    g, _, _, out25 = run16
    assert tuple(out25.shape) == (1, 3, 40, 50)
    ok, err, mx = close(out25[0], g["out_scale_40x50"])
    assert ok, (err, mx)


def test_psnr_criterion(run16, sd):
    """|PSNR(gpu, GT) - PSNR(ref, GT)| < 1e-3 dB with GT = the fp64 oracle perturbed by noise."""
    g, outs, _, _ = run16
    ref = g["out"][2]
    gt = O.forward(g["x"], [0.5], sd)[0][0] + np.random.default_rng(0).standard_normal(ref.shape) * 0.01
    d = abs(psnr(outs[2][0].cpu().numpy(), gt) - psnr(ref, gt))
    assert d < 1e-3, d


def test_window_matches_reference(model, golden):
    """custom_video_test's pair loop (custom_video_test.py:81-97) as one batched window."""
    g = golden["window_7x16x16"]
    frames = torch.from_numpy(g["frames"]).cuda()
    with torch.no_grad():
        model.gen_feat_window(frames)
        out = model.decoding([torch.tensor([[0.5]])])[0]
    ok, err, mx = close(out, g["out"])
    assert ok, (err, mx)


def test_pairs_are_independent(model, golden):
    """Batching pairs (B>1) gives the same per-pair output as B=1 (bit-exact)."""
    g = golden["window_7x16x16"]
    fr = torch.from_numpy(g["frames"]).cuda()
    x = torch.stack([fr[:-1], fr[1:]], 1)
    with torch.no_grad():
        allp = model(x, [0.5])[0]
        one = model(x[3:4], [0.5])[0]
    assert torch.equal(allp[3:4], one)


def test_deterministic(model, golden):
    g = golden["model_16x20"]
    x = torch.from_numpy(g["x"]).cuda()
    with torch.no_grad():
        a = model(x, [0.5])[0].clone()
        b = model(x, [0.5])[0]
    assert torch.equal(a, b)


def test_larger_size_vs_oracle(model, sd):
    """A non-square 32x48 pair at 4x against the fp64 oracle (tile edges, multi-tile grids)."""
    rng = np.random.default_rng(7)
    x = rng.random((1, 2, 3, 32, 48)).astype(np.float32)
    ref = O.forward(x, [0.3], sd)[0]
    with torch.no_grad():
        out = model(torch.from_numpy(x).cuda(), [0.3])[0]
    ok, err, mx = close(out, ref)
    assert ok, (err, mx)


def test_direct_conv_path_matches_reference(stif, sd, golden):
    """winograd=False (every 3x3 conv on the direct implicit-GEMM kernel) against the fixtures."""
    g = golden["model_16x20"]
    m = stif.LunaTokis(64, 6, 8, 5, 40, winograd=False)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    with torch.no_grad():
        outs = m(torch.from_numpy(g["x"]).cuda(), [torch.tensor([[float(t)]]) for t in g["times"]])
    ok, err, mx = close(m.feat.detach().cpu().numpy()[0], g["feat"])
    assert ok, (err, mx)
    for i, o in enumerate(outs):
        ok, err, mx = close(o[0], g["out"][i])
        assert ok, (i, err, mx)
