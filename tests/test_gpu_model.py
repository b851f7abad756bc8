"""End-to-end parity of the MI355X LunaTokis against the reference's own outputs
(golden fixtures) and the CPU oracle, plus the size-independent checks used at
full benchmark sizes."""
import numpy as np
import pytest
import torch

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu

# north_star: outputs within rtol 1e-4 (fp32) and PSNR within 1e-3 dB of the reference.
# Elementwise: |gpu - ref| <= 1e-4 * |ref| + 1e-6 for every element.
RTOL = 1e-4
ATOL = 1e-6


def close(a, b, rtol=RTOL, atol=ATOL):
    """(ok, max |a - b|, worst ratio of |a - b| to its elementwise bound)"""
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = np.asarray(b, np.float64)
    d = np.abs(a - b)
    lim = rtol * np.abs(b) + atol
    return bool((d <= lim).all()), float(d.max()), float((d / lim).max())


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


def test_intermediates_match_reference(model, golden):
    """PCD_Align output, fusion and BiConvLSTM latents (model_16x20.npz holds the reference's
    forward-hook captures, make_golden.py:142-166) against the engine's own buffers."""
    g = golden["model_16x20"]
    x = torch.from_numpy(g["x"]).cuda()
    cap = {}
    orig_bilstm, orig_pcd = model._bilstm_steps, model._pcd_align

    def bilstm(X, *a, **k):                             # a stage generator (LunaTokis._run_lanes)
        cap["fusion"] = X[1].detach().clone()           # fusion output = latent step 1 input
        out = yield from orig_bilstm(X, *a, **k)
        cap["bilstm"] = out.detach().clone()
        return out

    def pcd(units, **kw):
        orig_pcd(units, **kw)
        if units[0][0] == "pcd_align." and "pcd" not in cap:
            cap["pcd"] = [u[4].detach().clone() for u in units]
    model._bilstm_steps, model._pcd_align = bilstm, pcd
    try:
        with torch.no_grad():
            model.gen_feat(x)
    finally:
        del model._bilstm_steps, model._pcd_align
    nchw = lambda t: t.permute(0, 3, 1, 2)[0].cpu().numpy()
    pcd_out = np.concatenate([nchw(cap["pcd"][0]), nchw(cap["pcd"][1])], 0)     # cat(y1, y2) (:130)
    for name, got, ref in (("pcd_align", pcd_out, g["pcd_align"]), ("fusion", nchw(cap["fusion"]), g["fusion"]),
                           ("bilstm", np.stack([nchw(cap["bilstm"][t]) for t in range(3)]), g["bilstm"])):
        assert got.shape == ref.shape, (name, got.shape, ref.shape)
        ok, err, worst = close(got, ref)
        assert ok, (name, err, worst)


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
    """|PSNR(gpu, GT) - PSNR(ref, GT)| < 1e-3 dB, GT = the reference output quantised to 8-bit levels
    (the precision the harness writes frames in) -- a GT close to both, so the delta is sensitive."""
    g, outs, _, _ = run16
    ref = g["out"][2]
    gt = np.round(np.clip(ref.astype(np.float64), 0, 1) * 255) / 255
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


@pytest.fixture(scope="module")
def latent16(model, golden):
    x = torch.from_numpy(golden["model_16x20"]["x"]).cuda()
    with torch.no_grad():
        model.gen_feat(x)
    return model


def test_forward_test_true_is_decoding_test(model, golden):
    """forward(test=True) -> decoding_test (Sakuya_arch_test.py:1225-1226, 461-598): flow / encode
    stages sample the x4 bilinear-upsampled frames."""
    d = golden["decoders_16x20"]
    x = torch.from_numpy(golden["model_16x20"]["x"]).cuda()
    with torch.no_grad():
        outs = model(x, [torch.tensor([[float(t)]]) for t in d["test_times"]], test=True)
    for i, o in enumerate(outs):
        assert tuple(o.shape) == (1, 3, 64, 80)
        ok, err, mx = close(o[0], d["test_out"][i])
        assert ok, (i, err, mx)


def test_decoding_test_scale3(latent16, golden):
    d = golden["decoders_16x20"]
    with torch.no_grad():
        o = latent16.decoding_test([torch.tensor([[0.5]])], 3)[0]
    assert tuple(o.shape) == (1, 3, 48, 60)
    ok, err, mx = close(o[0], d["test_out_scale3"])
    assert ok, (err, mx)


@pytest.mark.parametrize("which", ["fast", "fast_40x50"])
def test_decoding_fasttest(latent16, golden, which):
    d = golden["decoders_16x20"]
    with torch.no_grad():
        if which == "fast":
            o, ref = latent16.decoding_fasttest([float(t) for t in d["fast_times"]]), d["fast_out"]
        else:
            o, ref = latent16.decoding_fasttest([0.5], (40, 50)), d["fast_out_40x50"]
    assert tuple(o.shape) == ref.shape
    ok, err, mx = close(o, ref)
    assert ok, (err, mx)


@pytest.mark.parametrize("which", ["ens", "ens_40x50"])
def test_decoding_localensemble(latent16, golden, which):
    """four shifted decodes (HRfeat read at the shifted query's nearest HR pixel) + area blend"""
    d = golden["decoders_16x20"]
    with torch.no_grad():
        if which == "ens":
            o, ref = latent16.decoding_localensemble([0.5]), d["ens_out"]
        else:
            o, ref = latent16.decoding_localensemble([0.25], (40, 50)), d["ens_out_40x50"]
    assert tuple(o.shape) == ref.shape
    ok, err, mx = close(o, ref)
    assert ok, (err, mx)


@pytest.fixture(scope="module")
def model_f32(stif, sd):
    m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f32")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return m.eval()


def test_f32_mfma_outputs_match_reference(model_f32, golden):
    """mfma='f32' (every contraction on fp32 MFMA; the default 'f16x3' runs the Winograd convs and
    the DCN core on split-fp16 MFMA operands) against the reference's outputs, same bar."""
    g = golden["model_16x20"]
    with torch.no_grad():
        outs = model_f32(torch.from_numpy(g["x"]).cuda(), [torch.tensor([[float(t)]]) for t in g["times"]])
    ok, err, mx = close(model_f32.feat.detach().cpu().numpy()[0], g["feat"])
    assert ok, (err, mx)
    for i, o in enumerate(outs):
        ok, err, mx = close(o[0], g["out"][i])
        assert ok, (i, err, mx)


def test_f32_mfma_window_and_psnr(model_f32, golden, sd):
    """7-frame window against the reference, and the PSNR criterion (< 1e-3 dB)."""
    g = golden["window_7x16x16"]
    with torch.no_grad():
        model_f32.gen_feat_window(torch.from_numpy(g["frames"]).cuda())
        out = model_f32.decoding([torch.tensor([[0.5]])])[0]
    ok, err, mx = close(out, g["out"])
    assert ok, (err, mx)
    gt = np.round(np.clip(g["out"].astype(np.float64), 0, 1) * 255) / 255
    d = abs(psnr(out.cpu().numpy(), gt) - psnr(g["out"], gt))
    assert d < 1e-3, d


def test_f32_mfma_larger_size_vs_oracle(model_f32, sd):
    rng = np.random.default_rng(7)
    x = rng.random((1, 2, 3, 32, 48)).astype(np.float32)
    ref = O.forward(x, [0.3], sd)[0]
    with torch.no_grad():
        out = model_f32(torch.from_numpy(x).cuda(), [0.3])[0]
    ok, err, mx = close(out, ref)
    assert ok, (err, mx)


def test_decoder_stage2_flags_nonfinite_flow(stif, sd, golden):
    """f16x3 range guard through the decoder's stage boundary: a flow_imnet operand outside the split
    range makes that pixel's flow NaN; stage 2's warpgrid clamp would turn it into a finite grid, so
    stage 2 reports the flow it reads (status word -> the fp32 re-run) instead of a finite wrong pixel."""
    m = stif.LunaTokis(64, 6, 8, 5, 40)
    m.load_state_dict(sd, strict=True)
    g = golden["model_16x20"]
    ops = stif.ops
    with torch.no_grad():
        m.gen_feat(torch.from_numpy(g["x"]).cuda())
        proj = m._projection()
        _, H, W, _ = proj.shape
        HH, WW = 4 * H, 4 * W
        tab = m._tab(H, W, HH, WW)
        t = torch.full((1,), 0.5, device="cuda")
        hrf = torch.empty(1, HH, WW, 64, device="cuda")
        flow = torch.empty(1, HH, WW, 4, device="cuda")
        mlp = m.layers["dec.mlp"]
        assert m._dec_flags & stif._lib.CONV_F16X3
        ops.dec_stage1(proj, mlp, tab, t, hrf, flow, flags=m._dec_flags)
        out = torch.empty(1, 3, HH, WW, device="cuda")
        for poison in (False, True):
            st = torch.zeros(1, dtype=torch.int32, device="cuda")
            f = flow.clone()
            if poison:
                f[0, 7, 11, 2] = float("nan")
            ops.dec_stage2(proj, mlp, hrf, f, tab, t, out, flags=m._dec_flags, status=st)
            assert int(st.item()) == int(poison)
            assert bool(torch.isfinite(out).all())      # the clamp keeps the pixel finite: only the flag tells


def test_cached_constants_follow_the_weights(stif):
    """The encoder caches weight-only constants across calls (the zero-state pyramids and L1 DCN maps,
    LunaTokis._const).  Loading other weights into the same module must not reuse them: the second run equals
    a fresh module's bit for bit, and a repeated call equals the first."""
    dev = torch.device("cuda", 0)
    fr = torch.rand(3, 3, 32, 48, generator=torch.Generator().manual_seed(3)).to(dev)
    tq = [torch.tensor([[0.5]])]

    def run(m):
        with torch.no_grad():
            m.gen_feat_window(fr)
            out = m.decoding(tq)[0]
        torch.cuda.synchronize()
        return m._feat.clone(), out.clone()

    m = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
    m.load_state_dict(stif.weights.make_state_dict(0), strict=True)
    a0 = run(m)
    assert torch.equal(run(m)[1], a0[1])               # second call on the cached constants
    m.load_state_dict(stif.weights.make_state_dict(1), strict=True)
    b = run(m)
    fresh = stif.LunaTokis(64, 6, 8, 5, 40, device=dev)
    fresh.load_state_dict(stif.weights.make_state_dict(1), strict=True)
    ref = run(fresh)
    assert torch.equal(b[0], ref[0]) and torch.equal(b[1], ref[1])
    assert not torch.equal(b[1], a0[1])
