"""Every BASELINE.json config on the GPU, the model API as an nn.Module, the halo path, the f16x3
range guard and the harness's single_forward.

Tolerance (SURVEY.md section 8d / BASELINE.json north_star "rtol 1e-4 fp32"): elementwise
|a - b| <= 1e-4 |b| + 1e-6 against the reference's output (C0: one full 128x128 pair, fixture made
by running the reference model, tests/golden/make_golden.py c0) and, at the sizes the CPU cannot
reach in a test (C1-C4 per rank), between the two operand modes of this engine (f16x3 vs fp32 MFMA,
which agree with the reference to ~1e-6 of max|ref| at every size the oracle covers), plus
finiteness and bit-exact batch independence.
"""
import os
import warnings

import numpy as np
import pytest
import torch

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
RTOL, ATOL = 1e-4, 1e-6


def elementwise_ok(a, b, rtol=RTOL, atol=ATOL):
    """(all within |a - b| <= rtol |b| + atol, worst excess ratio, max |a - b|) on the device."""
    a = torch.as_tensor(a).to("cuda", torch.float64)
    b = torch.as_tensor(b).to("cuda", torch.float64)
    d = (a - b).abs()
    lim = rtol * b.abs() + atol
    return bool((d <= lim).all()), float((d / lim).max()), float(d.max())


def synth(first, count, H, W):
    """bench.synth_frames: frame k = torch.rand(3, H, W) from Generator(1234 + k)."""
    out = torch.empty(count, 3, H, W)
    for i in range(count):
        out[i] = torch.rand(3, H, W, generator=torch.Generator().manual_seed(1234 + first + i))
    return out.cuda()


@pytest.fixture(scope="module")
def models(stif, sd):
    ms = {}
    for mf in ("f16x3", "f32"):
        m = stif.LunaTokis(64, 6, 8, 5, 40, mfma=mf)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        ms[mf] = m.eval()
    return ms


@pytest.mark.parametrize("mf", ["f16x3", "f32"])
def test_c0_full_pair_matches_reference(models, mf):
    """C0 (BASELINE configs[0]): the metric's 128x128 pair, 4x, t = 0.5, against the reference
    model's own output, elementwise, and the PSNR criterion (< 1e-3 dB)."""
    g = np.load(os.path.join(GOLD, "c0_pair_128.npz"))
    with torch.no_grad():
        out = models[mf](torch.from_numpy(g["x"]).cuda(), [torch.tensor([[0.5]])])[0][0]
    ok, worst, dmax = elementwise_ok(out, g["out"])
    assert ok, (worst, dmax)
    gt = np.round(np.clip(g["out"].astype(np.float64), 0, 1) * 255) / 255
    psnr = lambda a: 10 * np.log10(1.0 / np.mean((np.asarray(a, np.float64) - gt) ** 2))
    assert abs(psnr(out.cpu().numpy()) - psnr(g["out"])) < 1e-3


@pytest.mark.parametrize("mf", ["f16x3", "f32"])
def test_c1_full_pair_matches_reference_at_pins(models, mf):
    """BASELINE config C1 at full size: one 256x256 pair (bench.py's frames 0-1), 4x, t = 0.5, against the
    reference model's own latent and 1024x1024 output (tests/golden/make_golden.py c1) at the positions
    make_golden.c1_pins keeps: the rows / columns where the engine's conv, DCN and decoder tiles meet,
    the frame edges, and random pixels -- elementwise |a - b| <= 1e-4 |b| + 1e-6."""
    g = np.load(os.path.join(GOLD, "c1_pair_pins.npz"))
    m = models[mf]
    with torch.no_grad():
        out = m(torch.from_numpy(g["x"]).cuda(), [torch.tensor([[0.5]])])[0][0]
        feat = m.feat[0]                                       # [3, 64, 256, 256] (view of the NHWC latent)
        fy, fx = torch.from_numpy(g["feat_y"]).cuda(), torch.from_numpy(g["feat_x"]).cuda()
        oy, ox = torch.from_numpy(g["out_y"]).cuda(), torch.from_numpy(g["out_x"]).cuda()
        ok, worst, dmax = elementwise_ok(feat[:, :, fy, fx], g["feat"])
        assert ok, ("latent", worst, dmax)
        assert tuple(out.shape) == (3, 1024, 1024)
        ok, worst, dmax = elementwise_ok(out[:, oy, ox], g["out"])
        assert ok, ("output", worst, dmax)


def test_c0_window_pairs_equal_single_pairs(models):
    """The C0 7-frame window (bench's workload) batched = every pair run alone, bit for bit."""
    fr = synth(0, 7, 128, 128)
    m = models["f16x3"]
    with torch.no_grad():
        m.gen_feat_window(fr)
        win = m.decoding([torch.tensor([[0.5]])])[0].clone()
        for p in (0, 5):
            one = m(torch.stack([fr[p], fr[p + 1]])[None], [0.5])[0]
            assert torch.equal(win[p:p + 1], one), p


def test_c0_window_dcn_sep_launches_deterministic(stif, models):
    """Every fused DCN_sep launch of the C0 window (k_dcn_sep: the L3 / L2 / L1 alignments of the PCD and
    the three Bi-ConvLSTM steps, launch groups of up to 8 weight sets at two waves per SIMD), re-run into
    fresh buffers, reproduces its output bit for bit (a kernel whose result depended on wave timing --
    the removed tap-pipelined form -- fails here)."""
    fr = synth(0, 7, 128, 128)
    ops = stif.ops
    orig = ops.dcn_sep
    seen = []

    def traced(groups, epi=0, status=None):
        orig(groups, epi=epi, status=status)
        ref = [g["out"].clone() for g in groups]
        for _ in range(2):
            g2 = [dict(g, out=torch.full_like(g["out"], float("nan"))) for g in groups]
            orig(g2, epi=epi, status=None)
            seen.append(all(torch.equal(a["out"], b) for a, b in zip(g2, ref)))
    ops.dcn_sep = traced
    try:
        with torch.no_grad():
            models["f16x3"].gen_feat_window(fr)
    finally:
        ops.dcn_sep = orig
    assert len(seen) >= 2 * 12 and all(seen), seen


@pytest.mark.parametrize("mf", ["f16x3", "f32"])
def test_c0_window_runs_bit_identical(models, mf):
    """The whole C0 window (encoder, PCD, Bi-ConvLSTM, recon trunk on its side streams, both decoder stages) run three
    times on the same frames gives the same latent and the same decoded frames bit for bit, in both operand modes:
    no kernel of the path may depend on wave timing or co-residency (the property the packed-fp32 tap-pipelined
    DCN_sep broke)."""
    fr = synth(0, 7, 128, 128)
    m = models[mf]
    runs = []
    with torch.no_grad():
        for _ in range(3):
            m.gen_feat_window(fr)
            runs.append((m.feat.clone(), [o.clone() for o in m.decoding([torch.tensor([[0.5]]), torch.tensor([[0.75]])])]))
    for feat, outs in runs[1:]:
        assert torch.equal(feat, runs[0][0])
        assert all(torch.equal(a, b) for a, b in zip(outs, runs[0][1]))


CONFIG_CASES = {
    # BASELINE configs[1..4] at their full per-GPU sizes: (frames, H, W, output size or None, times)
    "C1": (7, 256, 256, None, [0.5]),
    "C2": (7, 540, 960, None, [0.25, 0.5, 0.75]),
    "C3_rank": (9, 720, 1280, None, [0.0, 0.5]),           # 64 frames / 8 ranks: 8 pairs per rank
    "C4_rank": (2, 1080, 1920, (2700, 4800), [0.0, 0.25, 0.5, 0.75]),   # 1080p -> 2.5x, 4 t
}


@pytest.mark.parametrize("cfg", sorted(CONFIG_CASES))
def test_config_full_size_f16x3_vs_f32(models, cfg):
    F_, H, W, size, times = CONFIG_CASES[cfg]
    fr = synth(0, F_, H, W)
    tq = [torch.tensor([[t]]) for t in times]
    outs = {}
    with torch.no_grad():
        for mf in ("f16x3", "f32"):
            m = models[mf]
            m.gen_feat_window(fr)
            outs[mf] = m.decoding(tq, size)
            m._feat = None
    for a, b in zip(outs["f16x3"], outs["f32"]):
        HH, WW = size or (4 * H, 4 * W)
        assert tuple(a.shape) == (F_ - 1, 3, HH, WW)
        assert bool(torch.isfinite(a).all()) and bool(torch.isfinite(b).all())
        ok, worst, dmax = elementwise_ok(a, b)
        assert ok, (cfg, worst, dmax)
    del outs
    torch.cuda.empty_cache()


def test_chunked_window_is_bit_identical(models):
    """Pair chunking of the encoder (chunk_px) and of the decoder (dec_chunk_px): bounded working sets at
    720p / 1080p, not a bit changed."""
    m = models["f16x3"]
    fr = synth(3, 5, 64, 96)
    with torch.no_grad():
        keep = m.chunk_px
        m.gen_feat_window(fr)
        a = m.decoding([0.5])[0].clone()
        m.chunk_px = 64 * 96 + 1          # one pair per chunk
        m.gen_feat_window(fr)
        b = m.decoding([0.5])[0]
        m.chunk_px = keep
        keep = m.dec_chunk_px
        m.dec_chunk_px = 2 * 256 * 384      # decoder passes of two pairs (2, 2, 0 + the last one)
        c = m.decoding([0.5])[0]
        m.dec_chunk_px = keep
    assert torch.equal(a, b)
    assert torch.equal(a, c)


def test_lanes_are_bit_identical(models):
    """Lanes (concurrent streams over pair ranges, LunaTokis(lanes=)), trunk lanes (the recon trunk's
    items over streams, trunk_lanes=), decoder lanes (dec_lanes=), the BiConvLSTM directions on two
    streams (lstm_lanes=2) and the PCD DCN branch on a side stream (pcd_streams=2) do not change a bit:
    the window path
    (shared boundary frames encoded per lane), the gen_feat(x) path and decoding, against one stream
    everywhere (4 lanes over 5 pairs: ranges 2, 2, 1; trunk 15 items as 8 + 7 or 5 + 5 + 5)."""
    m = models["f16x3"]
    fr = synth(20, 6, 64, 96)
    x = torch.stack([fr[:-1], fr[1:]], 1)
    keep = (m.lanes, m.trunk_lanes, m.dec_lanes, m.lstm_lanes, m.pcd_streams)
    res = {}
    combos = [(1, 1, None, 1, 1), (2, 1, None, 1, 1), (4, 1, None, 1, 1), (1, 2, None, 1, 1), (1, 3, None, 1, 1),
              (2, 2, None, 1, 1), (1, 2, 2, 1, 1), (1, 1, None, 2, 1), (2, 2, None, 2, 1), (1, 2, None, 1, 2),
              (2, 2, None, 2, 2)]
    with torch.no_grad():
        try:
            for k in combos:
                m.lanes, m.trunk_lanes, m.dec_lanes, m.lstm_lanes, m.pcd_streams = k
                m.gen_feat_window(fr)
                f = m.feat.clone()
                d = [o.clone() for o in m.decoding([0.25, 0.5])]
                g = m(x, [0.75])[0].clone()
                res[k] = (f, d, g)
        finally:
            m.lanes, m.trunk_lanes, m.dec_lanes, m.lstm_lanes, m.pcd_streams = keep
    ref = res[combos[0]]
    for k in combos[1:]:
        assert torch.equal(res[k][0], ref[0]), k
        assert all(torch.equal(a, b) for a, b in zip(res[k][1], ref[1])), k
        assert torch.equal(res[k][2], ref[2]), k


@pytest.mark.parametrize("mf", ["f16x3", "f32"])
def test_zero_state_l1_skip_is_bit_identical(models, mf):
    """PCD alignment of the ConvLSTM's first step: a unit whose sampled L1 map is the all-zero initial
    state gets its L1 DCN bias without running the L1 offset branch (_pcd_align zero_l1) -- the
    same bits as running it."""
    m = models[mf]
    B, H, W = 2, 32, 48
    g = torch.Generator(device="cuda").manual_seed(5)
    lv = [(H, W), (H // 2, W // 2), (H // 4, W // 4)]
    x = [torch.rand(B, h, w, 64, device="cuda", generator=g) for h, w in lv]
    st = [torch.zeros(B, H, W, 64, device="cuda")] + [torch.rand(B, h, w, 64, device="cuda", generator=g)
                                                      for h, w in lv[1:]]
    pf = "ConvBLSTM.forward_net.pcd_c.pcd_align."
    outs = []
    for zl in ((), (1,)):
        y = torch.full((2, B, H, W, 64), float("nan"), device="cuda")
        with torch.no_grad():
            m._call(m._pcd_align, [(pf, 1, x, st, y[0]), (pf, 2, st, x, y[1])], zero_l1=zl)
        outs.append(y)
    assert bool(torch.isfinite(outs[1]).all())
    assert torch.equal(outs[0], outs[1])


def test_halo_features_are_bit_identical(models, stif):
    """The multi-GPU halo path: the boundary frame's encoder features handed in (last_frame_feats /
    frame_feats, what parallel.halo_exchange delivers) give bit-identical latents and outputs."""
    m = models["f16x3"]
    fr = synth(10, 4, 64, 64)
    with torch.no_grad():
        m.gen_feat_window(fr)
        ref_feat = m.feat.clone()
        ref = m.decoding([0.25])[0].clone()
        last = m.frame_features(fr[-1:])
        m.gen_feat_window(fr, last_frame_feats=last)
        assert torch.equal(m.feat, ref_feat)
        assert torch.equal(m.decoding([0.25])[0], ref)
        allf = m.frame_features(fr)
        m.gen_feat_window(fr, frame_feats=allf)
        assert torch.equal(m.feat, ref_feat)
        # a one-rank "world": gen_feat_shard without a neighbour is the plain window
        stif.parallel.gen_feat_shard(m, fr, 0, 1)
        assert torch.equal(m.feat, ref_feat)


def test_module_api_dataparallel_and_device(models, golden):
    """nn.Module drop-in: DataParallel(netG) as VideoSR_base_model.py:29-32 wraps it, state_dict
    round trip, and a call made while another device context / stream is current."""
    m = models["f16x3"]
    g = golden["model_16x20"]
    x = torch.from_numpy(g["x"]).cuda()
    tq = [torch.tensor([[0.5]]).cuda()]
    with torch.no_grad():
        ref = m(x, tq)[0].clone()
        dp = torch.nn.DataParallel(m)
        out = dp(x, tq)[0]
        assert torch.equal(out, ref)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            out2 = m(x, tq)[0]
        s.synchronize()
        assert torch.equal(out2, ref)
    sd = m.state_dict()
    assert len(sd) == 442 and all(not v.requires_grad for v in m.parameters())


def test_f16x3_activation_range_is_guarded(stif, sd, golden):
    """Inputs far outside the split-fp16 range: the kernels flag the non-finite outputs, the call is
    re-run in fp32 (bit-identical to an fp32-MFMA model), or raises with range_check='raise';
    never silent inf/NaN."""
    x = torch.from_numpy(golden["model_16x20"]["x"] * 5000.0).cuda()
    tq = [torch.tensor([[0.5]])]
    mk = lambda **kw: stif.LunaTokis(64, 6, 8, 5, 40, **kw)
    m16, m32, mr = mk(), mk(mfma="f32"), mk(range_check="raise")
    for m in (m16, m32, mr):
        m.load_state_dict(sd)
    with torch.no_grad():
        ref = m32(x, tq)[0]
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            out = m16(x, tq)[0]
        assert m16.range_reruns >= 1 and any("split-fp16 range" in str(i.message) for i in w)
        assert bool(torch.isfinite(out).all())
        assert torch.equal(out, ref)
        with pytest.raises(stif._lib.StifError):
            mr(x, tq)
        # in range: no re-run
        n = m16.range_reruns
        m16(torch.from_numpy(golden["model_16x20"]["x"]).cuda(), tq)
        assert m16.range_reruns == n


def test_f16x3_weight_range_falls_back_per_layer(stif, sd, golden):
    """A weight outside the split range (|U| >= 64) makes its layer pack in fp32 (the others stay
    f16x3); the forward still matches the fp64 oracle on the same state dict."""
    sd2 = dict(sd)
    k = "recon_trunk.3.conv1.weight"
    sd2[k] = sd[k].copy()
    sd2[k][5, 7, 0, 0] = 80.0      # one corner tap: U[0][0] = 80 > 64, activations stay in range
    m = stif.LunaTokis(64, 6, 8, 5, 40)
    m.load_state_dict(sd2)
    x = golden["model_16x20"]["x"]
    with torch.no_grad():
        out = m(torch.from_numpy(x).cuda(), [0.5])[0]
    lay = m.layers["recon_trunk.3.conv1"]
    assert not lay.mode & stif._lib.PACK_F16X3
    assert m.layers["recon_trunk.3.conv2"].mode & stif._lib.PACK_F16X3
    ref = O.forward(x, [0.5], sd2)[0]
    d = np.abs(out.cpu().numpy() - ref).max()
    assert d <= 1e-4 * np.abs(ref).max() + 1e-6, d


def test_single_forward_matches_reference_harness(stif, models):
    """custom_video_test.py:41-54 (single_forward): an 11x13 pair zero-padded to 12x16, eight times
    i/8, uncropped 48x64 outputs -- against the reference run of the same five lines."""
    g = np.load(os.path.join(GOLD, "single_11x13.npz"))
    outs = stif.video.single_forward(models["f16x3"], torch.from_numpy(g["x"]).cuda())
    assert len(outs) == 8
    for i, o in enumerate(outs):
        assert tuple(o.shape) == (1, 3, 48, 64)
        ok, worst, dmax = elementwise_ok(o[0], g["out"][i])
        assert ok, (i, worst, dmax)


def test_f16x3_dcn_sep_range_flag_triggers_rerun(stif, sd, golden):
    """The model's range guard through k_dcn_sep's own flag (advisor finding, round 3): only the first
    fused DCN_sep launch sees a poisoned offset feature (one value of 5000, outside the split range);
    that launch itself sets the status word, the call is re-run in fp32 (range_reruns + 1), and the
    result equals an fp32-MFMA model's on the clean input."""
    ops = stif.ops
    orig = ops.dcn_sep
    seen = []

    def poisoned(groups, epi=0, status=None):
        if not seen:
            g0 = dict(groups[0])
            f = g0["fea"].clone()
            f.view(-1)[f.numel() // 3] = 5000.0
            g0["fea"] = f
            groups = [g0] + list(groups[1:])
            if status is not None:
                status.zero_()
            orig(groups, epi=epi, status=status)
            seen.append(None if status is None else int(status.item()))
            return
        orig(groups, epi=epi, status=status)

    x = torch.from_numpy(golden["model_16x20"]["x"]).cuda()
    m16 = stif.LunaTokis(64, 6, 8, 5, 40)
    m32 = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f32")
    for m in (m16, m32):
        m.load_state_dict(sd)
    with torch.no_grad():
        ref = m32(x, [0.5])[0]
        ops.dcn_sep = poisoned
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                out = m16(x, [0.5])[0]
        finally:
            ops.dcn_sep = orig
    assert seen == [1], seen
    assert m16.range_reruns == 1
    assert torch.equal(out, ref)


LARGE_WINDOWS = {
    # fixture: frames in the window (pairs chosen so chunk_px = 2^21 LR pixels splits the encoder's pairs:
    # C2 5 pairs -> chunks of 3 + 2, C3 3 pairs -> 2 + 1, C4 2 pairs -> 1 + 1)
    "c2": 6,
    "c3": 4,
    "c4": 3,
}


@pytest.mark.parametrize("mf", ["f16x3", "f32"])
@pytest.mark.parametrize("cfg", sorted(LARGE_WINDOWS))
def test_large_config_latent_matches_reference_at_pins(models, cfg, mf):
    """BASELINE configs[2..4] at full size: the reference's own encoder (gen_feat, Sakuya_arch_test.py:313-362)
    run on bench.py's frames 0-1 at 540x960 / 720x1280 / 1080x1920 (tests/golden/make_golden.py c2|c3|c4)
    against pair 0 of a multi-pair window of this engine -- the window is long enough that chunk_px splits
    its pairs into several encoder passes -- at the tile seams of every pyramid level (incl. the partial last
    32-column L3 tile at 960 / 1920), the frame edges and random pixels, elementwise
    |a - b| <= 1e-4 |b| + 1e-6."""
    path = os.path.join(GOLD, f"{cfg}_pair_feat_pins.npz")
    if not os.path.exists(path):
        pytest.skip(f"{cfg} fixture not generated")
    g = np.load(path)
    H, W = int(g["H"]), int(g["W"])
    m = models[mf]
    n = LARGE_WINDOWS[cfg]
    per = max(1, m.chunk_px // (H * W))
    assert per < n - 1, "the window must span more than one encoder chunk"
    fr = synth(0, n, H, W)
    with torch.no_grad():
        m.gen_feat_window(fr)
        feat = m.feat[0]                                       # pair 0: [3, 64, H, W]
        fy, fx = torch.from_numpy(g["feat_y"]).cuda(), torch.from_numpy(g["feat_x"]).cuda()
        got = feat[:, :, fy, fx]
        m._feat = None
    ok, worst, dmax = elementwise_ok(got, g["feat"])
    assert ok, (cfg, mf, worst, dmax)
    del fr, feat, got
    torch.cuda.empty_cache()
