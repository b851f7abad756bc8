"""The CPU oracle against the golden fixtures produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from oracle import stif_oracle as O


def relmax(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def test_dcn_zero_offset_kat(golden):
    """DCNv2/test.py:32-67: zero offset, mask = sigmoid(0), identity kernel -> 2*dcn(x) == x."""
    x = golden["ops"]["kat_input"].astype(np.float64)
    N, C, H, W = x.shape
    w = np.zeros((C, C, 3, 3))
    for p in range(C):
        w[p, p, 1, 1] = 1.0
    out = O.dcn_v2_forward(x, w, np.zeros(C), np.zeros((N, 18, H, W), np.float32),
                           np.full((N, 9, H, W), 0.5), 3, 3, 1, 1, 1, 1, 1, 1, 1)
    assert np.abs(x - 2 * out).max() < 1e-10


def test_dcn_sep_module(golden, sd):
    g = golden["ops"]
    out = O.dcn_sep(g["dcnsep_in"], g["dcnsep_fea"], sd, "pcd_align.L2_dcnpack_1")
    assert relmax(out, g["dcnsep_out"]) < 2e-5


def test_upsample(golden):
    g = golden["ops"]
    assert relmax(O.upsample2x(g["up2_in"].astype(np.float64)), g["up2_out"]) < 1e-6


def test_grid_sample_bilinear(golden):
    g = golden["ops"]
    img = g["gs_in"]
    grid = g["gs_grid"][0, 0]
    out = O.bilinear_sample(img, grid[None, :, 0], grid[None, :, 1])   # [1,Q,C]
    ref = g["gs_bilinear"][0, :, 0].T
    assert relmax(out[0], ref) < 1e-5


def test_siren(golden, sd):
    g = golden["ops"]
    assert relmax(O.siren(g["siren_in"].astype(np.float64), sd, "feat_imnet.", 3, np.float64), g["siren_out"]) < 1e-5


def test_convlstm_cell(golden, sd):
    g = golden["ops"]
    h, c = O.conv_lstm_cell(g["cell_x"], g["cell_h"], g["cell_c"], sd, "ConvBLSTM.forward_net.cell_list.0.", np.float64)
    assert relmax(h, g["cell_hn"]) < 1e-5
    assert relmax(c, g["cell_cn"]) < 1e-5


def test_make_coord_and_linspace(golden):
    g = golden["ops"]
    c = g["coord_40x50"].reshape(40, 50, 2)
    assert np.array_equal(O.make_coord_1d(40), c[:, 0, 0])
    assert np.array_equal(O.make_coord_1d(50), c[0, :, 1])
    # warpgrid base (flow = 0 part of warp_grid)
    fl = g["warp_flow"][0]
    grid = g["warp_grid"][0]
    gx = O.linspace_f32(16)[None, :] + fl[0] / ((16 - 1.0) / 2.0)
    gy = O.linspace_f32(12)[:, None] + fl[1] / ((12 - 1.0) / 2.0)
    assert np.abs(gx - grid[..., 0]).max() < 1e-6
    assert np.abs(gy - grid[..., 1]).max() < 1e-6


@pytest.fixture(scope="module")
def model_run(golden, sd):
    g = golden["model_16x20"]
    cap = {}
    outs = O.forward(g["x"], [float(t) for t in g["times"]], sd, capture=cap)
    return g, cap, outs


def test_model_intermediates(model_run):
    g, cap, _ = model_run
    assert relmax(cap["pcd_align"][0], g["pcd_align"]) < 1e-5
    assert relmax(cap["fusion"][0], g["fusion"]) < 1e-5
    assert relmax(cap["bilstm"][0], g["bilstm"]) < 1e-5
    assert relmax(cap["feat"][0], g["feat"]) < 1e-5
    assert relmax(cap["hrfeat"][2][0], g["hrfeat_t05"]) < 1e-5
    assert relmax(cap["flow"][2][0], g["flow_t05"]) < 1e-5


def test_model_outputs(model_run, sd):
    g, cap, outs = model_run
    for i in range(len(outs)):
        assert relmax(outs[i][0], g["out"][i]) < 1e-5
    o25 = O.decoding(cap["feat"], g["x"], [0.5], sd, scale=(40, 50))[0]
    assert relmax(o25[0], g["out_scale_40x50"]) < 1e-5


def test_window(golden, sd):
    g = golden["window_7x16x16"]
    fr = g["frames"]
    x = np.stack([fr[:-1], fr[1:]], axis=1)      # 6 pairs batched: pairs are independent
    outs = O.forward(x, [0.5], sd)[0]
    assert relmax(outs, g["out"]) < 1e-5


@pytest.mark.parametrize("which", ["test", "test_scale3", "fast", "fast_40x50", "ens", "ens_40x50"])
def test_oracle_decoder_variants_match_reference(sd, golden, which):
    """decoding_test / decoding_fasttest / decoding_localensemble restatements against the
    reference's own outputs (tests/golden/decoders_16x20.npz, same latent as model_16x20)."""
    g, d = golden["model_16x20"], golden["decoders_16x20"]
    feat, x = g["feat"][None], g["x"]
    if which == "test":
        got, ref = np.stack([o[0] for o in O.decoding_test(feat, x, list(d["test_times"]), sd)]), d["test_out"]
    elif which == "test_scale3":
        got, ref = O.decoding_test(feat, x, [0.5], sd, scale=3)[0][0], d["test_out_scale3"]
    elif which == "fast":
        got, ref = O.decoding_fasttest(feat, x, list(d["fast_times"]), sd), d["fast_out"]
    elif which == "fast_40x50":
        got, ref = O.decoding_fasttest(feat, x, [0.5], sd, (40, 50)), d["fast_out_40x50"]
    elif which == "ens":
        got, ref = O.decoding_localensemble(feat, x, [0.5], sd), d["ens_out"]
    else:
        got, ref = O.decoding_localensemble(feat, x, [0.25], sd, (40, 50)), d["ens_out_40x50"]
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_oracle_imresize_matches_reference():
    """data.util.imresize_np(uint8 BGR frame, 1/2, True) restatement vs the reference's outputs."""
    h = np.load(os.path.join(os.path.dirname(__file__), "golden", "harness.npz"))
    w, i0, s0, s1 = O.resize_weights_indices(37, 19, 0.5)
    assert np.array_equal(w, h["w_37_19"]) and np.array_equal(i0, h["i_37_19"][:, 0])
    assert (s0, s1) == tuple(h["sym_37_19"])
    for k in ("37x50", "64x90", "21x33"):
        assert np.abs(O.imresize_np(h["img_" + k], 0.5) - h["half_" + k]).max() < 1e-3


def _dcn_fd_case(seed, B=2, C=2, H=4, W=4, Co=2, dg=1, k=3, s=1, p=1, d=1):
    """DCNv2/test.py:69-103 check_gradient_dconv inputs: input U[0,1)*0.01, offset N(0,1)*2,
    mask sigmoid(U[0,1)), weight N(0,1), bias U[0,1)."""
    rng = np.random.default_rng(seed)
    Ho = (H + 2 * p - (d * (k - 1) + 1)) // s + 1
    Wo = (W + 2 * p - (d * (k - 1) + 1)) // s + 1
    x = rng.random((B, C, H, W)) * 0.01
    off = (rng.standard_normal((B, dg * 2 * k * k, Ho, Wo)) * 2).astype(np.float32)
    msk = 1 / (1 + np.exp(-rng.random((B, dg * k * k, Ho, Wo))))
    w = rng.standard_normal((Co, C, k, k))
    b = rng.random(Co)
    go = rng.standard_normal((B, Co, Ho, Wo))
    return x, w, b, off, msk, go, (k, k, s, s, p, p, d, d, dg)


@pytest.mark.parametrize("case", [dict(seed=3), dict(seed=4, dg=2, C=4, Co=3),
                                  dict(seed=5, H=6, W=5, s=2, d=2, p=2, C=2, Co=2)])
def test_dcn_backward_oracle_matches_finite_differences(case):
    """The backward restatement (dcn_v2_cuda_backward) against central differences of the forward
    restatement at the reference's own gradcheck configuration and tolerances (DCNv2/test.py:69-103:
    eps 1e-3, atol 1e-4, rtol 1e-2), over every input of dcn_v2_conv."""
    x, w, b, off, msk, go, dims = _dcn_fd_case(**case)
    gi, goff, gm, gw, gb = O.dcn_v2_backward(x, w, b, off, msk, go, *dims)
    f = lambda x_, w_, b_, o_, m_: float((O.dcn_v2_forward(x_, w_, b_, o_, m_, *dims) * go).sum())
    args = [x, w, b, off, msk]

    def fd(ai, eps):
        num = np.zeros(args[ai].shape)
        for idx in np.ndindex(args[ai].shape):
            ap, am = [a.copy() for a in args], [a.copy() for a in args]
            ap[ai][idx] += eps
            am[ai][idx] -= eps
            num[idx] = (f(*ap) - f(*am)) / (2 * eps)
        return num
    for ai, g in zip(range(5), (gi, gw, gb, goff, gm)):
        num = fd(ai, 1e-3)
        tol = dict(atol=1e-4 * max(1.0, np.abs(num).max()), rtol=1e-2)
        if ai == 3:
            # the output is piecewise bilinear in the offsets: a sample within eps of a cell edge or of
            # the (-1, H) gate has no derivative there; such elements are the ones whose difference
            # quotient changes with eps (at most a few of them)
            smooth = np.isclose(num, fd(ai, 2.5e-4), **tol)
            assert smooth.mean() > 0.98
            g, num = g[smooth], num[smooth]
        np.testing.assert_allclose(g, num, **tol)


@pytest.mark.parametrize("size", [None, (40, 50)], ids=["4x", "2.5x"])
def test_decoding_at_pixels_equals_full_decode(golden, sd, size):
    """decoding_at (the pixel-subset decoder the full-size GPU tests pin against) = the full oracle
    decode at every pixel it is asked for, incl. the 2.5x round-half-even tie rows/columns, the last
    row/column and samples whose warped grid is clamped at the frame edge; and the full decode is the
    reference's own output (fixture)."""
    g = golden["model_16x20"]
    feat, x = g["feat"].reshape(1, 3, 64, *g["feat"].shape[-2:]), g["x"]
    H, W = feat.shape[-2:]
    HH, WW = size or (4 * H, 4 * W)
    full = O.decoding(feat, x, [0.5, 0.25], sd, size)
    rng = np.random.default_rng(3)
    py = np.concatenate([rng.integers(0, HH, 300), np.full(20, HH - 1), np.arange(20) % HH, [0, HH - 1]])
    px = np.concatenate([rng.integers(0, WW, 300), rng.integers(0, WW, 20), np.full(20, WW - 1), [WW - 1, 0]])
    # a strided view, as the GPU engine's latent arrives ([3,B,H,W,64] NHWC permuted)
    fv = np.ascontiguousarray(feat.transpose(1, 0, 3, 4, 2)).transpose(1, 0, 4, 2, 3)
    st = {}
    sub = O.decoding_at(fv, x, [0.5, 0.25], sd, HH, WW, py, px, stats=st)
    for a, b in zip(sub, full):
        assert relmax(a, b[:, :, py, px]) < 1e-12
    assert st["clamped"] > 0
    if size is None:
        assert relmax(full[0][0], g["out"][2]) < 1e-5                    # t = 0.5
    else:
        assert relmax(full[0], g["out_scale_40x50"]) < 1e-5


def test_c1_pin_fixture_is_consistent():
    """c1_pair_pins.npz (make_golden.py c1: the reference's own 256x256 pair) keeps exactly the positions
    make_golden.c1_pins() names -- tile seams, frame edges, random pixels -- with finite values, and its
    input is bench.py's frames 0-1 (seeds 1234 / 1235)."""
    import importlib.util
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(here, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    g = np.load(os.path.join(here, "golden", "c1_pair_pins.npz"))
    fy, fx, oy, ox = mg.c1_pins()
    for k, v in (("feat_y", fy), ("feat_x", fx), ("out_y", oy), ("out_x", ox)):
        assert np.array_equal(g[k], v), k
    assert g["feat"].shape == (3, 64, len(fy)) and g["out"].shape == (3, len(oy))
    assert np.isfinite(g["feat"]).all() and np.isfinite(g["out"]).all()
    for i in range(2):
        fr = torch.rand(3, 256, 256, generator=torch.Generator().manual_seed(1234 + i)).numpy()
        assert np.array_equal(g["x"][0, i], fr)


def test_chunked_dcn_shim_equals_unchunked_and_oracle():
    """the C2 / C3 / C4 latent fixtures come from make_golden's row-chunked CPU DCN shim.  Its
    equality with the unchunked shim (which the model fixtures use) was only printed by `make_golden.py
    chunk-check`; here it is asserted on that case (offsets up to 6 px, 150 rows in 32-row blocks incl. a
    partial one and both image edges), and both shims are checked against the oracle's restatement."""
    import importlib.util
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(here, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    g = torch.Generator().manual_seed(5)
    B, C, H, W, dg = 1, 16, 150, 40, 2
    inp = torch.randn(B, C, H, W, generator=g)
    wt = torch.randn(8, C, 3, 3, generator=g)
    bs = torch.randn(8, generator=g)
    off = torch.rand(B, 2 * dg * 9, H, W, generator=g) * 12 - 6
    m = torch.rand(B, dg * 9, H, W, generator=g)
    a = mg.dcn_v2_forward_cpu(inp, wt, bs, off, m, 3, 3, 1, 1, 1, 1, 1, 1, dg)
    b = mg.dcn_v2_forward_cpu_chunked(inp, wt, bs, off, m, 3, 3, 1, 1, 1, 1, 1, 1, dg, rows=32)
    scale = float(a.abs().max())
    assert float((a - b).abs().max()) <= 1e-6 * scale
    ref = O.dcn_v2_forward(inp.numpy().astype(np.float64), wt.numpy().astype(np.float64), bs.numpy().astype(np.float64),
                           off.numpy(), m.numpy(), 3, 3, 1, 1, 1, 1, 1, 1, dg)
    assert np.abs(b.numpy() - ref).max() <= 1e-5 * scale
