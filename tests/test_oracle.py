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
