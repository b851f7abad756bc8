"""Per-kernel parity of the HIP path (through the C ABI) against the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5   # fp32 MFMA vs fp64 oracle, relative to max |ref|


def relmax(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def nhwc(x_nchw):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x_nchw, np.float32).transpose(0, 2, 3, 1))).cuda()


def to_nchw(t):
    return t.detach().cpu().numpy().transpose(0, 3, 1, 2)


@pytest.fixture(scope="module")
def L(stif):
    return stif._lib


@pytest.fixture(scope="module")
def ops(stif):
    return stif.ops


def rnd(*shape, seed=0, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


@pytest.mark.parametrize("epi", ["none", "lrelu", "relu", "res"])
@pytest.mark.parametrize("hw", [(13, 37), (8, 32), (33, 70)])
def test_conv3x3(ops, L, epi, hw):
    H, W = hw
    x = rnd(3, 64, H, W, seed=1)
    w = rnd(64, 64, 3, 3, seed=2, scale=0.05)
    b = rnd(64, seed=3)
    r = rnd(3, 64, H, W, seed=4)
    ref = O.conv2d(x, w, b)
    e = dict(none=L.EPI_NONE, lrelu=L.EPI_LRELU, relu=L.EPI_RELU, res=L.EPI_RES)[epi]
    if epi == "lrelu":
        ref = O.lrelu(ref)
    if epi == "relu":
        ref = O.relu(ref)
    if epi == "res":
        ref = ref + r
    layer = ops.pack_conv(w, b)
    out = torch.empty(3, H, W, 64, device="cuda")
    ops.conv2d([dict(layer=layer, in0=nhwc(x), out=out, res=nhwc(r) if epi == "res" else None)], epi=e)
    assert relmax(to_nchw(out), ref) < RTOL


@pytest.mark.parametrize("mode", [1, 2])
def test_conv_two_inputs_and_upsample(ops, L, mode):
    H, W = 14, 38
    x0 = rnd(2, 64, H, W, seed=5)
    h1, w1 = (H, W) if mode == 1 else (H // 2, W // 2)
    x1 = rnd(2, 64, h1, w1, seed=6)
    w = rnd(64, 128, 3, 3, seed=7, scale=0.04)
    b = rnd(64, seed=8)
    up = x1.astype(np.float64) if mode == 1 else O.upsample2x(x1.astype(np.float64)) * 2
    ref = O.lrelu(O.conv2d(np.concatenate([x0, up], 1), w, b))
    out = torch.empty(2, H, W, 64, device="cuda")
    ops.conv2d([dict(layer=ops.pack_conv(w, b), in0=nhwc(x0), in1=nhwc(x1), out=out)], epi=L.EPI_LRELU,
               in1_mode=mode, in1_scale=1.0 if mode == 1 else 2.0)
    assert relmax(to_nchw(out), ref) < RTOL


def test_conv_groups_and_strided_items(ops, L):
    """Two weight groups over strided item views (the PCD direction batching)."""
    H, W = 12, 20
    fr = rnd(6, 64, H, W, seed=9)
    wa, wb = rnd(64, 128, 3, 3, seed=10, scale=0.04), rnd(64, 128, 3, 3, seed=11, scale=0.04)
    ba, bb = rnd(64, seed=12), rnd(64, seed=13)
    t = nhwc(fr)
    f1, f2 = t[0::2], t[1::2]
    out = torch.empty(2, 3, H, W, 64, device="cuda")
    ops.conv2d([dict(layer=ops.pack_conv(wa, ba), in0=f1, in1=f2, out=out[0]),
                dict(layer=ops.pack_conv(wb, bb), in0=f2, in1=f1, out=out[1])], in1_mode=1)
    refa = O.conv2d(np.concatenate([fr[0::2], fr[1::2]], 1), wa, ba)
    refb = O.conv2d(np.concatenate([fr[1::2], fr[0::2]], 1), wb, bb)
    assert relmax(to_nchw(out[0]), refa) < RTOL
    assert relmax(to_nchw(out[1]), refb) < RTOL


@pytest.mark.parametrize("f16", [0, 1], ids=["f32", "f16x3"])
@pytest.mark.parametrize("hw", [(20, 36), (7, 13)])
def test_conv_stride2(ops, L, f16, hw):
    H, W = hw
    x = rnd(2, 64, H, W, seed=14)
    w = rnd(64, 64, 3, 3, seed=15, scale=0.05)
    b = rnd(64, seed=16)
    out = torch.empty(2, (H + 1) // 2, (W + 1) // 2, 64, device="cuda")
    lay = ops.pack_conv(w, b, L.PACK_PLAIN | (L.PACK_F16X3 if f16 else 0))
    ops.conv2d([dict(layer=lay, in0=nhwc(x), out=out)], epi=L.EPI_LRELU, stride=2)
    assert relmax(to_nchw(out), O.lrelu(O.conv2d(x, w, b, stride=2))) < RTOL


def test_conv_f16x3_rejects_other_shapes(ops, L):
    lay = ops.pack_conv(rnd(64, 64, 3, 3), rnd(64), L.PACK_PLAIN | L.PACK_F16X3)
    x = torch.zeros(1, 8, 8, 64, device="cuda")
    with pytest.raises(Exception):   # stride 1 direct conv has no f16x3 form
        ops.conv2d([dict(layer=lay, in0=x, out=torch.empty(1, 8, 8, 64, device="cuda"))])


@pytest.mark.parametrize("f16", [0, 1], ids=["f32", "f16x3"])
def test_conv1x1_wide(ops, L, f16):
    """The decoder's LR projection shape (200 -> 256): direct fp32 kernel, or k_conv1x1<13> whose last
    16-channel chunk is half used."""
    x = rnd(2, 200, 9, 11, seed=17)
    w = rnd(256, 200, 1, 1, seed=18, scale=0.05)
    b = rnd(256, seed=19)
    out = torch.full((2, 9, 11, 256), float("nan"), device="cuda")
    lay = ops.pack_conv(w, b, L.PACK_PLAIN | (L.PACK_F16X3 if f16 else 0))
    assert bool(lay.mode & L.PACK_F16X3) == bool(f16)
    ops.conv2d([dict(layer=lay, in0=nhwc(x), out=out)])
    assert relmax(to_nchw(out), O.conv2d(x, w, b)) < RTOL


@pytest.mark.parametrize("hw", [(12, 20), (7, 13), (32, 48)])   # 240 and 91 px: partial last M-tile
def test_conv1x1_cat_f16x3(ops, L, hw):
    """k_conv1x1 (the fusion / conv_1x1 convs on cat(a, b), split-fp16): two weight groups over
    strided item views, items whose pixel count is not a multiple of the 32-pixel M-tile."""
    H, W = hw
    fr = rnd(6, 64, H, W, seed=40)
    wa, wb = rnd(64, 128, 1, 1, seed=41, scale=0.1), rnd(64, 128, 1, 1, seed=42, scale=0.1)
    ba, bb = rnd(64, seed=43), rnd(64, seed=44)
    t = nhwc(fr)
    f1, f2 = t[0::2], t[1::2]
    out = torch.full((2, 3, H, W, 64), float("nan"), device="cuda")
    la, lb = ops.pack_conv(wa, ba, L.PACK_PLAIN | L.PACK_F16X3), ops.pack_conv(wb, bb, L.PACK_PLAIN | L.PACK_F16X3)
    assert la.mode & L.PACK_F16X3 and lb.mode & L.PACK_F16X3
    ops.conv2d([dict(layer=la, in0=f1, in1=f2, out=out[0]), dict(layer=lb, in0=f2, in1=f1, out=out[1])], in1_mode=1)
    refa = O.conv2d(np.concatenate([fr[0::2], fr[1::2]], 1), wa, ba)
    refb = O.conv2d(np.concatenate([fr[1::2], fr[0::2]], 1), wb, bb)
    assert bool(torch.isfinite(out).all())   # every pixel written, none past the item
    assert relmax(to_nchw(out[0]), refa) < RTOL
    assert relmax(to_nchw(out[1]), refb) < RTOL


def test_conv1x1_f16x3_range_status(ops, L):
    """An activation past the split-fp16 range turns the 1x1 outputs non-finite and sets the status."""
    x0, x1 = rnd(1, 64, 8, 8, seed=45), rnd(1, 64, 8, 8, seed=46)
    x1[0, 3, 2, 2] = 1e6
    lay = ops.pack_conv(rnd(64, 128, 1, 1, seed=47, scale=0.1), rnd(64, seed=48), L.PACK_PLAIN | L.PACK_F16X3)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty(1, 8, 8, 64, device="cuda")
    ops.conv2d([dict(layer=lay, in0=nhwc(x0), in1=nhwc(x1), out=out)], in1_mode=1, status=st)
    assert int(st.item()) == 1


def test_offmask_conv(ops, L):
    x = rnd(2, 64, 10, 40, seed=20)
    w = rnd(216, 64, 3, 3, seed=21, scale=0.05)
    b = rnd(216, seed=22)
    out = torch.empty(2, 10, 40, 216, device="cuda")
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_OFFMASK), in0=nhwc(x), out=out)], epi=L.EPI_OFFMASK)
    ref = O.conv2d(x, w, b)
    got = out.cpu().numpy().reshape(2, 10, 40, 8, 9, 3)
    for g in range(8):
        for k in range(9):
            assert relmax(got[..., g, k, 0], ref[:, g * 18 + 2 * k]) < RTOL
            assert relmax(got[..., g, k, 1], ref[:, g * 18 + 2 * k + 1]) < RTOL
            assert relmax(got[..., g, k, 2], O.sigmoid(ref[:, 144 + g * 9 + k])) < RTOL


def test_lstm_cell_conv(ops, L, sd):
    x, h, c = rnd(2, 64, 6, 40, seed=23), rnd(2, 64, 6, 40, seed=24), rnd(2, 64, 6, 40, seed=25)
    p = "ConvBLSTM.forward_net.cell_list.0."
    hn, cn = O.conv_lstm_cell(x, h, c, sd, p, np.float64)
    layer = ops.pack_conv(sd[p + "conv.weight"], sd[p + "conv.bias"], L.PACK_LSTM)
    ho = torch.empty(2, 6, 40, 64, device="cuda")
    co = torch.empty(2, 6, 40, 64, device="cuda")
    ops.conv2d([dict(layer=layer, in0=nhwc(x), in1=nhwc(h), res=nhwc(c), out=ho, out2=co)], epi=L.EPI_LSTM,
               in1_mode=1)
    assert relmax(to_nchw(ho), hn) < RTOL
    assert relmax(to_nchw(co), cn) < RTOL


def test_conv_first(ops):
    x = np.random.default_rng(26).random((3, 3, 12, 20)).astype(np.float32)
    w = rnd(64, 3, 3, 3, seed=27, scale=0.2)
    b = rnd(64, seed=28)
    out = torch.empty(3, 12, 20, 64, device="cuda")
    ops.conv_first(torch.from_numpy(x).cuda(), torch.from_numpy(w).cuda(), torch.from_numpy(b).cuda(), out)
    assert relmax(to_nchw(out), O.lrelu(O.conv2d(x, w, b))) < RTOL


def _offsets(B, H, W, seed, scale=2.0):
    rng = np.random.default_rng(seed)
    off = (rng.standard_normal((B, 144, H, W)) * scale).astype(np.float32)
    off[:, 0, 0, 0] = -1.0        # exactly on the `> -1` gate
    off[:, 1, 2, 3] = -2.0
    off[:, 2, 1, 1] = float(H)    # exactly on the `< H` gate
    off[:, 5, 3, 2] = 0.5
    mask = rng.random((B, 72, H, W)).astype(np.float32)
    return off, mask


@pytest.mark.parametrize("epi", ["none", "lrelu"])
@pytest.mark.parametrize("hw", [(9, 11), (16, 40), (21, 70)])
@pytest.mark.parametrize("oscale", [0.7, 2.0, 7.0])   # 7.0: many samples leave the staged margin
@pytest.mark.parametrize("f16", [0, 1], ids=["f32", "f16x3"])
def test_dcn_fused(ops, L, epi, hw, oscale, f16):
    H, W = hw
    B = 2
    x = rnd(B, 64, H, W, seed=30)
    w = rnd(64, 64, 3, 3, seed=31, scale=0.05)
    b = rnd(64, seed=32)
    off, mask = _offsets(B, H, W, 33, oscale)
    ref = O.dcn_v2_forward(x, w, b, off, mask, 3, 3, 1, 1, 1, 1, 1, 1, 8)
    if epi == "lrelu":
        ref = O.lrelu(ref)
    om = np.zeros((B, H, W, 216), np.float32)
    o = off.reshape(B, 8, 9, 2, H, W).transpose(0, 4, 5, 1, 2, 3)
    m = mask.reshape(B, 8, 9, H, W).transpose(0, 3, 4, 1, 2)
    om = np.concatenate([o, m[..., None]], -1).reshape(B, H, W, 216)
    out = torch.empty(B, H, W, 64, device="cuda")
    lay = ops.pack_conv(w, b, L.PACK_PLAIN | (L.PACK_F16X3 if f16 else 0))
    ops.dcn([dict(layer=lay, inp=nhwc(x), offmask=torch.from_numpy(np.ascontiguousarray(om)).cuda(),
                  out=out)], epi=L.EPI_LRELU if epi == "lrelu" else L.EPI_NONE)
    assert relmax(to_nchw(out), ref) < RTOL


@pytest.mark.parametrize("oscale", [2.0, 7.0])
@pytest.mark.parametrize("G,N", [(8, 16), (8, 2), (1, 2)], ids=["two_rows", "one_row", "one_row_small"])
def test_dcn_fused_two_rows_per_wave(ops, L, oscale, G, N):
    """The f16x3 launch shapes of k_dcn, picked by grid size (stif_dcn_nhwc): >= 1024 two-row workgroups
    run k_dcn<., 1, 2> (two output rows per wave, 8-row tiles: 8 weight groups x 16 items of one 70x37
    map, 2 x 9 tiles each, rows past the map in the last tile); fewer run the one-row kernel (G = 8,
    N = 2: 576 workgroups of 4 rows; G = 1, N = 2: 72).  Every output against the oracle of item 0 --
    all G x N are the same computation."""
    H, W = 70, 37
    x = rnd(1, 64, H, W, seed=34)
    w = rnd(64, 64, 3, 3, seed=35, scale=0.05)
    b = rnd(64, seed=36)
    off, mask = _offsets(1, H, W, 37, oscale)
    ref = O.lrelu(O.dcn_v2_forward(x, w, b, off, mask, 3, 3, 1, 1, 1, 1, 1, 1, 8))
    o = off.reshape(1, 8, 9, 2, H, W).transpose(0, 4, 5, 1, 2, 3)
    m = mask.reshape(1, 8, 9, H, W).transpose(0, 3, 4, 1, 2)
    om = torch.from_numpy(np.ascontiguousarray(np.concatenate([o, m[..., None]], -1).reshape(1, H, W, 216))).cuda()
    xs, oms = nhwc(x).repeat(N, 1, 1, 1), om.repeat(N, 1, 1, 1)
    out = torch.full((G, N, H, W, 64), float("nan"), device="cuda")
    lay = ops.pack_conv(w, b, L.PACK_PLAIN | L.PACK_F16X3)
    ops.dcn([dict(layer=lay, inp=xs, offmask=oms, out=out[i]) for i in range(G)], epi=L.EPI_LRELU)
    assert relmax(to_nchw(out[0, :1]), ref) < RTOL
    assert bool((out == out[0, 0]).all())   # every group and item bit-identical to the checked one


@pytest.mark.parametrize("cfg", [
    dict(B=2, C=64, Co=64, H=9, W=11, k=3, s=1, p=1, d=1, g=8),
    dict(B=1, C=16, Co=24, H=10, W=7, k=3, s=2, p=1, d=1, g=2),
    dict(B=2, C=6, Co=5, H=8, W=9, k=3, s=1, p=2, d=2, g=3),
    dict(B=1, C=4, Co=70, H=6, W=6, k=1, s=1, p=0, d=1, g=1),
])
def test_dcn_v2_forward_dropin(ops, cfg):
    c = cfg
    K = c["k"] * c["k"]
    ho = (c["H"] + 2 * c["p"] - (c["d"] * (c["k"] - 1) + 1)) // c["s"] + 1
    wo = (c["W"] + 2 * c["p"] - (c["d"] * (c["k"] - 1) + 1)) // c["s"] + 1
    x = rnd(c["B"], c["C"], c["H"], c["W"], seed=40)
    w = rnd(c["Co"], c["C"], c["k"], c["k"], seed=41, scale=0.1)
    b = rnd(c["Co"], seed=42)
    rng = np.random.default_rng(43)
    off = (rng.standard_normal((c["B"], c["g"] * 2 * K, ho, wo)) * 1.5).astype(np.float32)
    mask = rng.random((c["B"], c["g"] * K, ho, wo)).astype(np.float32)
    ref = O.dcn_v2_forward(x, w, b, off, mask, c["k"], c["k"], c["s"], c["s"], c["p"], c["p"], c["d"], c["d"], c["g"])
    T = lambda a: torch.from_numpy(a).cuda()
    out = ops.dcn_v2_forward(T(x), T(w), T(b), T(off), T(mask), c["k"], c["k"], c["s"], c["s"], c["p"], c["p"],
                             c["d"], c["d"], c["g"])
    assert tuple(out.shape) == ref.shape
    assert relmax(out, ref) < RTOL


def test_dcn_zero_offset_kat_gpu(ops, golden):
    """The reference's own known-answer test (DCNv2/test.py:32-67) through the drop-in op."""
    x = golden["ops"]["kat_input"]
    N, C, H, W = x.shape
    w = np.zeros((C, C, 3, 3), np.float32)
    for p in range(C):
        w[p, p, 1, 1] = 1.0
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
    out = ops.dcn_v2_forward(T(x), T(w), T(np.zeros(C)), T(np.zeros((N, 18, H, W))), T(np.full((N, 9, H, W), 0.5)),
                             3, 3, 1, 1, 1, 1, 1, 1, 1)
    assert float((T(x) - 2 * out).abs().max()) < 1e-6


def test_entry_points_reject_items_over_2gb(L):
    """Items whose NHWC maps exceed the 32-bit buffer-descriptor range are refused before any launch
    (the pointers are never dereferenced)."""
    import ctypes as C
    lib = L.lib()
    H = W = 12000   # 144M px x 64 ch x 4 B > 2 GB
    a = L.ConvArgs()
    for f in ("in0", "in1", "w", "bias", "out", "res"):
        getattr(a, f)[0] = 0x1000
    a.ngroups = a.nitems = 1
    a.H, a.W, a.C0, a.Ho, a.Wo, a.cout, a.ks, a.stride = H, W, 64, H, W, 64, 3, 1
    for fn in (lib.stif_conv2d_nhwc, lib.stif_conv3x3_wino):
        assert fn(C.byref(a), None) == L.E_INVALID
        assert b"2 GB" in lib.stif_last_error()
    d = L.DcnArgs()
    for f in ("inp", "offmask", "w", "bias", "out"):
        getattr(d, f)[0] = 0x1000
    d.ngroups = d.nitems = 1
    d.H, d.W = H, W
    assert lib.stif_dcn_nhwc(C.byref(d), None) == L.E_INVALID
    assert b"2 GB" in lib.stif_last_error()


def test_dcn_dropin_rejects_bad_args(ops):
    x = torch.zeros(1, 4, 5, 5, device="cuda")
    with pytest.raises(RuntimeError, match="kernel channels"):
        ops.dcn_v2_forward(x, torch.zeros(2, 3, 3, 3, device="cuda"), torch.zeros(2, device="cuda"),
                           torch.zeros(1, 18, 5, 5, device="cuda"), torch.zeros(1, 9, 5, 5, device="cuda"),
                           3, 3, 1, 1, 1, 1, 1, 1, 1)


def test_ext_shim_dcn_sep_matches_reference(sd, golden):
    """integration/_ext.py (the `_ext` the reference's dcn_v2.py imports)
    driven the way DCN_sep.forward drives it (dcn_v2.py:127-140: conv_offset_mask, chunk, cat,
    sigmoid, _backend.dcn_v2_forward), against the reference's own DCN_sep output."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "_ext", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_ext.py"))
    ext = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ext)
    g = golden["ops"]
    p = "pcd_align.L2_dcnpack_1"
    inp, fea = g["dcnsep_in"], g["dcnsep_fea"]
    om = torch.from_numpy(O.conv2d(fea, sd[p + ".conv_offset_mask.weight"], sd[p + ".conv_offset_mask.bias"]).astype(
        np.float32)).cuda()
    o1, o2, m = torch.chunk(om, 3, dim=1)
    offset = torch.cat((o1, o2), dim=1).contiguous()
    mask = torch.sigmoid(m).contiguous()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
    out = ext.dcn_v2_forward(T(inp), T(sd[p + ".weight"]), T(sd[p + ".bias"]), offset, mask, 3, 3, 1, 1, 1, 1, 1, 1, 8)
    assert relmax(out, g["dcnsep_out"]) < 1e-4
    assert callable(ext.dcn_v2_backward)
    with pytest.raises(NotImplementedError):
        ext.dcn_v2_psroi_pooling_forward()


DCN_BWD_CASES = [
    # the reference's gradcheck configuration (DCNv2/test.py:15-19,69-103)
    dict(B=2, C=2, H=4, W=4, Co=2, k=3, s=1, p=1, d=1, dg=1, seed=1),
    # the STIF DCN_sep shape (64 -> 64, 8 groups) on a small map, far offsets and gate boundaries
    dict(B=2, C=64, H=13, W=21, Co=64, k=3, s=1, p=1, d=1, dg=8, seed=2),
    # stride 2 / dilation 2 / 1x1 / several groups / non-square kernels of the drop-in's shape classes
    dict(B=1, C=6, H=11, W=9, Co=5, k=3, s=2, p=2, d=2, dg=3, seed=3),
    dict(B=3, C=4, H=7, W=10, Co=3, k=1, s=1, p=0, d=1, dg=2, seed=4),
]


@pytest.mark.parametrize("case", DCN_BWD_CASES)
def test_dcn_v2_backward_dropin_matches_oracle(ops, case):
    """stif_dcn_v2_backward (drop-in for _ext.dcn_v2_backward) == the oracle's restatement of
    dcn_v2_cuda_backward, every gradient, relative to its max (fp32 GEMMs and fp32 atomics vs float64)."""
    B, C, H, W, Co, k, s, p, d, dg = (case[x] for x in ("B", "C", "H", "W", "Co", "k", "s", "p", "d", "dg"))
    rng = np.random.default_rng(case["seed"])
    Ho = (H + 2 * p - (d * (k - 1) + 1)) // s + 1
    Wo = (W + 2 * p - (d * (k - 1) + 1)) // s + 1
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    off = (rng.standard_normal((B, dg * 2 * k * k, Ho, Wo)) * 3).astype(np.float32)
    off[0, 0, 0, 0] = -1.0                                  # gate boundary: h_im exactly -1 (not sampled)
    msk = (1 / (1 + np.exp(-rng.standard_normal((B, dg * k * k, Ho, Wo))))).astype(np.float32)
    w = (rng.standard_normal((Co, C, k, k)) * 0.1).astype(np.float32)
    b = rng.standard_normal(Co).astype(np.float32)
    go = rng.standard_normal((B, Co, Ho, Wo)).astype(np.float32)
    dims = (k, k, s, s, p, p, d, d, dg)
    ref = O.dcn_v2_backward(x, w, b, off, msk, go, *dims)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    got = ops.dcn_v2_backward(T(x), T(w), T(b), T(off), T(msk), T(go), *dims)
    for name, g, r in zip(("input", "offset", "mask", "weight", "bias"), got, ref):
        assert tuple(g.shape) == r.shape, name
        assert relmax(g, r) < 2e-5, name


def test_dcn_v2_backward_through_reference_autograd_wiring(ops):
    """_DCNv2 (DCNv2/dcn_v2.py:15-45) wiring -- forward = _ext.dcn_v2_forward, backward =
    _ext.dcn_v2_backward -- in a torch.autograd.Function: the gradients reaching the inputs of
    dcn_v2_conv(input, offset, sigmoid(m), weight, bias) match the oracle (sigmoid chain rule by torch)."""
    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, inp, off, msk, wt, bs):
            ctx.save_for_backward(inp, off, msk, wt, bs)
            return ops.dcn_v2_forward(inp, wt, bs, off, msk, 3, 3, 1, 1, 1, 1, 1, 1, 2)

        @staticmethod
        def backward(ctx, gout):
            inp, off, msk, wt, bs = ctx.saved_tensors
            gi, goff, gm, gw, gb = ops.dcn_v2_backward(inp, wt, bs, off, msk, gout, 3, 3, 1, 1, 1, 1, 1, 1, 2)
            return gi, goff, gm, gw, gb

    rng = np.random.default_rng(9)
    x = torch.tensor(rng.standard_normal((2, 4, 6, 7)), dtype=torch.float32, device="cuda", requires_grad=True)
    off = torch.tensor(rng.standard_normal((2, 36, 6, 7)) * 2, dtype=torch.float32, device="cuda", requires_grad=True)
    m = torch.tensor(rng.standard_normal((2, 18, 6, 7)), dtype=torch.float32, device="cuda", requires_grad=True)
    wt = torch.tensor(rng.standard_normal((3, 4, 3, 3)) * 0.2, dtype=torch.float32, device="cuda", requires_grad=True)
    bs = torch.tensor(rng.standard_normal(3), dtype=torch.float32, device="cuda", requires_grad=True)
    go = torch.tensor(rng.standard_normal((2, 3, 6, 7)), dtype=torch.float32, device="cuda")
    F.apply(x, off, torch.sigmoid(m), wt, bs).backward(go)
    sig = 1 / (1 + np.exp(-m.detach().cpu().numpy().astype(np.float64)))
    gi, goff, gm, gw, gb = O.dcn_v2_backward(x.detach().cpu().numpy(), wt.detach().cpu().numpy(),
                                             bs.detach().cpu().numpy(), off.detach().cpu().numpy(), sig,
                                             go.cpu().numpy(), 3, 3, 1, 1, 1, 1, 1, 1, 2)
    for t, r in ((x, gi), (off, goff), (m, gm * sig * (1 - sig)), (wt, gw), (bs, gb)):
        assert relmax(t.grad, r) < 2e-5


@pytest.mark.parametrize("hw", [(33, 70), (64, 64)])
def test_dcn_v2_forward_dropin_stif_shape_fused(ops, hw):
    """The STIF shape (64 -> 64, 3x3, s1 p1 d1, 8 groups) through the drop-in runs the fused kernel
    (NCHW <-> NHWC transposes, device-side weight packing): gate boundaries and far offsets."""
    H, W = hw
    B = 2
    x = rnd(B, 64, H, W, seed=50)
    w = rnd(64, 64, 3, 3, seed=51, scale=0.05)
    b = rnd(64, seed=52)
    off, mask = _offsets(B, H, W, 53, 3.0)
    ref = O.dcn_v2_forward(x, w, b, off, mask, 3, 3, 1, 1, 1, 1, 1, 1, 8)
    T = lambda a: torch.from_numpy(a).cuda()
    out = ops.dcn_v2_forward(T(x), T(w), T(b), T(off), T(mask), 3, 3, 1, 1, 1, 1, 1, 1, 8)
    assert relmax(out, ref) < RTOL


def _dcnsep_weights(seed, oscale, boundary=False, H=0):
    """conv_offset_mask / DCN weights whose offsets have std ~ oscale px on N(0,1) features; with
    `boundary`, a few offset channels get zero weights and a bias that lands samples exactly on the
    `> -1` / `< H` gates (tap 0: dy = -1 -> h_im = oy - 2, exactly -1 at row 1; tap 4 of group 3: dx = -1.5;
    tap 8 of group 7: dy = H -> h_im >= H everywhere)."""
    w_om = rnd(216, 64, 3, 3, seed=seed, scale=oscale / 24.0)
    b_om = rnd(216, seed=seed + 1, scale=0.5)
    if boundary:
        for ch, v in ((0, -1.0), (3 * 18 + 2 * 4 + 1, -1.5), (7 * 18 + 2 * 8, float(H)), (144 + 5 * 9 + 2, 40.0)):
            w_om[ch] = 0.0
            b_om[ch] = v
    w = rnd(64, 64, 3, 3, seed=seed + 2, scale=0.05)
    b = rnd(64, seed=seed + 3)
    return {"x.conv_offset_mask.weight": w_om, "x.conv_offset_mask.bias": b_om, "x.weight": w, "x.bias": b}


def _dcnsep_layers(ops, L, sdx):
    om = ops.pack_conv(sdx["x.conv_offset_mask.weight"], sdx["x.conv_offset_mask.bias"], L.PACK_DCNSEP | L.PACK_F16X3,
                       range_fallback=False)
    core = ops.pack_conv(sdx["x.weight"], sdx["x.bias"], L.PACK_DCNPAIR | L.PACK_F16X3, range_fallback=False)
    return om, core


@pytest.mark.parametrize("epi", ["none", "lrelu"])
@pytest.mark.parametrize("hw", [(9, 11), (8, 32), (16, 40), (21, 70), (70, 37)])
@pytest.mark.parametrize("oscale", [0.7, 2.0, 7.0])   # 7.0: many samples leave the staged margin
def test_dcn_sep_fused_matches_oracle(ops, L, epi, hw, oscale):
    """k_dcn_sep (stif_dcn_sep_nhwc): conv_offset_mask + chunk/cat/sigmoid + the deformable conv in one
    launch == DCN_sep.forward (dcn_v2.py:127-140) restated by the oracle; partial tiles (9x11, 21x70,
    70x37), exact tiles (8x32), samples beyond the staged margin, two items."""
    H, W = hw
    B = 2
    sdx = _dcnsep_weights(40, oscale)
    x = rnd(B, 64, H, W, seed=41)
    fea = rnd(B, 64, H, W, seed=42)
    ref = O.dcn_sep(x, fea, sdx, "x")
    if epi == "lrelu":
        ref = O.lrelu(ref)
    om, core = _dcnsep_layers(ops, L, sdx)
    out = torch.full((B, H, W, 64), float("nan"), device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    ops.dcn_sep([dict(om_layer=om, layer=core, fea=nhwc(fea), inp=nhwc(x), out=out)],
                epi=L.EPI_LRELU if epi == "lrelu" else L.EPI_NONE, status=st)
    assert int(st.item()) == 0
    assert relmax(to_nchw(out), ref) < RTOL


def test_dcn_sep_fused_many_workgroups(ops, L):
    """k_dcn_sep with more workgroups than CUs (two resident per CU, several rounds, two weight sets):
    == the oracle, and three launches agree bit for bit."""
    H, W, B = 64, 128, 6
    sds = [_dcnsep_weights(90 + 10 * i, 2.0) for i in range(2)]
    xs = [rnd(B, 64, H, W, seed=91 + i) for i in range(2)]
    fs = [rnd(B, 64, H, W, seed=93 + i) for i in range(2)]
    groups, outs = [], []
    for i in range(2):
        om, core = _dcnsep_layers(ops, L, sds[i])
        outs.append(torch.full((B, H, W, 64), float("nan"), device="cuda"))
        groups.append(dict(om_layer=om, layer=core, fea=nhwc(fs[i]), inp=nhwc(xs[i]), out=outs[i]))
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    ops.dcn_sep(groups, epi=L.EPI_NONE, status=st)
    first = [o.clone() for o in outs]
    for _ in range(2):
        ops.dcn_sep(groups, epi=L.EPI_NONE, status=st)
        for o, f in zip(outs, first):
            assert torch.equal(o, f)
    assert int(st.item()) == 0
    for i in range(2):
        assert relmax(to_nchw(first[i]), O.dcn_sep(xs[i], fs[i], sds[i], "x")) < RTOL


@pytest.mark.parametrize("oscale", [2.0, 7.0])
def test_dcn_sep_fused_batch_independent(ops, L, oscale):
    """k_dcn_sep: an item's output does not depend on the other items of the launch (tile placement,
    workgroup scheduling, which lanes of a wave take the global fallback), bit for bit, and two launches
    of the same batch agree bit for bit."""
    H, W, B = 37, 100, 5
    sdx = _dcnsep_weights(80, oscale)
    x = torch.from_numpy(rnd(B, H, W, 64, seed=81)).cuda()
    fea = torch.from_numpy(rnd(B, H, W, 64, seed=82)).cuda()
    om, core = _dcnsep_layers(ops, L, sdx)

    def run(xs, fs):
        out = torch.full(xs.shape, float("nan"), device="cuda")
        ops.dcn_sep([dict(om_layer=om, layer=core, fea=fs, inp=xs, out=out)], epi=L.EPI_NONE)
        return out

    full = run(x, fea)
    assert torch.equal(full, run(x, fea))
    for i in (0, 3):
        assert torch.equal(full[i:i + 1], run(x[i:i + 1].clone(), fea[i:i + 1].clone())), i


def test_dcn_sep_fused_gates_and_groups(ops, L):
    """Offsets exactly on the sampling gates (bias-only offset channels), and a launch of 3 weight sets
    over strided items (a [3, n, H, W, 64] buffer's sub-tensors), each against its own oracle."""
    H, W = 19, 45
    B = 3
    xs = torch.from_numpy(np.ascontiguousarray(np.stack([rnd(B, H, W, 64, seed=50 + i) for i in range(3)]))).cuda()
    fs = torch.from_numpy(np.ascontiguousarray(np.stack([rnd(B, H, W, 64, seed=60 + i) for i in range(3)]))).cuda()
    out = torch.full((3, B, H, W, 64), float("nan"), device="cuda")
    sds = [_dcnsep_weights(70 + 10 * i, 2.0 + i, boundary=True, H=H) for i in range(3)]
    groups = []
    for i, sdx in enumerate(sds):
        om, core = _dcnsep_layers(ops, L, sdx)
        groups.append(dict(om_layer=om, layer=core, fea=fs[i], inp=xs[i], out=out[i]))
    ops.dcn_sep(groups, epi=L.EPI_NONE)
    for i, sdx in enumerate(sds):
        x = xs[i].cpu().numpy().transpose(0, 3, 1, 2)
        f = fs[i].cpu().numpy().transpose(0, 3, 1, 2)
        assert relmax(to_nchw(out[i]), O.dcn_sep(x, f, sdx, "x")) < RTOL, i


def test_dcn_sep_fused_equals_two_kernel_path(ops, L):
    """The fused kernel and the two-launch path it replaces (k_wino_om -> 216-channel map -> k_dcn, both
    f16x3) agree to the parity bar on the STIF shape."""
    H, W = 32, 48
    sdx = _dcnsep_weights(80, 3.0)
    x, fea = rnd(2, 64, H, W, seed=81), rnd(2, 64, H, W, seed=82)
    om, core = _dcnsep_layers(ops, L, sdx)
    a = torch.empty(2, H, W, 64, device="cuda")
    ops.dcn_sep([dict(om_layer=om, layer=core, fea=nhwc(fea), inp=nhwc(x), out=a)])
    omw = ops.pack_conv(sdx["x.conv_offset_mask.weight"], sdx["x.conv_offset_mask.bias"],
                        L.PACK_WINO_OFFMASK | L.PACK_F16X3)
    omap = torch.empty(2, H, W, 216, device="cuda")
    ops.conv2d([dict(layer=omw, in0=nhwc(fea), out=omap)], epi=L.EPI_OFFMASK)
    b = torch.empty(2, H, W, 64, device="cuda")
    core2 = ops.pack_conv(sdx["x.weight"], sdx["x.bias"], L.PACK_PLAIN | L.PACK_F16X3)
    ops.dcn([dict(layer=core2, inp=nhwc(x), offmask=omap, out=b)])
    ref = O.dcn_sep(x, fea, sdx, "x")
    assert relmax(to_nchw(a), ref) < RTOL and relmax(to_nchw(b), ref) < RTOL


@pytest.mark.parametrize("which", ["fea", "inp"])
def test_dcn_sep_fused_reports_range(ops, L, which):
    """k_dcn_sep's own range reporting (advisor finding, round 3): one offset-feature value (phase 1: the
    offset/mask sums go non-finite, the `chk` sum) or one DCN-input value (phase 2: the output goes
    non-finite, `chk2`) far outside the split-fp16 range sets the status word; the same call in range
    leaves it 0.  The phase-2 operand is the *sampled* value (bilinear weight x mask x pixel), so the
    poisoned input pixel is 1e6: any sample that touches it with weight x mask > 0.004 overflows (a
    5000 gives in-range samples below weight x mask 0.8 -- correctly not flagged)."""
    H, W, B = 20, 40, 2
    sdx = _dcnsep_weights(40, 2.0)
    x = rnd(B, 64, H, W, seed=41)
    fea = rnd(B, 64, H, W, seed=42)
    om, core = _dcnsep_layers(ops, L, sdx)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty(B, H, W, 64, device="cuda")
    xi, fi = nhwc(x), nhwc(fea)
    ops.dcn_sep([dict(om_layer=om, layer=core, fea=fi, inp=xi, out=out)], status=st)
    assert int(st.item()) == 0
    if which == "fea":
        fi = fi.clone()
        fi[1, 7, 13, 5] = 5000.0
    else:
        xi = xi.clone()
        xi[0, 11, 30, 60] = 1.0e6
    ops.dcn_sep([dict(om_layer=om, layer=core, fea=fi, inp=xi, out=out)], status=st)
    assert int(st.item()) == 1, which



@pytest.mark.parametrize("shape", [(3, 37, 53, 8), (5, 61, 29, 3), (1, 130, 97, 2), (4, 17, 250, 5)])
def test_dcn_sep_fused_launches_deterministic_odd_shapes(ops, L, shape):
    """Round-5 review item 4: launch groups of 2-8 weight sets with odd H / W (partial tiles in both directions,
    several workgroups per CU and so two per CU sharing it) and 1-5 items; every launch re-run three times into
    fresh NaN buffers reproduces its output bit for bit.  (The tap-pipelined diagnostic variant, DCNSEP_TAPPIPE=1,
    fails this whenever two workgroups share a CU -- DESIGN.md section 3d.)"""
    B, H, W, G = shape
    groups = []
    for i in range(G):
        sdx = _dcnsep_weights(200 + 7 * i, 1.0 + 0.7 * i)
        om, core = _dcnsep_layers(ops, L, sdx)
        groups.append(dict(om_layer=om, layer=core, fea=torch.from_numpy(rnd(B, H, W, 64, seed=300 + i)).cuda(),
                           inp=torch.from_numpy(rnd(B, H, W, 64, seed=400 + i)).cuda(),
                           out=torch.full((B, H, W, 64), float("nan"), device="cuda")))
    ops.dcn_sep(groups, epi=L.EPI_LRELU)
    ref = [g["out"].clone() for g in groups]
    assert all(bool(torch.isfinite(r).all()) for r in ref)
    for _ in range(3):
        g2 = [dict(g, out=torch.full_like(g["out"], float("nan"))) for g in groups]
        ops.dcn_sep(g2, epi=L.EPI_LRELU)
        assert all(torch.equal(a["out"], b) for a, b in zip(g2, ref))
