"""Winograd F(2x2,3x3) conv path (stif_conv3x3_wino) against the CPU oracle's direct conv."""
import numpy as np
import pytest
import torch

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5   # relative to max |ref|, same bar as the direct conv kernels (both operand modes)


@pytest.fixture(params=[0, 16], ids=["f32", "f16x3"])
def pf(request):
    """Winograd operand mode: fp32 MFMA, or fp32 products from 3 fp16 MFMAs on split operands
    (STIF_PACK_F16X3 packing; ops.conv2d sets STIF_CONV_F16X3 from it)."""
    return request.param


def relmax(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def nhwc(x):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x, np.float32).transpose(0, 2, 3, 1))).cuda()


def to_nchw(t):
    return t.detach().cpu().numpy().transpose(0, 3, 1, 2)


def rnd(*shape, seed=0, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


@pytest.mark.parametrize("epi", ["none", "lrelu", "relu", "res"])
@pytest.mark.parametrize("hw", [(13, 37), (8, 32), (33, 70), (4, 4)])
def test_wino_conv3x3(stif, epi, hw, pf):
    L, ops = stif._lib, stif.ops
    H, W = hw
    x = rnd(3, 64, H, W, seed=1)
    w = rnd(64, 64, 3, 3, seed=2, scale=0.05)
    b = rnd(64, seed=3)
    r = rnd(3, 64, H, W, seed=4)
    ref = O.conv2d(x, w, b)
    e = dict(none=L.EPI_NONE, lrelu=L.EPI_LRELU, relu=L.EPI_RELU, res=L.EPI_RES)[epi]
    ref = {"lrelu": O.lrelu, "relu": O.relu}.get(epi, lambda v: v)(ref)
    if epi == "res":
        ref = ref + r
    out = torch.empty(3, H, W, 64, device="cuda")
    layer = ops.pack_conv(w, b, L.PACK_WINO | pf)
    ops.conv2d([dict(layer=layer, in0=nhwc(x), out=out, res=nhwc(r) if epi == "res" else None)], epi=e)
    assert relmax(to_nchw(out), ref) < RTOL


def test_wino_residual_in_place(stif, pf):
    """out == res (the ResidualBlock_noBN in-place update the model uses)."""
    L, ops = stif._lib, stif.ops
    x = rnd(2, 64, 16, 64, seed=5)
    t = rnd(2, 64, 16, 64, seed=6)
    w = rnd(64, 64, 3, 3, seed=7, scale=0.05)
    b = rnd(64, seed=8)
    xd = nhwc(x)
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_WINO | pf), in0=nhwc(t), out=xd, res=xd)], epi=L.EPI_RES)
    assert relmax(to_nchw(xd), x + O.conv2d(t, w, b)) < RTOL


@pytest.mark.parametrize("cin1", [64, 32])
def test_wino_two_inputs_groups(stif, cin1, pf):
    """cat(in0, in1) input (PCD offset convs) in two weight groups over strided item views."""
    L, ops = stif._lib, stif.ops
    H, W = 12, 40
    fr = rnd(4, 64, H, W, seed=9)
    f1n = fr[0::2]
    f2n = fr[1::2, :cin1]
    wa, wb = rnd(64, 64 + cin1, 3, 3, seed=10, scale=0.04), rnd(64, 64 + cin1, 3, 3, seed=11, scale=0.04)
    ba, bb = rnd(64, seed=12), rnd(64, seed=13)
    t = nhwc(fr)
    in1 = t[1::2, :, :, :cin1].contiguous() if cin1 != 64 else t[1::2]
    out = torch.empty(2, 2, H, W, 64, device="cuda")
    ops.conv2d([dict(layer=ops.pack_conv(wa, ba, L.PACK_WINO | pf), in0=t[0::2], in1=in1, out=out[0]),
                dict(layer=ops.pack_conv(wb, bb, L.PACK_WINO | pf), in0=t[0::2], in1=in1, out=out[1])],
               epi=L.EPI_LRELU, in1_mode=1)
    cat = np.concatenate([f1n, f2n], 1)
    assert relmax(to_nchw(out[0]), O.lrelu(O.conv2d(cat, wa, ba))) < RTOL
    assert relmax(to_nchw(out[1]), O.lrelu(O.conv2d(cat, wb, bb))) < RTOL


def test_wino_multi_slice(stif, pf):
    L, ops = stif._lib, stif.ops
    x = rnd(1, 128, 10, 36, seed=14)
    w = rnd(128, 128, 3, 3, seed=15, scale=0.03)
    b = rnd(128, seed=16)
    out = torch.empty(1, 10, 36, 128, device="cuda")
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_WINO | pf), in0=nhwc(x), out=out)])
    assert relmax(to_nchw(out), O.conv2d(x, w, b)) < RTOL


def test_wino_matches_direct_kernel(stif, pf):
    """Winograd vs the direct implicit-GEMM kernel on the trunk shape: both fp32, both ~1e-7."""
    L, ops = stif._lib, stif.ops
    x = rnd(2, 64, 32, 64, seed=17)
    w = rnd(64, 64, 3, 3, seed=18, scale=0.05)
    b = rnd(64, seed=19)
    o1 = torch.empty(2, 32, 64, 64, device="cuda")
    o2 = torch.empty_like(o1)
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_WINO | pf), in0=nhwc(x), out=o1)], epi=L.EPI_RELU)
    ops.conv2d([dict(layer=ops.pack_conv(w, b), in0=nhwc(x), out=o2)], epi=L.EPI_RELU)
    ref = O.relu(O.conv2d(x, w, b))
    e1, e2 = relmax(to_nchw(o1), ref), relmax(to_nchw(o2), ref)
    assert e1 < RTOL and e2 < RTOL, (e1, e2)


def test_wino_rejects_bad_shapes(stif, pf):
    L, ops = stif._lib, stif.ops
    w = rnd(64, 64, 3, 3)
    lay = ops.pack_conv(w, rnd(64), L.PACK_WINO | pf)
    x = torch.zeros(1, 8, 8, 64, device="cuda")
    with pytest.raises(Exception):
        ops.conv2d([dict(layer=lay, in0=x, out=torch.empty(1, 4, 4, 64, device="cuda"))], stride=2)


@pytest.mark.parametrize("scale,h,w", [(1.0, 7, 9), (2.0, 7, 9), (2.0, 1, 5), (1.0, 4, 1), (2.0, 1, 1)])
def test_upsample2x(stif, scale, h, w):
    """stif_upsample2x_nhwc against the oracle's F.interpolate restatement, strided items (incl. 1-row /
    1-column / 1-pixel maps, where the 2x2-quad kernel's clamped neighbourhood slots matter)."""
    x = rnd(4, 64, h, w, seed=20)
    t = nhwc(x)
    out = torch.empty(2, 2 * h, 2 * w, 64, device="cuda")
    stif.ops.upsample2x(t[1::2], out, scale)
    ref = O.upsample2x(x[1::2].astype(np.float64)) * scale
    assert relmax(to_nchw(out), ref) < 1e-6


@pytest.mark.parametrize("n,h,w", [(2, 512, 512), (1, 513, 1025)])
def test_upsample2x_quad_kernel(stif, n, h, w):
    """Launches of >= 8M quad threads take the 2x2-quad kernel (k_up2q): checked against torch's
    F.interpolate(bilinear, x2, align_corners=False) on the GPU (fp32 reference of the same op;
    tolerance 2e-6 of max |ref|), incl. an odd-sized map for the clamped border neighbourhoods."""
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, h, w, 64, device="cuda", generator=g)
    out = torch.empty(n, 2 * h, 2 * w, 64, device="cuda")
    stif.ops.upsample2x(x, out, 2.0)
    ref = torch.nn.functional.interpolate(x.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                                          align_corners=False).permute(0, 2, 3, 1) * 2.0
    assert float((out - ref).abs().max()) <= 2e-6 * float(ref.abs().max())


def test_wino_cat_upsampled_matches_fused_direct(stif, pf):
    """cat(x, 2*up2(c)) conv: materialised upsample + Winograd == the direct kernel's fused path."""
    L, ops = stif._lib, stif.ops
    H, W = 12, 36
    x0 = rnd(2, 64, H, W, seed=21)
    c = rnd(2, 64, H // 2, W // 2, seed=22)
    w = rnd(64, 128, 3, 3, seed=23, scale=0.04)
    b = rnd(64, seed=24)
    up = torch.empty(2, H, W, 64, device="cuda")
    ops.upsample2x(nhwc(c), up, 2.0)
    o1 = torch.empty(2, H, W, 64, device="cuda")
    o2 = torch.empty_like(o1)
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_WINO | pf), in0=nhwc(x0), in1=up, out=o1)], epi=L.EPI_LRELU,
               in1_mode=1)
    ops.conv2d([dict(layer=ops.pack_conv(w, b), in0=nhwc(x0), in1=nhwc(c), out=o2)], epi=L.EPI_LRELU,
               in1_mode=2, in1_scale=2.0)
    ref = O.lrelu(O.conv2d(np.concatenate([x0, O.upsample2x(c.astype(np.float64)) * 2], 1), w, b))
    assert relmax(to_nchw(o1), ref) < RTOL and relmax(to_nchw(o2), ref) < RTOL


@pytest.mark.parametrize("epi", ["none", "lrelu"])
@pytest.mark.parametrize("hw", [(12, 36), (4, 4), (2, 66), (34, 70), (64, 64)])
def test_wino_fused_upsample(stif, epi, hw, pf):
    """cat(x, s * up2(c)) conv with the x2 upsample fused into the Winograd staging (in1_mode 2: coarse
    patch LDS-staged per tile and expanded between phases): two groups over strided coarse items,
    maps with partial tiles in both directions and 1-coarse-row/column borders, against the oracle."""
    L, ops = stif._lib, stif.ops
    H, W = hw
    x0 = rnd(4, 64, H, W, seed=60)
    c = rnd(4, 64, H // 2, W // 2, seed=61)
    wa, wb = rnd(64, 128, 3, 3, seed=62, scale=0.04), rnd(64, 128, 3, 3, seed=63, scale=0.04)
    ba, bb = rnd(64, seed=64), rnd(64, seed=65)
    e = L.EPI_LRELU if epi == "lrelu" else L.EPI_NONE
    act = O.lrelu if epi == "lrelu" else (lambda v: v)
    xt, ct = nhwc(x0), nhwc(c)
    out = torch.full((2, 2, H, W, 64), float("nan"), device="cuda")
    for scale in (2.0, 1.0):
        ops.conv2d([dict(layer=ops.pack_conv(wa, ba, L.PACK_WINO | pf), in0=xt[0::2], in1=ct[1::2], out=out[0]),
                    dict(layer=ops.pack_conv(wb, bb, L.PACK_WINO | pf), in0=xt[1::2], in1=ct[0::2], out=out[1])],
                   epi=e, in1_mode=2, in1_scale=scale)
        up = O.upsample2x(c.astype(np.float64)) * scale
        refa = act(O.conv2d(np.concatenate([x0[0::2], up[1::2]], 1), wa, ba))
        refb = act(O.conv2d(np.concatenate([x0[1::2], up[0::2]], 1), wb, bb))
        assert relmax(to_nchw(out[0]), refa) < RTOL and relmax(to_nchw(out[1]), refb) < RTOL


def test_wino_offmask_matches_direct(stif, pf):
    """64 -> 216 offset/mask conv (permuted [group][tap][dy,dx,sigmoid(m)] rows, 4 cout slices with
    the last one partial) on the Winograd kernel == the direct kernel, and == the oracle."""
    L, ops = stif._lib, stif.ops
    x = rnd(2, 64, 10, 40, seed=30)
    w = rnd(216, 64, 3, 3, seed=31, scale=0.05)
    b = rnd(216, seed=32)
    o1 = torch.empty(2, 10, 40, 216, device="cuda")
    o2 = torch.empty_like(o1)
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_WINO_OFFMASK | pf), in0=nhwc(x), out=o1)], epi=L.EPI_OFFMASK)
    ops.conv2d([dict(layer=ops.pack_conv(w, b, L.PACK_OFFMASK), in0=nhwc(x), out=o2)], epi=L.EPI_OFFMASK)
    a1, a2 = o1.cpu().numpy(), o2.cpu().numpy()
    assert np.abs(a1 - a2).max() < 1e-5 * np.abs(a2).max()
    ref = O.conv2d(x, w, b)                                      # [2,216,10,40] reference order
    got = a1.reshape(2, 10, 40, 8, 9, 3)
    off = ref[:, :144].reshape(2, 8, 9, 2, 10, 40).transpose(0, 4, 5, 1, 2, 3)
    msk = 1 / (1 + np.exp(-ref[:, 144:].reshape(2, 8, 9, 10, 40).transpose(0, 3, 4, 1, 2)))
    assert relmax(got[..., :2], off) < RTOL
    assert np.abs(got[..., 2] - msk).max() < 1e-5


@pytest.mark.parametrize("hw", [(6, 40), (13, 37), (32, 64)])
def test_wino_lstm_cell_conv(stif, sd, hw, pf):
    """ConvLSTMCell conv + gates (convlstm.py:42-58) on the Winograd path (STIF_PACK_WINO_LSTM),
    both BiConvLSTM directions as two launch groups, against the oracle cell."""
    L, ops = stif._lib, stif.ops
    H, W = hw
    p = "ConvBLSTM.forward_net.cell_list.0."
    layer = ops.pack_conv(sd[p + "conv.weight"], sd[p + "conv.bias"], L.PACK_WINO_LSTM | pf)
    groups, refs = [], []
    for d in range(2):
        x, h, c = (rnd(2, 64, H, W, seed=30 + 3 * d + k) for k in range(3))
        refs.append(O.conv_lstm_cell(x, h, c, sd, p, np.float64))
        groups.append(dict(layer=layer, in0=nhwc(x), in1=nhwc(h), res=nhwc(c),
                           out=torch.empty(2, H, W, 64, device="cuda"), out2=torch.empty(2, H, W, 64, device="cuda")))
    ops.conv2d(groups, epi=L.EPI_LSTM, in1_mode=1)
    for g, (hn, cn) in zip(groups, refs):
        assert relmax(to_nchw(g["out"]), hn) < RTOL
        assert relmax(to_nchw(g["out2"]), cn) < RTOL


@pytest.mark.parametrize("hw", [(10, 40), (4, 4), (33, 70), (128, 128)])
def test_wino_offmask_groups_items(stif, hw, pf):
    """Offset/mask conv launches as the model issues them (several weight sets x strided items;
    f16x3: the all-couts k_wino_om kernel, border tiles, more tiles than workgroups) == the direct
    fp32 kernel per group."""
    L, ops = stif._lib, stif.ops
    H, W = hw
    G, N = 2, 3
    xs = [rnd(N, 64, H, W, seed=40 + g) for g in range(G)]
    ws = [rnd(216, 64, 3, 3, seed=50 + g, scale=0.05) for g in range(G)]
    bs = [rnd(216, seed=60 + g) for g in range(G)]
    src = torch.empty(G, N + 1, H, W, 64, device="cuda")          # item stride of N + 1 pixels maps
    for g in range(G):
        src[g, :N] = nhwc(xs[g])
    out = torch.full((G, N, H, W, 216), float("nan"), device="cuda")
    ops.conv2d([dict(layer=ops.pack_conv(ws[g], bs[g], L.PACK_WINO_OFFMASK | pf), in0=src[g, :N], out=out[g])
                for g in range(G)], epi=L.EPI_OFFMASK)
    for g in range(G):
        ref = torch.empty(N, H, W, 216, device="cuda")
        ops.conv2d([dict(layer=ops.pack_conv(ws[g], bs[g], L.PACK_OFFMASK), in0=nhwc(xs[g]), out=ref)],
                   epi=L.EPI_OFFMASK)
        a1, a2 = out[g].cpu().numpy(), ref.cpu().numpy()
        assert np.isfinite(a1).all()
        assert np.abs(a1 - a2).max() <= 1e-5 * np.abs(a2).max()


@pytest.mark.parametrize("kind", ["plain", "offmask"])
@pytest.mark.parametrize("pos", [(0, 0, 0), (12, 69, 63), (5, 33, 17), (6, 1, 40)])
def test_wino_f16x3_range_status_single_element(stif, kind, pos):
    """One input element past the split range (|x| * 2^4 > 65504) anywhere in the map -- tile
    corners, tile row 0 / 1, any channel -- sets the status word (k_wino and k_wino_om), and an
    in-range map leaves it clear."""
    L, ops = stif._lib, stif.ops
    H, W = 13, 70
    x = rnd(2, 64, H, W, seed=7)
    cout, mode, epi = (64, L.PACK_WINO, L.EPI_RELU) if kind == "plain" else (216, L.PACK_WINO_OFFMASK, L.EPI_OFFMASK)
    layer = ops.pack_conv(rnd(cout, 64, 3, 3, seed=8, scale=0.05), rnd(cout, seed=9), mode | L.PACK_F16X3)
    for big, want in ((0.0, 0), (1e5, 1)):
        xx = x.copy()
        if big:
            y, xc, c = pos
            xx[1, c, y, xc] = big
        st = torch.zeros(1, dtype=torch.int32, device="cuda")
        out = torch.empty(2, H, W, cout, device="cuda")
        ops.conv2d([dict(layer=layer, in0=nhwc(xx), out=out)], epi=epi, status=st)
        assert int(st.item()) == want, (big, pos)



def test_wino_dynamic_schedule_bit_identical(stif):
    """Dynamic per-XCD tile scheduling (stif_conv_args.sched, ops.DYNAMIC_TILES) changes only which
    workgroup computes a tile: outputs bit-identical to the static schedule, for launches with one to many
    tiles per workgroup, back to back on one stream (each launch's counter bases come from the host's
    running totals) and interleaved on two streams with their own counters."""
    L, ops = stif._lib, stif.ops
    layer = ops.pack_conv(rnd(64, 64, 3, 3, seed=21, scale=0.05), rnd(64, seed=22), L.PACK_WINO | L.PACK_F16X3)
    shapes = [(18, 64, 64), (1, 8, 32), (5, 70, 33), (24, 128, 128)]    # 576 / 1 / 95 / 24,576 tiles
    xs = [torch.from_numpy(rnd(n, h, w, 64, seed=30 + i)).cuda() for i, (n, h, w) in enumerate(shapes)]

    def run_all(outs):
        for x, o in zip(xs, outs):
            ops.conv2d([dict(layer=layer, in0=x, out=o, res=x)], epi=L.EPI_RES)

    keep = ops.DYNAMIC_TILES
    try:
        ops.DYNAMIC_TILES = False
        ref = [torch.empty_like(x) for x in xs]
        run_all(ref)
        ops.DYNAMIC_TILES = True
        for _ in range(2):
            got = [torch.full_like(x, float("nan")) for x in xs]
            run_all(got)
            torch.cuda.synchronize()
            assert all(torch.equal(a, b) for a, b in zip(got, ref))
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        g1 = [torch.full_like(x, float("nan")) for x in xs]
        g2 = [torch.full_like(x, float("nan")) for x in xs]
        for s in (s1, s2):
            s.wait_stream(torch.cuda.current_stream())
        for k in range(len(xs)):
            for s, g in ((s1, g1), (s2, g2)):
                with torch.cuda.stream(s):
                    ops.conv2d([dict(layer=layer, in0=xs[k], out=g[k], res=xs[k])], epi=L.EPI_RES)
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(g1, ref))
        assert all(torch.equal(a, b) for a, b in zip(g2, ref))
        assert any(int(b.sum()) > 0 for b in ops._SCHED.values())   # the counters were used
        # a block passed without the STIF_CONV_DYNAMIC flag bit is never read or written (advisor r5: a caller
        # that leaves the trailing field uninitialised must not get the dynamic schedule)
        s3 = torch.cuda.Stream()
        s3.wait_stream(torch.cuda.current_stream())
        keep_flag = L.CONV_DYNAMIC
        L.CONV_DYNAMIC = 0
        try:
            with torch.cuda.stream(s3):
                g3 = [torch.full_like(x, float("nan")) for x in xs]
                run_all(g3)
        finally:
            L.CONV_DYNAMIC = keep_flag
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(g3, ref))
        assert int(ops._SCHED[(s3.device.index, s3.cuda_stream)].abs().sum()) == 0
    finally:
        ops.DYNAMIC_TILES = keep
