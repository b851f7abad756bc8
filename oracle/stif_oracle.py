"""CPU oracle: a numpy restatement of the STIF ``LunaTokis`` forward.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline -- never as a product code path.

Every function follows the reference file:line it cites (paths relative to the
reference's ``codes/``).  Feature arithmetic runs in ``dtype`` (float64 by
default, so the oracle is a "truth" that both the reference's fp32 CPU run and
the HIP path are measured against); every *discrete* decision the reference
takes from fp32 coordinates (``make_coord``, ``grid_sample`` nearest rounding,
``linspace``) is reproduced in float32 exactly as the reference computes it.

Parity status: pinned against ``tests/golden/*.npz``, which were produced by
running the reference model itself (``tests/golden/make_golden.py``).  The one
piece the reference cannot run here is the DCNv2 native op (it needs the removed
THC API); its restatement below is pinned by the reference's zero-offset
known-answer test (``DCNv2/test.py:32-67``) and by the reference ``DCN_sep``
module run on that restatement.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


# ----------------------------------------------------------------------------- basic ops
def conv2d(x, w, b, stride=1, pad=None, dtype=np.float64):
    """nn.Conv2d forward (NCHW).  x [N,C,H,W], w [Co,C,kh,kw].

    Computed as a sum over taps of contiguous row-slices of the zero-padded image
    flattened to [(H+2p)*(W+2p), C] (output evaluated on the padded-width grid, the
    2p junk columns dropped): one BLAS GEMM per tap and no im2col copy."""
    Co, C, kh, kw = w.shape
    if pad is None:
        pad = kh // 2
    N, _, H, W = x.shape
    Hp, Wp = H + 2 * pad, W + 2 * pad
    xp = np.zeros((N, Hp + 1, Wp, C), dtype)            # +1 row: the last tap's slice stays in bounds
    xp[:, pad:pad + H, pad:pad + W, :] = np.asarray(x, dtype).transpose(0, 2, 3, 1)
    flat = xp.reshape(N, (Hp + 1) * Wp, C)
    Hf = Hp - kh + 1                                      # stride-1 output rows
    wt = np.asarray(w, dtype).transpose(2, 3, 1, 0)      # [kh,kw,C,Co]
    out = np.zeros((N, Hf * Wp, Co), dtype)
    for n in range(N):
        for i in range(kh):
            for j in range(kw):
                off = i * Wp + j
                out[n] += np.dot(flat[n, off:off + Hf * Wp], wt[i, j])   # 2-D contiguous -> BLAS
    out = out.reshape(N, Hf, Wp, Co)[:, ::stride, :Wp - kw + 1:stride]
    out = out + np.asarray(b, dtype)
    return np.ascontiguousarray(out.transpose(0, 3, 1, 2))


def lrelu(x):
    """nn.LeakyReLU(negative_slope=0.1) (Sakuya_arch_test.py:69)."""
    return np.where(x >= 0, x, x * 0.1)


def relu(x):
    return np.maximum(x, 0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def _up2_index(n_in):
    """Source indices/weights of F.interpolate(scale_factor=2, bilinear, align_corners=False)."""
    d = np.arange(2 * n_in, dtype=np.float64)
    src = np.maximum(0.5 * (d + 0.5) - 0.5, 0.0)
    i0 = src.astype(np.int64)
    i1 = np.where(i0 < n_in - 1, i0 + 1, i0)
    l1 = src - i0
    return i0, i1, 1.0 - l1, l1


def upsample2x(x):
    """F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=False)
    as used by PCD_Align (Sakuya_arch_test.py:86,90,95,99,112,116,121,125)."""
    N, C, H, W = x.shape
    h0, h1, lh0, lh1 = _up2_index(H)
    w0, w1, lw0, lw1 = _up2_index(W)
    top = x[:, :, h0][:, :, :, w0] * lw0 + x[:, :, h0][:, :, :, w1] * lw1
    bot = x[:, :, h1][:, :, :, w0] * lw0 + x[:, :, h1][:, :, :, w1] * lw1
    return top * lh0[:, None] + bot * lh1[:, None]


# ----------------------------------------------------------------------------- DCNv2
def dcn_v2_forward(inp, weight, bias, offset, mask, kh, kw, sh, sw, ph, pw, dh, dw, dg,
                   dtype=np.float64):
    """Restatement of ``dcn_v2_cuda_forward`` (DCNv2/src/cuda/dcn_v2_cuda.cu:42-172):
    output = bias + W . columns, where columns come from
    ``modulated_deformable_im2col_gpu_kernel`` (dcn_v2_im2col_cuda.cu:125-195):
      h_im = h_out*stride - pad + i*dil + offset_h   (fp32 in the reference)
      sampled only if h_im > -1 && w_im > -1 && h_im < H && w_im < W,
      bilinear with per-corner zero padding (dmcn_im2col_bilinear, :25-54),
      times the modulation mask.
    Offset channel of (group g, tap k): g*2*K + 2k (+0 for h, +1 for w); mask: g*K + k.
    """
    inp = np.asarray(inp, dtype)
    B, C, H, W = inp.shape
    Co = weight.shape[0]
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    K = kh * kw
    cpg = C // dg
    P = Ho * Wo
    off = np.asarray(offset, F32).reshape(B, dg, K, 2, P)
    msk = np.asarray(mask, dtype).reshape(B, dg, K, P)
    h_in = np.repeat(np.arange(Ho) * sh - ph, Wo)[None, None]          # [1,1,P]
    w_in = np.tile(np.arange(Wo) * sw - pw, Ho)[None, None]
    img = np.ascontiguousarray(inp.transpose(0, 2, 3, 1)).reshape(B, H * W, dg, cpg)
    bi = np.arange(B)[:, None, None]
    gi = np.arange(dg)[None, :, None]
    cols = np.empty((B, P, K, dg, cpg), dtype)
    for i in range(kh):
        for j in range(kw):
            k = i * kw + j
            h_im = (h_in + i * dh).astype(F32) + off[:, :, k, 0]     # fp32 as the reference
            w_im = (w_in + j * dw).astype(F32) + off[:, :, k, 1]
            inside = (h_im > -1) & (w_im > -1) & (h_im < H) & (w_im < W)
            h_low = np.floor(h_im)
            w_low = np.floor(w_im)
            lh = (h_im - h_low).astype(dtype)
            lw = (w_im - w_low).astype(dtype)
            hh, hw = 1 - lh, 1 - lw
            h_low = h_low.astype(np.int64)
            w_low = w_low.astype(np.int64)
            h_high, w_high = h_low + 1, w_low + 1
            val = 0
            for hc, wc, ok, wt in ((h_low, w_low, (h_low >= 0) & (w_low >= 0), hh * hw),
                                   (h_low, w_high, (h_low >= 0) & (w_high <= W - 1), hh * lw),
                                   (h_high, w_low, (h_high <= H - 1) & (w_low >= 0), lh * hw),
                                   (h_high, w_high, (h_high <= H - 1) & (w_high <= W - 1), lh * lw)):
                idx = np.clip(hc, 0, H - 1) * W + np.clip(wc, 0, W - 1)   # [B,dg,P]
                v = img[bi, idx, gi]                                        # [B,dg,P,cpg]
                val = val + v * np.where(ok, wt, 0)[..., None]
            val = val * np.where(inside, msk[:, :, k], 0)[..., None]
            cols[:, :, k] = val.transpose(0, 2, 1, 3)
    wr = np.asarray(weight, dtype).transpose(2, 3, 1, 0).reshape(K * C, Co)  # [(tap, c), Co]
    out = np.empty((B, P, Co), dtype)
    for b in range(B):
        out[b] = cols[b].reshape(P, K * C) @ wr
    out = out + np.asarray(bias, dtype)
    return np.ascontiguousarray(out.transpose(0, 2, 1)).reshape(B, Co, Ho, Wo)


def _dcn_sample_geometry(B, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, offset, dg, k):
    """fp32 sampling coordinates of tap k (dcn_v2_im2col_cuda.cu:173-176, :216-235, :300-307):
    h_im / w_im [B, dg, P], with the floor corners, fractions and the (-1, H) x (-1, W) gate."""
    K = kh * kw
    P = Ho * Wo
    off = np.asarray(offset, F32).reshape(B, dg, K, 2, P)
    i, j = divmod(k, kw)
    h_in = np.repeat(np.arange(Ho) * sh - ph, Wo)[None, None]
    w_in = np.tile(np.arange(Wo) * sw - pw, Ho)[None, None]
    h_im = (h_in + i * dh).astype(F32) + off[:, :, k, 0]
    w_im = (w_in + j * dw).astype(F32) + off[:, :, k, 1]
    inside = (h_im > -1) & (w_im > -1) & (h_im < H) & (w_im < W)
    h_low = np.floor(h_im)
    w_low = np.floor(w_im)
    lh = (h_im - h_low).astype(np.float64)     # fp32 subtraction, exact in float64
    lw = (w_im - w_low).astype(np.float64)
    return inside, h_low.astype(np.int64), w_low.astype(np.int64), lh, lw


def dcn_v2_backward(inp, weight, bias, offset, mask, grad_out, kh, kw, sh, sw, ph, pw, dh, dw, dg,
                    dtype=np.float64):
    """Restatement of ``dcn_v2_cuda_backward`` (DCNv2/src/cuda/dcn_v2_cuda.cu:204-335), per sample:
      columns = W^T . grad_out                                       (:274-277, Sgemm n/t)
      grad_offset, grad_mask <- modulated_deformable_col2im_coord   (dcn_v2_im2col_cuda.cu:256-327):
        per (group, tap, pixel): sum over the group's channels of
          dmcn_get_coordinate_weight(h, w, im_c, dir) * col * mask   (:80-121; dir 0 = d/dh, 1 = d/dw)
          and, for the mask, col * dmcn_im2col_bilinear(im_c, h, w)   (:314-317)
        with (h, w) outside (-1, H) x (-1, W) contributing nothing (:308-313);
      grad_input <- modulated_deformable_col2im (:197-254): col * mask scattered to the in-bounds
        bilinear corners with dmcn_get_gradient_weight (:55-78);
      grad_weight += grad_out . columns_fwd^T (:308-315, columns_fwd = the forward im2col);
      grad_bias += sum over pixels of grad_out (:320-326).
    Returns (grad_input, grad_offset, grad_mask, grad_weight, grad_bias) in the reference's shapes
    (vision.cpp dcn_v2_backward order).  ``mask`` is the modulation after the sigmoid, as the
    reference's backend receives it."""
    inp = np.asarray(inp, dtype)
    B, C, H, W = inp.shape
    Co = weight.shape[0]
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    K = kh * kw
    cpg = C // dg
    P = Ho * Wo
    go = np.asarray(grad_out, dtype).reshape(B, Co, P)
    wm = np.asarray(weight, dtype).reshape(Co, C, K)
    msk = np.asarray(mask, dtype).reshape(B, dg, K, P)
    img = inp.reshape(B, dg, cpg, H * W)
    cols = np.einsum("ock,bop->bckp", wm, go).reshape(B, dg, cpg, K, P)     # columns per sample
    g_in = np.zeros((B, dg, cpg, H * W), dtype)
    g_off = np.zeros((B, dg, K, 2, P), dtype)
    g_msk = np.zeros((B, dg, K, P), dtype)
    bi = np.arange(B)[:, None, None, None]
    gi = np.arange(dg)[None, :, None, None]
    ci = np.arange(cpg)[None, None, :, None]
    for k in range(K):
        inside, h_low, w_low, lh, lw = _dcn_sample_geometry(B, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw,
                                                            offset, dg, k)
        hh, hw = 1 - lh, 1 - lw
        h_high, w_high = h_low + 1, w_low + 1
        corners = ((h_low, w_low, (h_low >= 0) & (w_low >= 0), hh * hw, -hw, -hh),
                   (h_low, w_high, (h_low >= 0) & (w_high <= W - 1), hh * lw, -lw, hh),
                   (h_high, w_low, (h_high <= H - 1) & (w_low >= 0), lh * hw, hw, -lh),
                   (h_high, w_high, (h_high <= H - 1) & (w_high <= W - 1), lh * lw, lw, lh))
        col = cols[:, :, :, k]                                  # [B, dg, cpg, P]
        m = np.where(inside, msk[:, :, k], 0)                   # [B, dg, P]
        gh = gw = bil = 0
        for hc, wc, ok, wt, dwh, dww in corners:
            ok = ok & inside
            idx = np.clip(hc, 0, H - 1) * W + np.clip(wc, 0, W - 1)                 # [B, dg, P]
            v = img[bi, gi, ci, idx[:, :, None, :]]                                   # [B, dg, cpg, P]
            v = np.where(ok[:, :, None], v, 0)
            bil = bil + v * wt[:, :, None]
            gh = gh + v * dwh[:, :, None]
            gw = gw + v * dww[:, :, None]
            # col2im: col * mask * bilinear weight into the in-bounds corner
            contrib = col * (np.where(ok, wt, 0) * m)[:, :, None]
            np.add.at(g_in, (bi, gi, ci, idx[:, :, None, :]), contrib)
        g_off[:, :, k, 0] = (gh * col).sum(2) * m
        g_off[:, :, k, 1] = (gw * col).sum(2) * m
        g_msk[:, :, k] = np.where(inside, (bil * col).sum(2), 0)
    cols_fwd = np.empty((B, dg, cpg, K, P), dtype)
    for k in range(K):
        inside, h_low, w_low, lh, lw = _dcn_sample_geometry(B, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw,
                                                            offset, dg, k)
        val = 0
        for hc, wc, ok, wt in ((h_low, w_low, (h_low >= 0) & (w_low >= 0), (1 - lh) * (1 - lw)),
                               (h_low, w_low + 1, (h_low >= 0) & (w_low + 1 <= W - 1), (1 - lh) * lw),
                               (h_low + 1, w_low, (h_low + 1 <= H - 1) & (w_low >= 0), lh * (1 - lw)),
                               (h_low + 1, w_low + 1, (h_low + 1 <= H - 1) & (w_low + 1 <= W - 1), lh * lw)):
            idx = np.clip(hc, 0, H - 1) * W + np.clip(wc, 0, W - 1)
            v = np.where(ok[:, :, None], img[bi, gi, ci, idx[:, :, None, :]], 0)
            val = val + v * wt[:, :, None]
        cols_fwd[:, :, :, k] = val * np.where(inside, msk[:, :, k], 0)[:, :, None]
    g_w = np.einsum("bop,bckp->ock", go, cols_fwd.reshape(B, C, K, P)).reshape(weight.shape)
    g_b = go.sum(axis=(0, 2))
    return (g_in.reshape(B, C, H, W), g_off.reshape(B, dg * K * 2, Ho, Wo), g_msk.reshape(B, dg * K, Ho, Wo),
            g_w, g_b)


def dcn_sep(inp, fea, sd, name, groups=8, dtype=np.float64):
    """DCN_sep.forward (DCNv2/dcn_v2.py:127-140): offsets/mask from a separate feature."""
    out = conv2d(fea, sd[name + ".conv_offset_mask.weight"], sd[name + ".conv_offset_mask.bias"], dtype=dtype)
    n = out.shape[1] // 3
    offset = out[:, :2 * n]                   # cat(o1, o2) == first two chunks
    mask = sigmoid(out[:, 2 * n:])
    w = sd[name + ".weight"]
    return dcn_v2_forward(inp, w, sd[name + ".bias"], offset, mask, 3, 3, 1, 1, 1, 1, 1, 1, groups, dtype)


# ----------------------------------------------------------------------------- encoder
def resblock(x, sd, name, dtype):
    """ResidualBlock_noBN (module_util.py:48-52): x + conv2(relu(conv1(x)))."""
    out = relu(conv2d(x, sd[name + ".conv1.weight"], sd[name + ".conv1.bias"], dtype=dtype))
    return x + conv2d(out, sd[name + ".conv2.weight"], sd[name + ".conv2.bias"], dtype=dtype)


def pcd_align(fea1, fea2, sd, p, dtype):
    """PCD_Align.forward (Sakuya_arch_test.py:71-130).  fea* = [L1, L2, L3]."""
    c = lambda n, t, **kw: conv2d(t, sd[p + n + ".weight"], sd[p + n + ".bias"], dtype=dtype, **kw)
    cat = lambda *t: np.concatenate(t, axis=1)
    y = []
    for d, (fa, fb) in ((1, (fea1, fea2)), (2, (fea2, fea1))):
        s = f"_{d}"
        L3_off = lrelu(c("L3_offset_conv1" + s, cat(fa[2], fb[2])))
        L3_off = lrelu(c("L3_offset_conv2" + s, L3_off))
        L3_fea = lrelu(dcn_sep(fa[2], L3_off, sd, p + "L3_dcnpack" + s, dtype=dtype))
        L2_off = lrelu(c("L2_offset_conv1" + s, cat(fa[1], fb[1])))
        L3_off = upsample2x(L3_off)
        L2_off = lrelu(c("L2_offset_conv2" + s, cat(L2_off, L3_off * 2)))
        L2_off = lrelu(c("L2_offset_conv3" + s, L2_off))
        L2_fea = dcn_sep(fa[1], L2_off, sd, p + "L2_dcnpack" + s, dtype=dtype)
        L3_fea = upsample2x(L3_fea)
        L2_fea = lrelu(c("L2_fea_conv" + s, cat(L2_fea, L3_fea)))
        L1_off = lrelu(c("L1_offset_conv1" + s, cat(fa[0], fb[0])))
        L2_off = upsample2x(L2_off)
        L1_off = lrelu(c("L1_offset_conv2" + s, cat(L1_off, L2_off * 2)))
        L1_off = lrelu(c("L1_offset_conv3" + s, L1_off))
        L1_fea = dcn_sep(fa[0], L1_off, sd, p + "L1_dcnpack" + s, dtype=dtype)
        L2_fea = upsample2x(L2_fea)
        L1_fea = c("L1_fea_conv" + s, cat(L1_fea, L2_fea))
        y.append(L1_fea)
    return np.concatenate(y, axis=1)


def pyramid(L1, sd, p, dtype):
    """fea_L2_conv1/2 + fea_L3_conv1/2 with lrelu (Sakuya_arch_test.py:321-325, :152-156)."""
    c = lambda n, t, s: lrelu(conv2d(t, sd[p + n + ".weight"], sd[p + n + ".bias"], stride=s, dtype=dtype))
    L2 = c("fea_L2_conv2", c("fea_L2_conv1", L1, 2), 1)
    L3 = c("fea_L3_conv2", c("fea_L3_conv1", L2, 2), 1)
    return L2, L3


def easy_pcd(f1, f2, sd, p, dtype):
    """Easy_PCD.forward (Sakuya_arch_test.py:144-166)."""
    B = f1.shape[0]
    L1 = np.concatenate([f1, f2], axis=0)          # stack on a batch axis; convs are per-image
    L2, L3 = pyramid(L1, sd, p, dtype)
    fea1 = [f1, L2[:B], L3[:B]]
    fea2 = [f2, L2[B:], L3[B:]]
    al = pcd_align(fea1, fea2, sd, p + "pcd_align.", dtype)
    return conv2d(al, sd[p + "fusion.weight"], sd[p + "fusion.bias"], dtype=dtype)


def conv_lstm_cell(x, h, c, sd, p, dtype):
    """ConvLSTMCell.forward (convlstm.py:42-58)."""
    cc = conv2d(np.concatenate([x, h], axis=1), sd[p + "conv.weight"], sd[p + "conv.bias"], dtype=dtype)
    nh = h.shape[1]
    i, f, o, g = (cc[:, k * nh:(k + 1) * nh] for k in range(4))
    c_next = sigmoid(f) * c + sigmoid(i) * np.tanh(g)
    h_next = sigmoid(o) * np.tanh(c_next)
    return h_next, c_next


def deformable_conv_lstm(xs, sd, p, dtype):
    """DeformableConvLSTM.forward (Sakuya_arch_test.py:192-242), one layer, zero initial state
    (convlstm.py:60-63).  xs: list over time of [B,64,H,W]."""
    h = np.zeros_like(xs[0])
    c = np.zeros_like(xs[0])
    outs = []
    for x in xs:
        ht = easy_pcd(x, h, sd, p + "pcd_h.", dtype)
        ct = easy_pcd(x, c, sd, p + "pcd_c.", dtype)
        h, c = conv_lstm_cell(x, ht, ct, sd, p + "cell_list.0.", dtype)
        outs.append(h)
    return outs


def bi_convlstm(xs, sd, dtype):
    """BiDeformableConvLSTM.forward (Sakuya_arch_test.py:256-266): same weights both directions."""
    p = "ConvBLSTM.forward_net."
    fwd = deformable_conv_lstm(xs, sd, p, dtype)
    rev = deformable_conv_lstm(xs[::-1], sd, p, dtype)[::-1]
    return [conv2d(np.concatenate([a, b], axis=1), sd["ConvBLSTM.conv_1x1.weight"],
                   sd["ConvBLSTM.conv_1x1.bias"], dtype=dtype) for a, b in zip(fwd, rev)]


def frame_features(frames, sd, front_RBs=5, dtype=np.float64):
    """Per-frame part of gen_feat (Sakuya_arch_test.py:318-325): [N,3,H,W] -> (L1, L2, L3)."""
    L1 = lrelu(conv2d(frames, sd["conv_first.weight"], sd["conv_first.bias"], dtype=dtype))
    for i in range(front_RBs):
        L1 = resblock(L1, sd, f"feature_extraction.{i}", dtype)
    L2, L3 = pyramid(L1, sd, "", dtype)
    return L1, L2, L3


def gen_feat_levels(fea1, fea2, sd, back_RBs=40, dtype=np.float64, capture=None):
    """gen_feat after the per-frame features (Sakuya_arch_test.py:337-362): pyramids of the first
    and second frame of each pair ([B,64,..] lists of 3 levels) -> latent [B,3,64,H,W]."""
    B, _, H, W = fea1[0].shape
    aligned = pcd_align(fea1, fea2, sd, "pcd_align.", dtype)
    fused = conv2d(aligned, sd["fusion.weight"], sd["fusion.bias"], dtype=dtype)
    if capture is not None:
        capture["pcd_align"] = aligned
        capture["fusion"] = fused
    xs = [fea1[0], fused, fea2[0]]
    feats = bi_convlstm(xs, sd, dtype)
    if capture is not None:
        capture["bilstm"] = np.stack(feats, axis=1)
    out = np.concatenate(feats, axis=0)            # [3B,...] ordered t-major
    for i in range(back_RBs):
        out = resblock(out, sd, f"recon_trunk.{i}", dtype)
    out = out.reshape(3, B, 64, H, W).transpose(1, 0, 2, 3, 4)
    return np.ascontiguousarray(out)


def gen_feat(x, sd, front_RBs=5, back_RBs=40, dtype=np.float64, capture=None):
    """LunaTokis.gen_feat (Sakuya_arch_test.py:313-362) for N=2 frames: x [B,2,3,H,W] -> [B,3,64,H,W]."""
    B, N, C, H, W = x.shape
    L1, L2, L3 = frame_features(np.asarray(x, dtype).reshape(B * N, C, H, W), sd, front_RBs, dtype)
    lv = [t.reshape(B, N, *t.shape[1:]) for t in (L1, L2, L3)]
    return gen_feat_levels([t[:, 0] for t in lv], [t[:, 1] for t in lv], sd, back_RBs, dtype, capture)


# ----------------------------------------------------------------------------- decoder
def make_coord_1d(n):
    """One axis of make_coord (Sakuya_arch_test.py:1233-1248) in the reference's fp32:
    seq = fp32(-1 + r) + fp32(2r) * arange(n).float(), r = 1/n."""
    r = 2.0 / (2 * n)
    return (F32(2 * r) * np.arange(n, dtype=F32)).astype(F32) + F32(-1 + r)


def linspace_f32(n):
    """torch.linspace(-1, 1, n) on CPU in fp32 (warplayer.py:27-30)."""
    if n == 1:
        return np.array([-1.0], F32)
    step = F32((1.0 - -1.0) / (n - 1))
    i = np.arange(n)
    lo = (F32(-1.0) + step * i.astype(F32)).astype(F32)
    hi = (F32(1.0) - step * (n - 1 - i).astype(F32)).astype(F32)
    return np.where(i < n // 2, lo, hi).astype(F32)



def nearest_index(coord, n):
    """grid_sample(mode='nearest', align_corners=False) source index: round-half-even in fp32."""
    coord = np.asarray(coord, F32)
    src = ((coord + F32(1)) * F32(n) - F32(1)) / F32(2)
    return np.rint(src).astype(np.int64)


def bilinear_sample(img, gx, gy, dtype=np.float64):
    """F.grid_sample(img, grid, 'bilinear', padding_mode='zeros', align_corners=False).
    img [B,C,H,W], gx/gy [B,Q] normalised (x along W, y along H) -> [B,Q,C]."""
    B, C, H, W = img.shape
    ix = ((np.asarray(gx, dtype) + 1) * W - 1) / 2
    iy = ((np.asarray(gy, dtype) + 1) * H - 1) / 2
    x0 = np.floor(ix)
    y0 = np.floor(iy)
    x1, y1 = x0 + 1, y0 + 1
    wnw = (x1 - ix) * (y1 - iy)
    wne = (ix - x0) * (y1 - iy)
    wsw = (x1 - ix) * (iy - y0)
    wse = (ix - x0) * (iy - y0)
    flat = np.asarray(img, dtype).reshape(B, C, H * W).transpose(0, 2, 1)   # [B,HW,C]
    b = np.arange(B)[:, None]
    out = 0
    for xx, yy, ww in ((x0, y0, wnw), (x1, y0, wne), (x0, y1, wsw), (x1, y1, wse)):
        xi = xx.astype(np.int64)
        yi = yy.astype(np.int64)
        ok = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
        v = flat[b, np.clip(yi, 0, H - 1) * W + np.clip(xi, 0, W - 1)]
        out = out + np.where(ok[..., None], v, 0) * ww[..., None]
    return out


def siren(x, sd, p, n_sine, dtype):
    """Siren.forward (SIREN.py:74-79): n_sine x sin(30*(xW^T+b)) then a final Linear."""
    for i in range(n_sine):
        x = np.sin(30.0 * (x @ np.asarray(sd[f"{p}net.{i}.linear.weight"], dtype).T
                           + np.asarray(sd[f"{p}net.{i}.linear.bias"], dtype)))
    return x @ np.asarray(sd[f"{p}net.{n_sine}.weight"], dtype).T + np.asarray(sd[f"{p}net.{n_sine}.bias"], dtype)


def upsample_bilinear(x, s, dtype=np.float64):
    """F.upsample(x, scale_factor=s, mode='bilinear') (align_corners=False; source index
    (d + 0.5) / s - 0.5 clamped at 0, ATen upsample_bilinear2d) as decoding_test builds HRinp
    (Sakuya_arch_test.py:513-514).  x [N,C,H,W] -> [N,C,sH,sW]."""
    x = np.asarray(x, dtype)
    N, C, H, W = x.shape

    def idx(n):
        src = np.maximum((np.arange(s * n, dtype=F32) + F32(0.5)) * F32(1.0 / s) - F32(0.5), F32(0))
        i0 = src.astype(np.int64)
        i1 = np.where(i0 < n - 1, i0 + 1, i0)
        l1 = (src - i0).astype(dtype)
        return i0, i1, 1 - l1, l1

    h0, h1, lh0, lh1 = idx(H)
    w0, w1, lw0, lw1 = idx(W)
    top = x[:, :, h0][:, :, :, w0] * lw0 + x[:, :, h0][:, :, :, w1] * lw1
    bot = x[:, :, h1][:, :, :, w0] * lw0 + x[:, :, h1][:, :, :, w1] * lw1
    return top * lh0[:, None] + bot * lh1[:, None]


def _decode(feat, inp, times, sd, HH, WW, dtype, capture=None, img=None, shift=None):
    """The decoder body shared by decoding / decoding_test / decoding_fasttest /
    decoding_localensemble (Sakuya_arch_test.py:364-459, 461-598, 863-1085).
    img: the image the flow / encode stages sample bilinearly (LR inp, or decoding_test's x4
    upsampled HRinp).  shift: (vx, vy) of the local ensemble -- the query coordinates move by
    (vx/H + 1e-6, vy/W + 1e-6) for every sampling step except rel_coord and the warpgrid base.
    Returns (list of [B,3,HH,WW], area [HH*WW] or None)."""
    B = feat.shape[0]
    H, W = feat.shape[-2:]
    featc = np.asarray(feat, dtype).reshape(B, 192, H, W)          # cat(feat[:,0..2]) (:365)
    inpc = np.asarray(inp, dtype).reshape(B, 6, H, W)
    img = inpc if img is None else np.asarray(img, dtype)
    lo, hi = F32(-1 + 1e-6), F32(1 - 1e-6)
    cy = np.clip(make_coord_1d(HH), lo, hi)                          # coord_highres (:373), row/col
    cx = np.clip(make_coord_1d(WW), lo, hi)
    sy, sx = cy, cx
    if shift is not None:                                            # :994-998 (fp32 tensor ops)
        sy = np.clip((cy + F32(shift[0] * (2 / H / 2) + 1e-6)).astype(F32), lo, hi)
        sx = np.clip((cx + F32(shift[1] * (2 / W / 2) + 1e-6)).astype(F32), lo, hi)
    ly, lx = make_coord_1d(H), make_coord_1d(W)                      # feat_coord (:375)
    iy = np.clip(nearest_index(sy, H), 0, H - 1)
    ix = np.clip(nearest_index(sx, W), 0, W - 1)
    rel_y = ((cy - ly[iy]) * F32(H)).astype(F32)                     # (:394-396)
    rel_x = ((cx - lx[ix]) * F32(W)).astype(F32)
    Q = HH * WW
    qy = np.repeat(np.arange(HH), WW)
    qx = np.tile(np.arange(WW), HH)
    gy = np.broadcast_to(sy[qy], (B, Q))
    gx = np.broadcast_to(sx[qx], (B, Q))
    lin = featc.reshape(B, 192, H * W).transpose(0, 2, 1)
    q_feat = lin[:, iy[qy] * W + ix[qx]]                              # nearest (:382-385)
    q_inp = inpc.reshape(B, 6, H * W).transpose(0, 2, 1)[:, iy[qy] * W + ix[qx]]
    rel = np.stack([np.broadcast_to(rel_y[qy], (B, Q)), np.broadcast_to(rel_x[qx], (B, Q))], -1).astype(dtype)
    area = None
    if shift is not None:                                            # :1003
        area = np.abs((rel_y[qy] * rel_x[qx]).astype(F32)).astype(dtype) + 1e-9
    # nearest HR pixel of the (shifted) query: identity without a shift (:406-409)
    hy = np.clip(nearest_index(sy, HH), 0, HH - 1)
    hx = np.clip(nearest_index(sx, WW), 0, WW - 1)
    gxs, gys = linspace_f32(WW), linspace_f32(HH)                     # warpgrid base (warplayer.py:27-31)
    preds = []
    for t in times:
        pe = np.full((B, Q, 1), t, dtype)
        x1 = np.concatenate([q_feat, q_inp, rel, pe], -1)             # 201 (:399)
        hrfeat = siren(x1, sd, "feat_imnet.", 3, dtype)               # [B,Q,64] (:400)
        hr_img = hrfeat.transpose(0, 2, 1).reshape(B, 64, HH, WW)
        q_hr = hrfeat[:, hy[qy] * WW + hx[qx]]
        q_inp2 = bilinear_sample(img, gx, gy, dtype)                  # (:410-413)
        q_feat0 = bilinear_sample(featc, gx, gy, dtype)               # (:414-417)
        flow = siren(np.concatenate([q_hr, q_feat0, q_inp2, pe], -1), sd, "flow_imnet.", 3, dtype)  # 263
        if capture is not None:
            capture.setdefault("hrfeat", []).append(hrfeat)
            capture.setdefault("flow", []).append(flow)
        fx = flow[..., [0, 2]]
        fy = flow[..., [1, 3]]
        # warpgrid (warplayer.py:25-39): base linspace grid + flow / ((n-1)/2); then clamp (:428,441)
        bx = gxs[qx].astype(dtype)[None]
        by = gys[qy].astype(dtype)[None]
        feats = []
        imgs = []
        for k in range(2):
            g_x = np.clip(bx + fx[..., k] / ((WW - 1.0) / 2.0), lo, hi)
            g_y = np.clip(by + fy[..., k] / ((HH - 1.0) / 2.0), lo, hi)
            feats.append((bilinear_sample(hr_img, g_x, g_y, dtype), bilinear_sample(featc, g_x, g_y, dtype)))
            imgs.append(bilinear_sample(img, g_x, g_y, dtype))
        x3 = np.concatenate([feats[0][0], feats[1][0], feats[0][1], feats[1][1], imgs[0], imgs[1], pe], -1)  # 525
        pred = siren(x3, sd, "encode_imnet.", 4, dtype)                # (:456)
        preds.append(pred.transpose(0, 2, 1).reshape(B, 3, HH, WW))
    return preds, area


def _bilinear_pts(get, H, W, gx, gy, dtype=np.float64):
    """bilinear_sample at n points: F.grid_sample(bilinear, zeros, align_corners=False) with the
    image read through ``get(yi, xi) -> [n, C]`` (fp32 source values) -> [n, C] in dtype."""
    ix = ((np.asarray(gx, dtype) + 1) * W - 1) / 2
    iy = ((np.asarray(gy, dtype) + 1) * H - 1) / 2
    x0 = np.floor(ix)
    y0 = np.floor(iy)
    x1, y1 = x0 + 1, y0 + 1
    out = 0
    for xx, yy, ww in ((x0, y0, (x1 - ix) * (y1 - iy)), (x1, y0, (ix - x0) * (y1 - iy)),
                       (x0, y1, (x1 - ix) * (iy - y0)), (x1, y1, (ix - x0) * (iy - y0))):
        xi = xx.astype(np.int64)
        yi = yy.astype(np.int64)
        ok = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
        v = np.asarray(get(np.clip(yi, 0, H - 1), np.clip(xi, 0, W - 1)), dtype)
        out = out + np.where(ok[:, None], v, 0) * ww[:, None]
    return out


def decoding_at(feat, inp, times, sd, HH, WW, py, px, dtype=np.float64, stats=None):
    """LunaTokis.decoding (Sakuya_arch_test.py:364-459) evaluated only at the HR pixels
    (py[i], px[i]) -> list over times of [B, 3, n].  Same arithmetic as ``_decode``: every HR pixel's
    stage 1 (feat_imnet -> HRfeat, flow_imnet -> flow, :380-422) depends only on that pixel's
    coordinates, so the HRfeat the warped bilinear gathers of stage 2 read (:424-457) is evaluated at
    just the corner pixels they touch.  ``feat`` [B,3,64,H,W] may be any strided view (it is read by
    gathers only, never copied whole: full-size latents from the GPU engine); ``stats`` (a dict)
    receives the number of warped samples whose grid was clamped at the frame edge (:428,441)."""
    B = feat.shape[0]
    H, W = feat.shape[-2:]
    py = np.asarray(py, np.int64)
    px = np.asarray(px, np.int64)
    lo, hi = F32(-1 + 1e-6), F32(1 - 1e-6)
    cy = np.clip(make_coord_1d(HH), lo, hi)
    cx = np.clip(make_coord_1d(WW), lo, hi)
    ly, lx = make_coord_1d(H), make_coord_1d(W)
    iy = np.clip(nearest_index(cy, H), 0, H - 1)
    ix = np.clip(nearest_index(cx, W), 0, W - 1)
    rel_y = ((cy - ly[iy]) * F32(H)).astype(F32)
    rel_x = ((cx - lx[ix]) * F32(W)).astype(F32)
    assert (np.clip(nearest_index(cy, HH), 0, HH - 1) == np.arange(HH)).all()   # q_feat = HRfeat (:406-409)
    assert (np.clip(nearest_index(cx, WW), 0, WW - 1) == np.arange(WW)).all()
    gxs, gys = linspace_f32(WW), linspace_f32(HH)
    preds = [np.empty((B, 3, len(py)), dtype) for _ in times]
    clamped = 0
    for b in range(B):
        lat = lambda yy, xx: np.asarray(feat[b, :, :, yy, xx], F32).reshape(len(yy), 192)   # cat(feat[:,0..2])
        img = lambda yy, xx: np.asarray(inp[b, :, :, yy, xx], F32).reshape(len(yy), 6)

        def stage1_in(qy, qx, t):
            """the 201 inputs of feat_imnet at HR pixels (qy, qx) (:382-399)"""
            return np.concatenate([np.asarray(lat(iy[qy], ix[qx]), dtype), np.asarray(img(iy[qy], ix[qx]), dtype),
                                   np.stack([rel_y[qy], rel_x[qx]], -1).astype(dtype),
                                   np.full((len(qy), 1), t, dtype)], -1)

        for ti, t in enumerate(times):
            hrf = siren(stage1_in(py, px, t), sd, "feat_imnet.", 3, dtype)                      # (:400)
            gx, gy = cx[px], cy[py]
            q_inp2 = _bilinear_pts(img, H, W, gx, gy, dtype)                                    # (:410-413)
            q_feat0 = _bilinear_pts(lat, H, W, gx, gy, dtype)                                   # (:414-417)
            pe = np.full((len(py), 1), t, dtype)
            flow = siren(np.concatenate([hrf, q_feat0, q_inp2, pe], -1), sd, "flow_imnet.", 3, dtype)
            bx, by = gxs[px].astype(dtype), gys[py].astype(dtype)
            grids = []
            for k in range(2):                                                                  # warpgrid + clamp
                ux = bx + flow[:, 2 * k] / ((WW - 1.0) / 2.0)
                uy = by + flow[:, 2 * k + 1] / ((HH - 1.0) / 2.0)
                clamped += int(((ux < lo) | (ux > hi) | (uy < lo) | (uy > hi)).sum())
                grids.append((np.clip(ux, lo, hi), np.clip(uy, lo, hi)))
            # HRfeat at every corner pixel the two warped gathers touch
            cyx = []
            for g_x, g_y in grids:
                fx = np.floor(((g_x + 1) * WW - 1) / 2).astype(np.int64)
                fy = np.floor(((g_y + 1) * HH - 1) / 2).astype(np.int64)
                for dy in (0, 1):
                    for dx in (0, 1):
                        cyx.append(np.clip(fy + dy, 0, HH - 1) * WW + np.clip(fx + dx, 0, WW - 1))
            uniq = np.unique(np.concatenate(cyx))
            hrc = siren(stage1_in(uniq // WW, uniq % WW, t), sd, "feat_imnet.", 3, dtype)
            hr_get = lambda yy, xx: hrc[np.searchsorted(uniq, yy * WW + xx)]
            feats, imgs = [], []
            for g_x, g_y in grids:
                feats.append((_bilinear_pts(hr_get, HH, WW, g_x, g_y, dtype), _bilinear_pts(lat, H, W, g_x, g_y, dtype)))
                imgs.append(_bilinear_pts(img, H, W, g_x, g_y, dtype))
            x3 = np.concatenate([feats[0][0], feats[1][0], feats[0][1], feats[1][1], imgs[0], imgs[1], pe], -1)
            preds[ti][b] = siren(x3, sd, "encode_imnet.", 4, dtype).T                              # (:456)
    if stats is not None:
        stats["clamped"] = clamped
    return preds


def decoding(feat, inp, times, sd, scale=None, dtype=np.float64, capture=None):
    """LunaTokis.decoding (Sakuya_arch_test.py:364-459).
    feat [B,3,64,H,W], inp [B,2,3,H,W], times: list of floats -> list of [B,3,HH,WW]."""
    H, W = feat.shape[-2:]
    HH, WW = (H * 4, W * 4) if scale is None else (int(scale[0]), int(scale[1]))
    return _decode(feat, inp, times, sd, HH, WW, dtype, capture)[0]


def decoding_test(feat, inp, times, sd, scale=None, dtype=np.float64):
    """LunaTokis.decoding_test (Sakuya_arch_test.py:461-598): decoding with the flow and encode
    stages sampling HRinp = F.upsample(inp, x4, bilinear) instead of the LR frames; HH = H*scale
    (scale an integer, default 4).  The q/3 chunking only bounds memory."""
    H, W = feat.shape[-2:]
    s = 4 if scale is None else int(scale)
    B = feat.shape[0]
    hr = upsample_bilinear(np.asarray(inp, dtype).reshape(B, 6, H, W), 4, dtype)
    return _decode(feat, inp, times, sd, H * s, W * s, dtype, img=hr)[0]


def decoding_fasttest(feat, inp, times, sd, scale=None, dtype=np.float64):
    """LunaTokis.decoding_fasttest (Sakuya_arch_test.py:863-960): every time of `times` (floats)
    as one batch of a batch-1 latent -> [len(times), 3, HH, WW]."""
    return np.concatenate(decoding(feat, inp, times, sd, scale, dtype), 0)


def decoding_localensemble(feat, inp, times, sd, scale=None, dtype=np.float64):
    """LunaTokis.decoding_localensemble (Sakuya_arch_test.py:962-1085): four decodes with the
    query shifted by (+-1/H, +-1/W) (+1e-6), blended by the diagonally opposite |rel_y rel_x|
    area over the total (batch-1 latent, times as the batch) -> [len(times), 3, HH, WW]."""
    H, W = feat.shape[-2:]
    HH, WW = (H * 4, W * 4) if scale is None else (int(scale[0]), int(scale[1]))
    preds, areas = [], []
    for vx in (-1, 1):
        for vy in (-1, 1):
            p, a = _decode(feat, inp, times, sd, HH, WW, dtype, shift=(vx, vy))
            preds.append(np.concatenate(p, 0))
            areas.append(a)
    tot = areas[0] + areas[1] + areas[2] + areas[3]
    areas = [areas[3], areas[2], areas[1], areas[0]]                   # :1079-1080
    ret = 0
    for p, a in zip(preds, areas):
        ret = ret + p * (a / tot).reshape(1, 1, HH, WW)
    return ret


def forward(x, times, sd, scale=None, front_RBs=5, back_RBs=40, dtype=np.float64, capture=None):
    """LunaTokis.forward(x, times, scale, test=False) (Sakuya_arch_test.py:1222-1231)."""
    feat = gen_feat(x, sd, front_RBs, back_RBs, dtype, capture)
    if capture is not None:
        capture["feat"] = feat
    return decoding(feat, x, times, sd, scale, dtype, capture)


# ----------------------------------------------------------------------------- harness I/O
def _cubic(x):
    """data/util.py:240-246 (fp32)."""
    ax = np.abs(x).astype(F32)
    ax2 = (ax * ax).astype(F32)
    ax3 = (ax2 * ax).astype(F32)
    a = ((F32(1.5) * ax3 - F32(2.5) * ax2 + F32(1)) * (ax <= 1)).astype(F32)
    b = ((F32(-0.5) * ax3 + F32(2.5) * ax2 - F32(4) * ax + F32(2)) * ((ax > 1) & (ax <= 2))).astype(F32)
    return (a + b).astype(F32)


def resize_weights_indices(in_len, out_len, scale, antialias=True):
    """calculate_weights_indices (data/util.py:248-300) in fp32: MATLAB-style cubic weights
    (widened by 1/scale when downscaling with antialiasing), rows normalised, all-zero edge
    columns dropped.  Returns (weights [out, P], first index into the symmetric-padded input
    [out], sym_len_s, sym_len_e)."""
    kw = 4.0 / scale if (scale < 1 and antialias) else 4.0
    x = np.linspace(1, out_len, out_len, dtype=np.float64).astype(F32)
    u = (x / F32(scale) + F32(0.5 * (1 - 1 / scale))).astype(F32)
    left = np.floor(u - F32(kw / 2)).astype(F32)
    P = int(np.ceil(kw)) + 2
    ind = (left[:, None] + np.arange(P, dtype=F32)[None, :]).astype(F32)
    dist = (u[:, None] - ind).astype(F32)
    if scale < 1 and antialias:
        w = (F32(scale) * _cubic((dist * F32(scale)).astype(F32))).astype(F32)
    else:
        w = _cubic(dist)
    w = (w / w.sum(1, dtype=F32)[:, None]).astype(F32)
    zeros = (w == 0).sum(0)           # counted once, before either narrow (:286-291)
    if zeros[0] != 0:
        ind, w = ind[:, 1:P - 1], w[:, 1:P - 1]
    if zeros[-1] != 0:
        ind, w = ind[:, :P - 2], w[:, :P - 2]      # a no-op after the first narrow
    s0 = int(-ind.min() + 1)
    s1 = int(ind.max() - in_len)
    return w, (ind[:, 0] + s0 - 1).astype(np.int64), s0, s1


def _sym_index(j, n, s0):
    """row of the symmetric-padded image (data/util.py:325-335) -> source row"""
    k = j - s0
    return np.where(k < 0, -k - 1, np.where(k >= n, 2 * n - 1 - k, k))


def imresize_np(img, scale, antialias=True, dtype=np.float64):
    """data/util.py:302-371 imresize_np: HWC image (the harness feeds cv2's uint8 BGR frames),
    separable cubic resize along H then W with symmetric padding; float output, no rounding."""
    img = np.asarray(img, dtype)
    H, W, Cc = img.shape
    oH, oW = int(np.ceil(H * scale)), int(np.ceil(W * scale))
    wH, iH, sH, _ = resize_weights_indices(H, oH, scale, antialias)
    wW, iW, sW, _ = resize_weights_indices(W, oW, scale, antialias)
    rows = _sym_index(iH[:, None] + np.arange(wH.shape[1])[None, :], H, sH)       # [oH, P]
    out1 = np.einsum("ip,ipxc->ixc", wH.astype(dtype), img[rows])
    cols = _sym_index(iW[:, None] + np.arange(wW.shape[1])[None, :], W, sW)       # [oW, P]
    return np.einsum("jp,ijpc->ijc", wW.astype(dtype), out1[:, cols])
