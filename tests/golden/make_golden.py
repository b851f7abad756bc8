"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
STIF model (``/root/reference/codes``) on CPU in this container.

Only this script touches ``/root/reference``; it is run by hand (it skips when the
reference is absent) and its outputs -- inputs + expected outputs, plain data --
are committed.  The GPU box never sees the reference.

Three shims make the reference importable without CUDA:
  1. a stub ``torchvision`` (``SIREN.py:8`` imports names it never uses);
  2. a stub ``_ext`` whose ``dcn_v2_forward`` is a CPU restatement of
     ``dcn_v2_cuda_forward`` (``DCNv2/src/cuda/dcn_v2_cuda.cu:42-172``) with the
     sampling of ``modulated_deformable_im2col_gpu_kernel`` /
     ``dmcn_im2col_bilinear`` (``dcn_v2_im2col_cuda.cu:25-54,125-195``).  The
     native extension itself cannot be built here (it needs the removed THC API),
     so the DCN core is pinned by the reference's own zero-offset known-answer
     test (``DCNv2/test.py:32-67``), which this script also records;
  3. ``Tensor.cuda = identity`` for the hard ``.cuda()`` calls
     (``convlstm.py:62-63``, ``Sakuya_arch_test.py:372-375``).
Weights come from ``stif_amd.weights.make_state_dict(seed=0)`` and are loaded
with ``load_state_dict(strict=True)``.

Usage:  python tests/golden/make_golden.py             (model, window and per-op fixtures)
        python tests/golden/make_golden.py decoders    (decoding_test / _fasttest / _localensemble)
        python tests/golden/make_golden.py harness     (custom_video_test's imresize_np input resize)
        python tests/golden/make_golden.py single      (custom_video_test's single_forward, 11x13 pair)
        python tests/golden/make_golden.py c0          (BASELINE config C0: one full 128x128 pair, t=0.5)
        python tests/golden/make_golden.py gratings    (C0-sized moving-grating pair, analytic ground truth)
        python tests/golden/make_golden.py c1          (BASELINE config C1: one full 256x256 pair, pinned pixels)
        python tests/golden/make_golden.py c2|c3|c4    (the encoder's latent of one full-size C2 / C3 / C4 pair, pinned)
        python tests/golden/make_golden.py chunk-check (the row-chunked DCN shim == the unchunked one)
        python tests/golden/make_golden.py sched       (lr sequences of the reference's two restart schedules)
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/codes"


def dcn_v2_forward_cpu(input, weight, bias, offset, mask, kh, kw, sh, sw, ph, pw, dh, dw, dg):
    """fp32 CPU restatement of the reference CUDA forward (see module docstring)."""
    B, C, H, W = input.shape
    Co = weight.shape[0]
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    cpg = C // dg
    K = kh * kw
    cols = torch.zeros(B, C, K, Ho, Wo, dtype=torch.float32)
    h_in = (torch.arange(Ho) * sh - ph).view(1, 1, Ho, 1)
    w_in = (torch.arange(Wo) * sw - pw).view(1, 1, 1, Wo)
    img = input.reshape(B, C, H * W)
    for i in range(kh):
        for j in range(kw):
            k = i * kw + j
            off = offset.view(B, dg, K, 2, Ho, Wo)
            off_h = off[:, :, k, 0]
            off_w = off[:, :, k, 1]
            m = mask.view(B, dg, K, Ho, Wo)[:, :, k]
            h_im = (h_in + i * dh).float() + off_h          # [B, dg, Ho, Wo]
            w_im = (w_in + j * dw).float() + off_w
            inside = (h_im > -1) & (w_im > -1) & (h_im < H) & (w_im < W)
            h_low = torch.floor(h_im)
            w_low = torch.floor(w_im)
            lh = h_im - h_low
            lw = w_im - w_low
            hh = 1 - lh
            hw = 1 - lw
            h_low = h_low.long()
            w_low = w_low.long()
            h_high = h_low + 1
            w_high = w_low + 1

            def corner(hc, wc, ok):
                idx = (hc.clamp(0, H - 1) * W + wc.clamp(0, W - 1))     # [B, dg, Ho, Wo]
                idx = idx.repeat_interleave(cpg, dim=1).view(B, C, Ho * Wo)
                v = torch.gather(img, 2, idx).view(B, C, Ho, Wo)
                return torch.where(ok.repeat_interleave(cpg, dim=1), v, torch.zeros((), dtype=v.dtype))

            v1 = corner(h_low, w_low, (h_low >= 0) & (w_low >= 0))
            v2 = corner(h_low, w_high, (h_low >= 0) & (w_high <= W - 1))
            v3 = corner(h_high, w_low, (h_high <= H - 1) & (w_low >= 0))
            v4 = corner(h_high, w_high, (h_high <= H - 1) & (w_high <= W - 1))
            rep = lambda t: t.repeat_interleave(cpg, dim=1)
            w1, w2, w3, w4 = rep(hh * hw), rep(hh * lw), rep(lh * hw), rep(lh * lw)
            val = w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4
            val = torch.where(rep(inside), val, torch.zeros((), dtype=val.dtype))
            cols[:, :, k] = val * rep(m)
    cols = cols.view(B, C * K, Ho * Wo)
    out = torch.einsum("ok,bkn->bon", weight.reshape(Co, C * K), cols) + bias.view(1, Co, 1)
    return out.view(B, Co, Ho, Wo)


def install_shims():
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    for n in ["Resize", "Compose", "ToTensor", "Normalize"]:
        setattr(tvt, n, object)
    tv.transforms = tvt
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tvt
    ext = types.ModuleType("_ext")
    ext.dcn_v2_forward = dcn_v2_forward_cpu
    sys.modules["_ext"] = ext
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF)


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    install_shims()
    sys.path.insert(0, REPO)
    import stif_pkg
    stif = stif_pkg.load()
    import models.modules.Sakuya_arch_test as S
    import models.modules.warplayer as WL
    from models.modules.convlstm import ConvLSTMCell
    from models.modules.DCNv2.dcn_v2 import dcn_v2_conv, DCNv2

    torch.set_num_threads(8)
    sd_np = stif.weights.make_state_dict(seed=0)
    model = S.LunaTokis(64, 6, 8, 5, 40)
    ref_sd = model.state_dict()
    json.dump([[k, list(v.shape)] for k, v in ref_sd.items()],
              open(os.path.join(HERE, "state_dict_spec.json"), "w"))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    model.eval()

    # ---------------- full model, small non-square LR -----------------
    cap = {}

    def hook(name):
        def fn(mod, inp, out):
            cap.setdefault(name, []).append(out)
        return fn

    model.pcd_align.register_forward_hook(hook("pcd_align"))
    model.fusion.register_forward_hook(hook("fusion"))
    model.ConvBLSTM.register_forward_hook(hook("bilstm"))
    model.feat_imnet.register_forward_hook(hook("feat_imnet"))
    model.flow_imnet.register_forward_hook(hook("flow_imnet"))
    model.ConvBLSTM.forward_net.pcd_h.register_forward_hook(hook("pcd_h"))
    model.ConvBLSTM.forward_net.cell_list[0].register_forward_hook(hook("cell"))

    g = torch.Generator().manual_seed(1234)
    H, W = 16, 20
    x = torch.rand(1, 2, 3, H, W, generator=g)
    times = [0.0, 0.25, 0.5, 0.75]
    with torch.no_grad():
        outs = model(x, [torch.tensor([[t]]) for t in times])
        feat = model.feat
        out25 = model.decoding([torch.tensor([[0.5]])], scale=(40, 50))[0]
    hr = cap["feat_imnet"][2].view(1, H * 4 * W * 4, 64)
    fl = cap["flow_imnet"][2].view(1, H * 4 * W * 4, 4)
    np.savez_compressed(
        os.path.join(HERE, "model_16x20.npz"),
        x=f32(x), times=np.array(times, np.float32), out=np.stack([f32(o[0]) for o in outs]),
        feat=f32(feat[0]), out_scale_40x50=f32(out25[0]),
        pcd_align=f32(cap["pcd_align"][0][0]), fusion=f32(cap["fusion"][0][0]),
        bilstm=f32(cap["bilstm"][0][0]), pcd_h_t0=f32(cap["pcd_h"][0][0]),
        cell_h_t0=f32(cap["cell"][0][0][0]), cell_c_t0=f32(cap["cell"][0][1][0]),
        hrfeat_t05=f32(hr[0]), flow_t05=f32(fl[0]),
    )
    print("model: out", [tuple(o.shape) for o in outs], "range", float(outs[2].min()), float(outs[2].max()))

    # ---------------- 7-frame sliding window (custom_video_test.py:81-97) -----
    g = torch.Generator().manual_seed(4321)
    frames = torch.rand(7, 3, 16, 16, generator=g)
    wouts = []
    with torch.no_grad():
        for i in range(6):
            wouts.append(model(frames[i:i + 2][None], [torch.tensor([[0.5]])])[0][0])
    np.savez_compressed(os.path.join(HERE, "window_7x16x16.npz"),
                        frames=f32(frames), out=np.stack([f32(o) for o in wouts]))
    print("window done")

    # ---------------- per-op fixtures -----------------
    ops = {}
    g = torch.Generator().manual_seed(99)
    # DCN zero-offset KAT, DCNv2/test.py:32-67 (identity kernel, mask = sigmoid(0))
    N_, C_, H_, W_ = 2, 2, 4, 4
    inp = torch.randn(N_, C_, H_, W_, generator=g)
    wid = torch.zeros(C_, C_, 3, 3)
    for p in range(C_):
        wid[p, p, 1, 1] = 1.0
    off0 = torch.zeros(N_, 2 * 9, H_, W_)
    m0 = torch.sigmoid(torch.zeros(N_, 9, H_, W_))
    out_kat = dcn_v2_conv(inp, off0, m0, wid, torch.zeros(C_), 1, 1, 1, 1)
    assert float((inp - 2 * out_kat).abs().max()) < 1e-10
    ops["kat_input"] = f32(inp)

    # DCN_sep module of the reference on random tensors (dcn_v2.py:127-140)
    dsep = model.pcd_align.L2_dcnpack_1
    a = torch.rand(2, 64, 9, 11, generator=g)
    b = torch.rand(2, 64, 9, 11, generator=g) * 2 - 0.5
    with torch.no_grad():
        ops["dcnsep_out"] = f32(dsep(a, b))
    ops["dcnsep_in"] = f32(a)
    ops["dcnsep_fea"] = f32(b)

    # bilinear x2 upsample (PCD_Align uses it 4x per direction, :86-125)
    u = torch.randn(2, 5, 6, 7, generator=g)
    ops["up2_in"] = f32(u)
    ops["up2_out"] = f32(F.interpolate(u, scale_factor=2, mode="bilinear", align_corners=False))

    # grid_sample bilinear, zeros padding, align_corners=False with out-of-range grid points
    gi = torch.randn(1, 7, 9, 11, generator=g)
    gg = torch.rand(1, 1, 500, 2, generator=g) * 2.6 - 1.3
    ops["gs_in"] = f32(gi)
    ops["gs_grid"] = f32(gg)
    ops["gs_bilinear"] = f32(F.grid_sample(gi, gg, mode="bilinear", align_corners=False))
    ops["gs_nearest"] = f32(F.grid_sample(gi, gg, mode="nearest", align_corners=False))

    # nearest-index maps of the decoder's first gather (Sakuya_arch_test.py:382-393), incl. 2.5x ties
    sizes = [(16, 20, 40, 50), (24, 32, 60, 80), (135, 240, 337, 600), (32, 32, 128, 128), (5, 7, 13, 17), (16, 20, 64, 80)]
    for (h, w, hh, ww) in sizes:
        c = S.make_coord((hh, ww)).clamp(-1 + 1e-6, 1 - 1e-6)
        idx_img = torch.arange(h * w).float().view(1, 1, h, w)
        o = F.grid_sample(idx_img, c.flip(-1).unsqueeze(0).unsqueeze(0), mode="nearest", align_corners=False)
        o = o[0, 0, 0].long().view(hh, ww)
        ops[f"nearest_{h}x{w}_{hh}x{ww}_row"] = (o[:, 0] // w).numpy().astype(np.int32)
        ops[f"nearest_{h}x{w}_{hh}x{ww}_col"] = (o[0, :] % w).numpy().astype(np.int32)
        ops[f"coord_{hh}x{ww}"] = f32(S.make_coord((hh, ww)))

    # SIREN (feat_imnet) on random input
    si = torch.rand(100, 201, generator=g) * 2 - 1
    with torch.no_grad():
        ops["siren_in"] = f32(si)
        ops["siren_out"] = f32(model.feat_imnet(si))

    # warpgrid (warplayer.py:25-39)
    fl_in = torch.randn(1, 2, 12, 16, generator=g) * 3
    ops["warp_flow"] = f32(fl_in)
    ops["warp_grid"] = f32(WL.warpgrid(torch.zeros(1, 3, 12, 16), fl_in)[0])

    # ConvLSTMCell (convlstm.py:42-58) with the model's cell weights
    cx = torch.randn(1, 64, 6, 8, generator=g)
    ch = torch.randn(1, 64, 6, 8, generator=g)
    cc = torch.randn(1, 64, 6, 8, generator=g)
    with torch.no_grad():
        hn, cn = model.ConvBLSTM.forward_net.cell_list[0](cx, [ch, cc])
    ops.update(cell_x=f32(cx), cell_h=f32(ch), cell_c=f32(cc), cell_hn=f32(hn), cell_cn=f32(cn))
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops)
    print("ops done:", len(ops))


def decoders():
    """decoding_test / decoding_fasttest / decoding_localensemble (Sakuya_arch_test.py:461-598,
    863-1085) on the model_16x20 latent -> decoders_16x20.npz"""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    install_shims()
    sys.path.insert(0, REPO)
    import stif_pkg
    stif = stif_pkg.load()
    import models.modules.Sakuya_arch_test as S

    torch.set_num_threads(8)
    sd_np = stif.weights.make_state_dict(seed=0)
    model = S.LunaTokis(64, 6, 8, 5, 40)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    model.eval()
    g = torch.Generator().manual_seed(1234)
    H, W = 16, 20
    x = torch.rand(1, 2, 3, H, W, generator=g)         # the model_16x20 input
    res = {"x": f32(x)}
    with torch.no_grad():
        t_test = [0.25, 0.5]
        outs = model(x, [torch.tensor([[t]]) for t in t_test], test=True)      # forward(test=True)
        res["test_times"] = np.array(t_test, np.float32)
        res["test_out"] = np.stack([f32(o[0]) for o in outs])
        o3 = model.decoding_test([torch.tensor([[0.5]])], 3)[0]                 # HH = 3H, HRinp still x4
        res["test_out_scale3"] = f32(o3[0])
        t_fast = [0.0, 0.5, 0.75]
        res["fast_times"] = np.array(t_fast, np.float32)
        res["fast_out"] = f32(model.decoding_fasttest(t_fast))
        res["fast_out_40x50"] = f32(model.decoding_fasttest([0.5], (40, 50)))
        res["ens_out"] = f32(model.decoding_localensemble([0.5]))
        res["ens_out_40x50"] = f32(model.decoding_localensemble([0.25], (40, 50)))
    np.savez_compressed(os.path.join(HERE, "decoders_16x20.npz"), **res)
    print("decoders:", {k: v.shape for k, v in res.items()})


def harness():
    """custom_video_test.py's input resize: data.util.imresize_np(img_uint8_bgr, 1/2, True)
    (data/util.py:240-371) on cv2-style uint8 HWC frames -> harness.npz"""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    install_shims()
    # data/util.py imports cv2 at module level; imresize_np itself is pure torch (stub only)
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    from data.util import imresize_np, calculate_weights_indices
    rng = np.random.default_rng(77)
    res = {}
    for (h, w) in [(37, 50), (64, 90), (21, 33)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        res[f"img_{h}x{w}"] = img
        res[f"half_{h}x{w}"] = imresize_np(img, 1 / 2, True).astype(np.float32)
    wts, idx, s0, s1 = calculate_weights_indices(37, 19, 0.5, "cubic", 4, True)
    res["w_37_19"] = wts.numpy().astype(np.float32)
    res["i_37_19"] = idx.numpy().astype(np.int64)
    res["sym_37_19"] = np.array([s0, s1], np.int64)
    np.savez_compressed(os.path.join(HERE, "harness.npz"), **res)
    print("harness:", {k: v.shape for k, v in res.items()})


def _reference_model():
    install_shims()
    sys.path.insert(0, REPO)
    import stif_pkg
    stif = stif_pkg.load()
    import models.modules.Sakuya_arch_test as S
    torch.set_num_threads(8)
    sd_np = stif.weights.make_state_dict(seed=0)
    model = S.LunaTokis(64, 6, 8, 5, 40)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    return model.eval()


def single():
    """custom_video_test.py:41-54 (single_forward) on an 11x13 pair: zero-pad bottom/right to 12x16,
    the eight times i/8, outputs not cropped -> single_11x13.npz.  The script itself cannot be
    imported (cv2, module-level file I/O), so its five lines are restated here around the reference
    model call."""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    model = _reference_model()
    g = torch.Generator().manual_seed(2024)
    imgs_in = torch.rand(1, 2, 3, 11, 13, generator=g)
    with torch.no_grad():
        b, n, c, h, w = imgs_in.size()
        h_n, w_n = int(4 * np.ceil(h / 4)), int(4 * np.ceil(w / 4))
        imgs_temp = imgs_in.new_zeros(b, n, c, h_n, w_n)
        imgs_temp[:, :, :, 0:h, 0:w] = imgs_in
        time_Tensors = [torch.tensor([i / 8])[None] for i in range(8)]
        outs = model(imgs_temp, time_Tensors)
    np.savez_compressed(os.path.join(HERE, "single_11x13.npz"), x=f32(imgs_in),
                        out=np.stack([f32(o[0]) for o in outs]))
    print("single_forward:", tuple(outs[0].shape), len(outs))


def c0():
    """BASELINE.json configs[0] (C0): one full 128x128 pair of bench.py's synthetic window (frames 0
    and 1, torch.Generator seeds 1234 / 1235, torch.rand(3, 128, 128)), 4x, t = 0.5, through the
    reference model -> c0_pair_128.npz (output [3, 512, 512] float32)."""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    model = _reference_model()
    fr = []
    for i in range(2):
        g = torch.Generator().manual_seed(1234 + i)
        fr.append(torch.rand(3, 128, 128, generator=g))
    x = torch.stack(fr)[None]
    with torch.no_grad():
        out = model(x, [torch.tensor([[0.5]])])[0]
    np.savez_compressed(os.path.join(HERE, "c0_pair_128.npz"), x=f32(x), out=f32(out[0]))
    print("c0 pair:", tuple(out.shape), float(out.min()), float(out.max()))


def c1_pins(H=256, W=256, seed=7):
    """(latent (y, x) positions, HR output (y, x) positions) pinned by c1(): the rows and columns where the
    engine's tiles meet (Winograd: 4-row x 32-column tiles; DCN: 4 x 32; decoder: 32-pixel blocks) and
    the frame's edges, plus random positions"""
    rng = np.random.default_rng(seed)
    ly = [0, 1, 3, 4, 127, 128, H - 2, H - 1]
    lx = [0, 31, 32, 33, W - 1]
    fy = np.concatenate([np.repeat(ly, W), np.tile(np.arange(H), len(lx)), rng.integers(0, H, 1024)])
    fx = np.concatenate([np.tile(np.arange(W), len(ly)), np.repeat(lx, H), rng.integers(0, W, 1024)])
    HH, WW = 4 * H, 4 * W
    hy = [0, 1, 2, 3, 4, 511, 512, HH - 1]
    hx = [0, 31, 32, 127, 128, WW - 1]
    k = 256
    oy = np.concatenate([np.repeat(hy, k), rng.integers(0, HH, len(hx) * k), rng.integers(0, HH, 4096)])
    ox = np.concatenate([rng.integers(0, WW, len(hy) * k), np.repeat(hx, k), rng.integers(0, WW, 4096)])
    return fy.astype(np.int64), fx.astype(np.int64), oy.astype(np.int64), ox.astype(np.int64)


def c1():
    """BASELINE.json configs[1] (C1) at full size: one 256x256 pair of bench.py's synthetic window (frames
    0 and 1, torch.Generator seeds 1234 / 1235), 4x, t = 0.5, through the reference model; the latent
    (reference ``self.feat``) and the 1024x1024 output are kept at the positions c1_pins() picks ->
    c1_pair_pins.npz (the full tensors would be 50 MB + 12 MB)."""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    model = _reference_model()
    fr = []
    for i in range(2):
        g = torch.Generator().manual_seed(1234 + i)
        fr.append(torch.rand(3, 256, 256, generator=g))
    x = torch.stack(fr)[None]
    with torch.no_grad():
        out = model(x, [torch.tensor([[0.5]])])[0][0]
    feat = model.feat[0]                        # [3, 64, 256, 256]
    fy, fx, oy, ox = c1_pins()
    np.savez_compressed(os.path.join(HERE, "c1_pair_pins.npz"), x=f32(x), feat_y=fy, feat_x=fx,
                        feat=f32(feat[:, :, fy, fx]), out_y=oy, out_x=ox, out=f32(out[:, oy, ox]))
    print("c1 pair:", tuple(out.shape), tuple(feat.shape), len(fy), len(oy))


LARGE = {
    # BASELINE configs whose encoder runs at sizes no test can run the reference at: (H, W, pins seed)
    "c2": (540, 960, 11),      # configs[2]: the Vimeo-septuplet shape
    "c3": (720, 1280, 13),     # configs[3]: one 720p pair of the 64-frame sequence (a rank's window)
    "c4": (1080, 1920, 17),    # configs[4]: one 1080p pair
}


def large_pins(H, W, seed):
    """Latent (y, x) positions pinned by large(): where the engine's tiles meet at every pyramid level
    (Winograd / DCN 4-row x 32-column tiles at L1, their L2 / L3 images at 2x / 4x -- at 960 / 1280 /
    1920 the L3 width 240 / 320 / 480 leaves a partial last 32-column tile at 960 and 1920), the
    frame edges and random pixels: 8 positions on each seam row / column, plus 1,536 random ones."""
    rng = np.random.default_rng(seed)
    seam_y = sorted({0, 1, 2, 3, 4, 7, 8, 15, 16, H // 2 - 1, H // 2, H - 8, H - 5, H - 4, H - 3, H - 2, H - 1})
    l3w = W // 4
    seam_x = sorted({0, 1, 31, 32, 63, 64, 127, 128, W // 2, 4 * (l3w // 32) * 32 - 1, 4 * (l3w // 32) * 32,
                     W - 33, W - 32, W - 2, W - 1})
    seam_y = [v for v in seam_y if 0 <= v < H]
    seam_x = [v for v in seam_x if 0 <= v < W]
    k = 8
    fy = np.concatenate([np.repeat(seam_y, k), rng.integers(0, H, len(seam_x) * k), rng.integers(0, H, 1536)])
    fx = np.concatenate([rng.integers(0, W, len(seam_y) * k), np.repeat(seam_x, k), rng.integers(0, W, 1536)])
    return fy.astype(np.int64), fx.astype(np.int64)


def large(cfg):
    """The encoder (LunaTokis.gen_feat, Sakuya_arch_test.py:313-362) of the reference on one full-size pair
    of bench.py's synthetic frames (frames 0 and 1: torch.Generator seeds 1234 / 1235, torch.rand(3, H, W))
    at a large BASELINE config; the latent (``self.feat`` [1, 3, 64, H, W]) is kept at large_pins() ->
    <cfg>_pair_feat_pins.npz.  The frames are not stored: the GPU test regenerates them from the seeds.
    The DCN shim runs in row chunks (dcn_v2_forward_cpu_chunked) so its columns buffer stays bounded."""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    import time
    H, W, seed = LARGE[cfg]
    model = _reference_model()
    sys.modules["_ext"].dcn_v2_forward = dcn_v2_forward_cpu_chunked
    fr = []
    for i in range(2):
        g = torch.Generator().manual_seed(1234 + i)
        fr.append(torch.rand(3, H, W, generator=g))
    x = torch.stack(fr)[None]
    t0 = time.time()
    with torch.no_grad():
        model.gen_feat(x)
    feat = model.feat[0]                        # [3, 64, H, W]
    fy, fx = large_pins(H, W, seed)
    np.savez_compressed(os.path.join(HERE, f"{cfg}_pair_feat_pins.npz"), H=np.int64(H), W=np.int64(W),
                        frame_seeds=np.array([1234, 1235], np.int64), feat_y=fy, feat_x=fx,
                        feat=f32(feat[:, :, fy, fx]))
    print(f"{cfg} pair latent:", tuple(feat.shape), len(fy), f"{time.time() - t0:.0f} s")


def dcn_v2_forward_cpu_chunked(input, weight, bias, offset, mask, kh, kw, sh, sw, ph, pw, dh, dw, dg, rows=64):
    """dcn_v2_forward_cpu over blocks of output rows (an output row depends only on its own offsets and mask
    and on the input), each block gathering from the window of input rows its samples can reach; bounds
    the columns buffer at 1080p.  Coordinates stay the image's own (same fp32 expressions as
    dcn_v2_forward_cpu), so the result is the unchunked one."""
    B, C, H, W = input.shape
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    if Ho <= rows or (kh, kw, sh, ph, dh) != (3, 3, 1, 1, 1):
        return dcn_v2_forward_cpu(input, weight, bias, offset, mask, kh, kw, sh, sw, ph, pw, dh, dw, dg)
    M = 8                                              # row margin: |row offset| < M (checked)
    cpg = C // dg
    K = kh * kw
    rep = lambda t: t.repeat_interleave(cpg, dim=1)
    off_all = offset.view(B, dg, K, 2, Ho, Wo)
    assert float(off_all[:, :, :, 0].abs().max()) < M, "chunked DCN shim: row offsets beyond the margin"
    msk_all = mask.view(B, dg, K, Ho, Wo)
    outs = []
    for r0 in range(0, Ho, rows):
        r1 = min(Ho, r0 + rows)
        n = r1 - r0
        lo = max(0, r0 - ph - M)                       # input rows the block can reach: lo .. hi - 1
        hi = min(H, r1 - 1 - ph + dh * (kh - 1) + M + 2)
        img = input[:, :, lo:hi].reshape(B, C, (hi - lo) * W)
        cols = torch.zeros(B, C, K, n, Wo, dtype=torch.float32)
        h_in = (torch.arange(r0, r1) * sh - ph).view(1, 1, n, 1)
        w_in = (torch.arange(Wo) * sw - pw).view(1, 1, 1, Wo)
        for i in range(kh):
            for j in range(kw):
                k = i * kw + j
                h_im = (h_in + i * dh).float() + off_all[:, :, k, 0, r0:r1]
                w_im = (w_in + j * dw).float() + off_all[:, :, k, 1, r0:r1]
                inside = (h_im > -1) & (w_im > -1) & (h_im < H) & (w_im < W)
                h_low = torch.floor(h_im)
                w_low = torch.floor(w_im)
                lh = h_im - h_low
                lw = w_im - w_low
                hh = 1 - lh
                hw = 1 - lw
                h_low = h_low.long()
                w_low = w_low.long()
                h_high = h_low + 1
                w_high = w_low + 1

                def corner(hc, wc, ok):
                    idx = ((hc.clamp(0, H - 1) - lo).clamp(0, hi - lo - 1) * W + wc.clamp(0, W - 1))
                    idx = idx.repeat_interleave(cpg, dim=1).view(B, C, n * Wo)
                    v = torch.gather(img, 2, idx).view(B, C, n, Wo)
                    return torch.where(rep(ok), v, torch.zeros((), dtype=v.dtype))

                v1 = corner(h_low, w_low, (h_low >= 0) & (w_low >= 0))
                v2 = corner(h_low, w_high, (h_low >= 0) & (w_high <= W - 1))
                v3 = corner(h_high, w_low, (h_high <= H - 1) & (w_low >= 0))
                v4 = corner(h_high, w_high, (h_high <= H - 1) & (w_high <= W - 1))
                val = rep(hh * hw) * v1 + rep(hh * lw) * v2 + rep(lh * hw) * v3 + rep(lh * lw) * v4
                val = torch.where(rep(inside), val, torch.zeros((), dtype=val.dtype))
                cols[:, :, k] = val * rep(msk_all[:, :, k, r0:r1])
        cols = cols.view(B, C * K, n * Wo)
        o = torch.einsum("ok,bkn->bon", weight.reshape(weight.shape[0], C * K), cols) + bias.view(1, -1, 1)
        outs.append(o.view(B, -1, n, Wo))
    return torch.cat(outs, dim=2)


def chunk_check():
    """dcn_v2_forward_cpu_chunked reproduces dcn_v2_forward_cpu bit for bit (offsets up to 6 px, a map whose
    rows span several blocks incl. a partial last one and the image edges)."""
    g = torch.Generator().manual_seed(5)
    B, C, H, W, dg = 1, 16, 150, 40, 2
    inp = torch.randn(B, C, H, W, generator=g)
    wt = torch.randn(8, C, 3, 3, generator=g)
    bs = torch.randn(8, generator=g)
    off = (torch.rand(B, 2 * dg * 9, H, W, generator=g) * 12 - 6)
    m = torch.rand(B, dg * 9, H, W, generator=g)
    a = dcn_v2_forward_cpu(inp, wt, bs, off, m, 3, 3, 1, 1, 1, 1, 1, 1, dg)
    b = dcn_v2_forward_cpu_chunked(inp, wt, bs, off, m, 3, 3, 1, 1, 1, 1, 1, 1, dg, rows=32)
    print("chunked shim max |diff|:", float((a - b).abs().max()), "equal:", bool(torch.equal(a, b)))


def gratings_c0():
    """The moving-grating pair of bench.py (frames 0 and 1 of bench.gratings at 128 x 128, SURVEY.md
    section 8d input (ii)) through the reference model, 4x, t = 0.5 -> gratings_128.npz; bench.py
    measures the PSNR criterion against its analytic ground truth (bench.gratings_gt)."""
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    sys.path.insert(0, REPO)
    from bench import gratings
    model = _reference_model()
    x = torch.from_numpy(gratings(0, 2, 128, 128))[None]
    with torch.no_grad():
        out = model(x, [torch.tensor([[0.5]])])[0]
    np.savez_compressed(os.path.join(HERE, "gratings_128.npz"), x=f32(x), out=f32(out[0]))
    print("gratings pair:", tuple(out.shape), float(out.min()), float(out.max()))


def sched():
    """lr_scheduler.py (CosineAnnealingLR_Restart, MultiStepLR_Restart) driven as VideoSRBaseModel drives them
    (base_model.py:51-63 update_learning_rate: scheduler.step() per iteration, then the warm-up override),
    recorded per iteration -> lr_schedules.json.  Pure torch: no shims needed."""
    sys.path.insert(0, os.path.join(REF, "models"))
    import lr_scheduler as LS
    cases = {
        # the shipped option file's shape (train_zsm.yml:57-65), periods scaled down 15,000x
        "cosine_zsm": dict(kind="cos", lr=2e-4, T_period=[10, 10, 10, 10], restarts=[10, 20, 30],
                           weights=[1, 1, 1], eta_min=1e-7, iters=45, warmup=-1),
        # one period, no restarts: the schedule runs past T_max (the k = T + 1 (mod 2T) branch)
        "cosine_wrap": dict(kind="cos", lr=1e-3, T_period=[5], restarts=None, weights=None, eta_min=1e-6,
                            iters=23, warmup=-1),
        # weighted restarts of different lengths, with a 3-iteration warm-up
        "cosine_weighted": dict(kind="cos", lr=4e-4, T_period=[6, 4, 8], restarts=[6, 10], weights=[0.5, 0.25],
                                eta_min=0, iters=24, warmup=3),
        "multistep": dict(kind="ms", lr=2e-4, milestones=[3, 6, 6, 9, 15], restarts=[12], weights=[0.3],
                          gamma=0.5, iters=20, warmup=-1),
    }
    out = {}
    for name, c in cases.items():
        p = torch.zeros(3, requires_grad=True)
        opt = torch.optim.Adam([p], lr=c["lr"], weight_decay=0, betas=(0.9, 0.99))
        if c["kind"] == "cos":
            sch = LS.CosineAnnealingLR_Restart(opt, c["T_period"], eta_min=c["eta_min"], restarts=c["restarts"],
                                               weights=c["weights"])
        else:
            sch = LS.MultiStepLR_Restart(opt, c["milestones"], restarts=c["restarts"], weights=c["weights"],
                                         gamma=c["gamma"])
        lrs = [opt.param_groups[0]["lr"]]
        for it in range(1, c["iters"] + 1):
            sch.step()
            if it < c["warmup"]:
                opt.param_groups[0]["lr"] = opt.param_groups[0]["initial_lr"] / c["warmup"] * it
            lrs.append(opt.param_groups[0]["lr"])
        out[name] = dict(case={k: v for k, v in c.items()}, lr=lrs)
        print(name, ["%.3e" % v for v in lrs[:8]], "...")
    with open(os.path.join(HERE, "lr_schedules.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["sched"]:
        sched()
        sys.exit(0)
    if sys.argv[1:] == ["gratings"]:
        gratings_c0()
        sys.exit(0)
    if sys.argv[1:] == ["single"]:
        single()
        sys.exit(0)
    if sys.argv[1:] == ["c0"]:
        c0()
        sys.exit(0)
    if sys.argv[1:] == ["c1"]:
        c1()
        sys.exit(0)
    if len(sys.argv) == 2 and sys.argv[1] in LARGE:
        large(sys.argv[1])
        sys.exit(0)
    if sys.argv[1:] == ["chunk-check"]:
        chunk_check()
        sys.exit(0)
    if sys.argv[1:] == ["decoders"]:
        decoders()
        sys.exit(0)
    if sys.argv[1:] == ["harness"]:
        harness()
        sys.exit(0)
    main()
