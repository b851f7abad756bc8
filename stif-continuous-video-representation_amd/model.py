"""LunaTokis host: the reference model API driving the gfx950 kernels.

Mirrors ``codes/models/modules/Sakuya_arch_test.py:LunaTokis`` -- constructor
``LunaTokis(nf, nframes, groups, front_RBs, back_RBs)`` (:268-311),
``forward(x, times, scale=None, test=False)`` (:1222-1231), ``gen_feat`` (:313-362),
``decoding`` (:364-459), ``load_state_dict(sd, strict=True)`` over the reference's
442 keys -- but holds repacked device weights and runs every layer through
libstif_hip.so (see ops.py); no torch.nn module is on the path.

Work is batched across everything the reference runs sequentially but that is
independent: both PCD_Align directions (different weights -> launch groups), both
ConvLSTM directions (BiDeformableConvLSTM runs the same net on x and reversed x,
:256-266), pcd_h and pcd_c, all pairs of a window, and all three latent steps of
the reconstruction trunk.  Per-frame encoder features are computed once per frame
(a sliding window shares each inner frame between two pairs).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from . import _lib as L
from . import ops
from . import weights as W
from .coords import ensemble_weights


def _np(v):
    if isinstance(v, np.ndarray):
        return v.astype(np.float32, copy=False)
    return v.detach().cpu().numpy().astype(np.float32, copy=False)


class LunaTokis:
    """STIF LunaTokis (Sakuya_arch_test.py:268) on MI355X."""

    def __init__(self, nf=64, nframes=3, groups=8, front_RBs=5, back_RBs=10, device="cuda", winograd=True,
                 mfma="f16x3"):
        if nf != 64 or groups != 8:
            raise ValueError("the gfx950 kernels implement nf=64, groups=8 (the shipped STIF configuration)")
        self.nf, self.groups = nf, groups
        self.in_frames = 1 + nframes // 2        # unused attributes kept for API parity (:272-273)
        self.ot_frames = nframes
        self.front_RBs, self.back_RBs = front_RBs, back_RBs
        self.device = torch.device(device)
        self._spec = W.state_dict_spec(nf, front_RBs, back_RBs, groups)
        self._host = None
        self.layers = {}
        self.feat = None
        self.inp = None
        self._tables = {}
        self.training = False
        # 3x3 convs by Winograd F(2x2,3x3) where the shape allows (fp32 throughout); False = direct
        self.winograd = bool(winograd)
        # operand arithmetic of the Winograd convs: "f32" (fp32 MFMA) or "f16x3" (fp32 products
        # from three fp16 MFMAs on split operands, ~22-bit operands, fp32 accumulation; stif.h)
        if mfma not in ("f32", "f16x3"):
            raise ValueError("mfma must be 'f32' or 'f16x3'")
        self.mfma = mfma
        self._dec_flags = L.CONV_F16X3 if mfma == "f16x3" else 0   # decoder SIREN layers likewise

    # ------------------------------------------------------------------ nn.Module-like API
    def eval(self):
        return self

    def train(self, mode=True):
        if mode:
            raise NotImplementedError("training (DCNv2 backward) is out of scope; inference only")
        return self

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("LunaTokis (stif_amd) runs on the GPU only")
        if self._host is not None and device != self.device:
            self.device = device
            self._pack()
        self.device = device
        return self

    def cuda(self, device=None):
        return self.to("cuda" if device is None else torch.device("cuda", device))

    def __call__(self, *a, **k):
        return self.forward(*a, **k)

    def state_dict(self):
        if self._host is None:
            raise RuntimeError("no weights loaded")
        return OrderedDict((k, torch.from_numpy(v.copy())) for k, v in self._host.items())

    def load_state_dict(self, state_dict, strict=True):
        """Same key contract as nn.Module.load_state_dict on the reference module; a
        'module.' prefix (DataParallel/DDP checkpoints) is stripped as base_model.py:93-98 does."""
        sd = OrderedDict()
        for k, v in state_dict.items():
            sd[k[7:] if k.startswith("module.") else k] = v
        missing = [k for k in self._spec if k not in sd]
        unexpected = [k for k in sd if k not in self._spec]
        if strict and (missing or unexpected):
            raise RuntimeError("Error(s) in loading state_dict for LunaTokis:\n"
                               f"\tMissing key(s): {missing}\n\tUnexpected key(s): {unexpected}")
        host = OrderedDict()
        for k, shape in self._spec.items():
            if k in sd:
                a = _np(sd[k])
                if tuple(a.shape) != tuple(shape):
                    raise RuntimeError(f"size mismatch for {k}: copying a param with shape {tuple(a.shape)}, "
                                       f"the shape in current model is {tuple(shape)}")
                host[k] = np.ascontiguousarray(a)
            elif self._host is not None:
                host[k] = self._host[k]
            else:
                host[k] = np.zeros(shape, np.float32)
        self._host = host
        self._pack()
        return type("IncompatibleKeys", (), {"missing_keys": missing, "unexpected_keys": unexpected})()

    # ------------------------------------------------------------------ weight packing
    def _pack(self):
        h, dev = self._host, self.device
        lay = {}

        def conv(name, mode=L.PACK_PLAIN):
            lay[name] = ops.pack_conv(h[name + ".weight"], h[name + ".bias"], mode, dev)

        # 3x3 / stride-1 / 64-cout convs run by Winograd F(2x2,3x3) (stif_conv3x3_wino; the
        # cat(., up(.)) ones on a materialised x2-upsampled second input), as do the offset/mask
        # (64 -> 216) and ConvLSTMCell (128 -> 256, gate epilogue) convs; the strided and 1x1
        # convs keep the direct kernel.
        f16 = L.PACK_F16X3 if self.mfma == "f16x3" else 0
        wino = (L.PACK_WINO | f16) if self.winograd else L.PACK_PLAIN

        lay["conv_first.w"] = torch.from_numpy(h["conv_first.weight"]).to(dev)
        lay["conv_first.b"] = torch.from_numpy(h["conv_first.bias"]).to(dev)
        for i in range(self.front_RBs):
            conv(f"feature_extraction.{i}.conv1", wino)
            conv(f"feature_extraction.{i}.conv2", wino)
        for n in ("fea_L2_conv1", "fea_L3_conv1"):      # 3x3 stride-2 64 -> 64
            conv(n, L.PACK_PLAIN | f16)
        for n in ("fea_L2_conv2", "fea_L3_conv2"):
            conv(n, wino)

        def pcd(prefix):
            for d in (1, 2):
                for ln, cin, _ in W._PCD_LAYERS:
                    n = f"{prefix}{ln}_{d}"
                    if cin is None:
                        conv(n, L.PACK_PLAIN | f16)     # the DCN core (k_dcn)
                        conv(n + ".conv_offset_mask", (L.PACK_WINO_OFFMASK | f16) if self.winograd else L.PACK_OFFMASK)
                    else:
                        conv(n, wino)

        pcd("pcd_align.")
        conv("fusion")
        conv("ConvBLSTM.forward_net.cell_list.0.conv", (L.PACK_WINO_LSTM | f16) if self.winograd else L.PACK_LSTM)
        for p in ("ConvBLSTM.forward_net.pcd_h.", "ConvBLSTM.forward_net.pcd_c."):
            for n in ("fea_L2_conv1", "fea_L3_conv1"):
                conv(p + n, L.PACK_PLAIN | f16)
            conv(p + "fusion")
            for n in ("fea_L2_conv2", "fea_L3_conv2"):
                conv(p + n, wino)
            pcd(p + "pcd_align.")
        conv("ConvBLSTM.conv_1x1")
        for i in range(self.back_RBs):
            conv(f"recon_trunk.{i}.conv1", wino)
            conv(f"recon_trunk.{i}.conv2", wino)
        # decoder
        lib = L.lib()
        self.layers = lay
        self._pack_proj(lr_image=True)

        def siren_ptrs(prefix, n_sine):
            arrs = []
            for i in range(n_sine):
                arrs += [h[f"{prefix}net.{i}.linear.weight"], h[f"{prefix}net.{i}.linear.bias"]]
            arrs += [h[f"{prefix}net.{n_sine}.weight"], h[f"{prefix}net.{n_sine}.bias"]]
            return arrs, (L._P * len(arrs))(*[a.ctypes.data for a in arrs])

        fa, fp = siren_ptrs("feat_imnet.", 3)
        la, lp = siren_ptrs("flow_imnet.", 3)
        ea, ep = siren_ptrs("encode_imnet.", 4)
        mlp = np.empty(lib.stif_dec_mlp_floats(), np.float32)
        L.check(lib.stif_pack_dec_mlp_ex(fp, lp, ep, mlp.ctypes.data, self._dec_flags), "stif_pack_dec_mlp_ex")
        lay["dec.mlp"] = torch.from_numpy(mlp).to(dev)
        self.layers = lay

    def _pack_proj(self, lr_image=True):
        """LR projection of the decoder's first layers (stif_pack_dec_proj_ex); lr_image=False leaves
        the LR frames out of P2..P4 for decoding_test, which samples the x4-upsampled frames."""
        h, dev, lib = self._host, self.device, L.lib()
        wd = np.empty(lib.stif_dec_proj_floats(), np.float32)
        bd = np.empty(lib.stif_conv_bias_floats(256, L.PACK_PLAIN), np.float32)
        L.check(lib.stif_pack_dec_proj_ex(h["feat_imnet.net.0.linear.weight"].ctypes.data,
                                          h["feat_imnet.net.0.linear.bias"].ctypes.data,
                                          h["flow_imnet.net.0.linear.weight"].ctypes.data,
                                          h["encode_imnet.net.0.linear.weight"].ctypes.data, int(lr_image),
                                          wd.ctypes.data, bd.ctypes.data), "stif_pack_dec_proj_ex")
        self.layers["dec.proj" if lr_image else "dec.proj_hrimg"] = ops.PackedConv(
            torch.from_numpy(wd).to(dev), torch.from_numpy(bd).to(dev), 256, 200, 1, L.PACK_PLAIN)

    # ------------------------------------------------------------------ encoder pieces
    def _empty(self, *shape):
        return torch.empty(*shape, device=self.device, dtype=torch.float32)

    def _frame_features(self, frames):
        """conv_first + feature_extraction + pyramid (:318-325) for frames [n,3,H,W] (NCHW)."""
        n, _, H, Wd = frames.shape
        l1 = self._empty(n, H, Wd, 64)
        ops.conv_first(frames, self.layers["conv_first.w"], self.layers["conv_first.b"], l1)
        tmp = self._empty(n, H, Wd, 64)
        for i in range(self.front_RBs):
            self._resblock(l1, tmp, f"feature_extraction.{i}")
        l2, l3 = self._pyramid([(l1, "")])
        return l1, l2[0], l3[0]

    def _resblock(self, x, tmp, name):
        """ResidualBlock_noBN (module_util.py:48-52), x updated in place."""
        ops.conv2d([dict(layer=self.layers[name + ".conv1"], in0=x, out=tmp)], epi=L.EPI_RELU)
        ops.conv2d([dict(layer=self.layers[name + ".conv2"], in0=tmp, out=x, res=x)], epi=L.EPI_RES)

    def _pyramid(self, srcs):
        """fea_L2_conv1/2, fea_L3_conv1/2 with lrelu for a list of (L1 map, weight prefix)."""
        G = len(srcs)
        n, H, Wd, _ = srcs[0][0].shape
        a2 = self._empty(G, n, H // 2, Wd // 2, 64)
        b2 = self._empty(G, n, H // 2, Wd // 2, 64)
        a3 = self._empty(G, n, H // 4, Wd // 4, 64)
        b3 = self._empty(G, n, H // 4, Wd // 4, 64)
        lay = self.layers
        ops.conv2d([dict(layer=lay[p + "fea_L2_conv1"], in0=s, out=a2[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU, stride=2)
        ops.conv2d([dict(layer=lay[p + "fea_L2_conv2"], in0=a2[i], out=b2[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU)
        ops.conv2d([dict(layer=lay[p + "fea_L3_conv1"], in0=b2[i], out=a3[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU, stride=2)
        ops.conv2d([dict(layer=lay[p + "fea_L3_conv2"], in0=a3[i], out=b3[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU)
        return b2, b3

    def _pcd_align(self, units):
        """PCD_Align.forward (:71-130) for up to 8 independent (module, direction) units.
        unit = (prefix, d, fa[L1,L2,L3], fb[L1,L2,L3], y_out)."""
        G = len(units)
        n, H, Wd, _ = units[0][2][0].shape
        lay = self.layers
        lv = [(H, Wd), (H // 2, Wd // 2), (H // 4, Wd // 4)]

        def buf(level, c=64):
            h_, w_ = lv[level]
            return self._empty(G, n, h_, w_, c)

        def L_(u, name):
            return lay[f"{u[0]}{name}_{u[1]}"]

        def LO(u, name):
            return lay[f"{u[0]}{name}_{u[1]}.conv_offset_mask"]

        conv, dcn = ops.conv2d, ops.dcn
        E = enumerate

        def conv_up(make, coarse, scale, epi):
            """conv on cat(x, scale * up2(coarse)) for every unit: fused x2 upsample in the direct
            kernel, or a materialised upsample + the Winograd kernel"""
            if not self.winograd:
                conv([make(i, u, coarse[i]) for i, u in E(units)], epi=epi, in1_mode=2, in1_scale=scale)
                return
            g_, n_, h_, w_, c_ = coarse.shape
            up = self._empty(g_, n_, 2 * h_, 2 * w_, c_)
            ops.upsample2x(coarse.view(g_ * n_, h_, w_, c_), up.view(g_ * n_, 2 * h_, 2 * w_, c_), scale)
            conv([make(i, u, up[i]) for i, u in E(units)], epi=epi, in1_mode=1)
        # ---- L3
        o = buf(2)
        conv([dict(layer=L_(u, "L3_offset_conv1"), in0=u[2][2], in1=u[3][2], out=o[i]) for i, u in E(units)],
             epi=L.EPI_LRELU, in1_mode=1)
        l3off = buf(2)
        conv([dict(layer=L_(u, "L3_offset_conv2"), in0=o[i], out=l3off[i]) for i, u in E(units)], epi=L.EPI_LRELU)
        om = buf(2, 216)
        conv([dict(layer=LO(u, "L3_dcnpack"), in0=l3off[i], out=om[i]) for i, u in E(units)], epi=L.EPI_OFFMASK)
        l3fea = buf(2)
        dcn([dict(layer=L_(u, "L3_dcnpack"), inp=u[2][2], offmask=om[i], out=l3fea[i]) for i, u in E(units)],
            epi=L.EPI_LRELU)
        # ---- L2
        o1 = buf(1)
        conv([dict(layer=L_(u, "L2_offset_conv1"), in0=u[2][1], in1=u[3][1], out=o1[i]) for i, u in E(units)],
             epi=L.EPI_LRELU, in1_mode=1)
        o2 = buf(1)
        conv_up(lambda i, u, c: dict(layer=L_(u, "L2_offset_conv2"), in0=o1[i], in1=c, out=o2[i]),
                l3off, 2.0, L.EPI_LRELU)
        l2off = buf(1)
        conv([dict(layer=L_(u, "L2_offset_conv3"), in0=o2[i], out=l2off[i]) for i, u in E(units)], epi=L.EPI_LRELU)
        om = buf(1, 216)
        conv([dict(layer=LO(u, "L2_dcnpack"), in0=l2off[i], out=om[i]) for i, u in E(units)], epi=L.EPI_OFFMASK)
        d2 = buf(1)
        dcn([dict(layer=L_(u, "L2_dcnpack"), inp=u[2][1], offmask=om[i], out=d2[i]) for i, u in E(units)])
        l2fea = buf(1)
        conv_up(lambda i, u, c: dict(layer=L_(u, "L2_fea_conv"), in0=d2[i], in1=c, out=l2fea[i]),
                l3fea, 1.0, L.EPI_LRELU)
        # ---- L1
        o1 = buf(0)
        conv([dict(layer=L_(u, "L1_offset_conv1"), in0=u[2][0], in1=u[3][0], out=o1[i]) for i, u in E(units)],
             epi=L.EPI_LRELU, in1_mode=1)
        o2 = buf(0)
        conv_up(lambda i, u, c: dict(layer=L_(u, "L1_offset_conv2"), in0=o1[i], in1=c, out=o2[i]),
                l2off, 2.0, L.EPI_LRELU)
        l1off = buf(0)
        conv([dict(layer=L_(u, "L1_offset_conv3"), in0=o2[i], out=l1off[i]) for i, u in E(units)], epi=L.EPI_LRELU)
        om = buf(0, 216)
        conv([dict(layer=LO(u, "L1_dcnpack"), in0=l1off[i], out=om[i]) for i, u in E(units)], epi=L.EPI_OFFMASK)
        d1 = buf(0)
        dcn([dict(layer=L_(u, "L1_dcnpack"), inp=u[2][0], offmask=om[i], out=d1[i]) for i, u in E(units)])
        conv_up(lambda i, u, c: dict(layer=L_(u, "L1_fea_conv"), in0=d1[i], in1=c, out=u[4]),
                l2fea, 1.0, L.EPI_NONE)

    def _bilstm(self, X):
        """BiDeformableConvLSTM.forward (:256-266) with DeformableConvLSTM.forward (:192-242) for
        both directions batched.  X: [3, B, H, W, 64] latent inputs (t-major).  Returns [3,B,H,W,64]."""
        _, B, H, Wd, _ = X.shape
        lay = self.layers
        pf = "ConvBLSTM.forward_net."
        pcds = (pf + "pcd_h.", pf + "pcd_c.")
        hs = self._empty(2, 3, B, H, Wd, 64)            # h of (direction, step)
        cs = torch.zeros(2, B, H, Wd, 64, device=self.device)
        zero = torch.zeros(B, H, Wd, 64, device=self.device)
        for t in range(3):
            xin = [X[t], X[2 - t]]                       # forward / reversed sequence
            state = [[zero if t == 0 else hs[d, t - 1] for d in range(2)], [cs[d] for d in range(2)]]
            # Easy_PCD pyramids (:148-160): groups (pcd, dir, which in {x, state})
            srcs = []
            for p in range(2):
                for d in range(2):
                    srcs.append((xin[d], pcds[p]))
                    srcs.append((state[p][d], pcds[p]))
            py2, py3 = self._pyramid(srcs)
            Y = self._empty(2, 2, 2, B, H, Wd, 64)       # (pcd, dir, align direction)
            units = []
            for p in range(2):
                for d in range(2):
                    gi = (p * 2 + d) * 2
                    f1 = [xin[d], py2[gi], py3[gi]]
                    f2 = [state[p][d], py2[gi + 1], py3[gi + 1]]
                    units.append((pcds[p] + "pcd_align.", 1, f1, f2, Y[p, d, 0]))
                    units.append((pcds[p] + "pcd_align.", 2, f2, f1, Y[p, d, 1]))
            self._pcd_align(units)
            T = self._empty(2, 2, B, H, Wd, 64)          # Easy_PCD.fusion outputs: (pcd, dir)
            ops.conv2d([dict(layer=lay[pcds[p] + "fusion"], in0=Y[p, d, 0], in1=Y[p, d, 1], out=T[p, d])
                        for p in range(2) for d in range(2)], in1_mode=1)
            # ConvLSTMCell (convlstm.py:42-58): combined = cat(x, h~); c_next = f*c~ + i*g
            ops.conv2d([dict(layer=lay[pf + "cell_list.0.conv"], in0=xin[d], in1=T[0, d], res=T[1, d],
                             out=hs[d, t], out2=cs[d]) for d in range(2)], epi=L.EPI_LSTM, in1_mode=1)
        feats = self._empty(3, B, H, Wd, 64)
        ops.conv2d([dict(layer=lay["ConvBLSTM.conv_1x1"], in0=hs[0, t], in1=hs[1, 2 - t], out=feats[t])
                    for t in range(3)], in1_mode=1)
        return feats

    def _gen_feat_core(self, fea1, fea2):
        """Everything after the per-frame features: PCD + fusion, BiConvLSTM, recon trunk."""
        B, H, Wd, _ = fea1[0].shape
        X = self._empty(3, B, H, Wd, 64)
        X[0].copy_(fea1[0])
        X[2].copy_(fea2[0])
        Y = self._empty(2, B, H, Wd, 64)
        self._pcd_align([("pcd_align.", 1, fea1, fea2, Y[0]), ("pcd_align.", 2, fea2, fea1, Y[1])])
        ops.conv2d([dict(layer=self.layers["fusion"], in0=Y[0], in1=Y[1], out=X[1])], in1_mode=1)
        feats = self._bilstm(X)
        trunk = feats.view(3 * B, H, Wd, 64)
        tmp = self._empty(3 * B, H, Wd, 64)
        for i in range(self.back_RBs):
            self._resblock(trunk, tmp, f"recon_trunk.{i}")
        return feats

    # ------------------------------------------------------------------ reference API
    def _check_input(self, x):
        if self._host is None:
            raise RuntimeError("LunaTokis: call load_state_dict first")
        x = x.to(self.device, torch.float32).contiguous()
        if x.dim() != 5 or x.shape[1] != 2 or x.shape[2] != 3:
            raise ValueError(f"x must be [B, 2, 3, H, W], got {tuple(x.shape)}")
        if x.shape[3] % 4 or x.shape[4] % 4:
            raise ValueError("H and W must be multiples of 4 (custom_video_test.py:44-48 pads to 4)")
        return x

    def gen_feat(self, x):
        """LunaTokis.gen_feat (:313-362): x [B,2,3,H,W] -> self.feat (NHWC [3,B,H,W,64] on device)."""
        x = self._check_input(x)
        self.inp = x
        B, N, C, H, Wd = x.shape
        l1, l2, l3 = self._frame_features(x.view(B * N, C, H, Wd))
        fea1 = [l1[0::2], l2[0::2], l3[0::2]]
        fea2 = [l1[1::2], l2[1::2], l3[1::2]]
        self._feat = self._gen_feat_core(fea1, fea2)
        return None

    def frame_features(self, frames):
        """Per-frame encoder (conv_first + feature_extraction + pyramid, :318-325) of frames
        [F,3,H,W] -> NHWC (L1, L2, L3); used for sliding windows and halo exchange."""
        frames = frames.to(self.device, torch.float32).contiguous()
        return self._frame_features(frames)

    def gen_feat_window(self, frames, last_frame_feats=None):
        """Sliding-window gen_feat: frames [F,3,H,W] -> latents of the F-1 adjacent pairs, with the
        per-frame encoder run once per frame (the reference harness runs it twice per inner frame,
        custom_video_test.py:81-97).  ``last_frame_feats`` = (L1, L2, L3) of the last frame computed
        elsewhere (parallel.halo_exchange); its encoder is then not recomputed here."""
        frames = frames.to(self.device, torch.float32).contiguous()
        x = torch.stack([frames[:-1], frames[1:]], dim=1).contiguous()
        self._check_input(x)
        self.inp = x
        if last_frame_feats is None:
            l1, l2, l3 = self._frame_features(frames)
        else:
            a1, a2, a3 = self._frame_features(frames[:-1].contiguous())
            l1, l2, l3 = (torch.cat([a, b.reshape(1, *a.shape[1:])]) for a, b in zip((a1, a2, a3), last_frame_feats))
        self._feat = self._gen_feat_core([l1[:-1], l2[:-1], l3[:-1]], [l1[1:], l2[1:], l3[1:]])
        return None

    @property
    def feat(self):
        """Latent video as the reference's [B, 3, 64, H, W] (a permuted view of the NHWC buffer)."""
        f = getattr(self, "_feat", None)
        return None if f is None else f.permute(1, 0, 4, 2, 3)

    @feat.setter
    def feat(self, v):
        if v is not None:
            raise AttributeError("feat is produced by gen_feat")
        self._feat = None

    def _time_vec(self, tq, B):
        if isinstance(tq, torch.Tensor):
            t = tq.detach().to(self.device, torch.float32).reshape(-1)
        else:
            t = torch.tensor([float(tq)], device=self.device, dtype=torch.float32)
        if t.numel() == 1:
            t = t.expand(B)
        if t.numel() != B:
            raise ValueError("each time query must hold 1 or B values")
        return t.contiguous()

    def _tab(self, H, Wd, HH, WW, shift=None):
        key = (H, Wd, HH, WW, shift)
        if key not in self._tables:
            self._tables[key] = ops.DecTablesDev(H, Wd, HH, WW, self.device, shift)
        return self._tables[key]

    def _projection(self, lr_image=True):
        """LR projections P1..P4 of the current latent (stage 0 of every decoder variant)."""
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        feats, x = self._feat, self.inp
        _, B, H, Wd, _ = feats.shape
        src = self._empty(B, H, Wd, 200)
        ops.dec_pack_lr(feats[0], feats[1], feats[2], x, src)
        proj = self._empty(B, H, Wd, 256)
        ops.conv2d([dict(layer=self.layers["dec.proj" if lr_image else "dec.proj_hrimg"], in0=src, out=proj)])
        return proj

    def _decode(self, proj, times, HH, WW, tab, image=None):
        B = proj.shape[0]
        mlp = self.layers["dec.mlp"]
        preds = []
        hrf = self._empty(B, HH, WW, 64)
        flow = self._empty(B, HH, WW, 4)
        for tq in times:
            t = self._time_vec(tq, B)
            ops.dec_stage1(proj, mlp, tab, t, hrf, flow, image, flags=self._dec_flags)
            out = self._empty(B, 3, HH, WW)
            ops.dec_stage2(proj, mlp, hrf, flow, tab, t, out, image, flags=self._dec_flags)
            preds.append(out)
        return preds

    def decoding(self, times=None, scale=None):
        """LunaTokis.decoding (:364-459): list over times of [B,3,HH,WW] (unclamped)."""
        if times is None:
            raise ValueError("times must be a list of query times")
        proj = self._projection()
        _, H, Wd, _ = proj.shape
        HH, WW = (H * 4, Wd * 4) if scale is None else (int(scale[0]), int(scale[1]))
        return self._decode(proj, times, HH, WW, self._tab(H, Wd, HH, WW))

    def decoding_test(self, times=None, scale=None):
        """LunaTokis.decoding_test (:461-598), what forward(test=True) returns: the flow and encode
        stages sample HRinp = F.upsample(inp, x4, bilinear) instead of the LR frames; HH = H * scale
        (integer scale, default 4).  The reference's q/3 chunking only bounds its memory."""
        if times is None:
            raise ValueError("times must be a list of query times")
        if "dec.proj_hrimg" not in self.layers:
            self._pack_proj(lr_image=False)
        proj = self._projection(lr_image=False)
        _, H, Wd, _ = proj.shape
        s = 4 if scale is None else int(scale)
        HH, WW = H * s, Wd * s
        image = ops.DecImageDev(self.inp, 4, HH, WW)
        return self._decode(proj, times, HH, WW, self._tab(H, Wd, HH, WW), image)

    def decoding_fasttest(self, times=None, scale=None):
        """LunaTokis.decoding_fasttest (:863-960): `times` is a list of floats, the latent a batch of
        one; all times come back as one batch [len(times), 3, HH, WW]."""
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        if self._feat.shape[1] != 1:
            raise ValueError("decoding_fasttest batches the query times: the latent must have batch 1")
        tq = [torch.tensor([[float(t)]]) for t in times]
        return torch.cat(self.decoding(tq, scale), 0)

    def decoding_localensemble(self, times=None, scale=None):
        """LunaTokis.decoding_localensemble (:962-1085): four decodes with the query shifted by
        (+-1/H, +-1/W), blended per HR pixel by the diagonally opposite |rel_y rel_x| area; batch-1
        latent, `times` a list of floats -> [len(times), 3, HH, WW]."""
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        if self._feat.shape[1] != 1:
            raise ValueError("decoding_localensemble batches the query times: the latent must have batch 1")
        proj = self._projection()
        _, H, Wd, _ = proj.shape
        HH, WW = (H * 4, Wd * 4) if scale is None else (int(scale[0]), int(scale[1]))
        key = ("ens", H, Wd, HH, WW)
        if key not in self._tables:
            self._tables[key] = [torch.from_numpy(a).to(self.device) for a in ensemble_weights(H, Wd, HH, WW)]
        wts = self._tables[key]
        tq = [torch.tensor([[float(t)]]) for t in times]
        outs = []
        decs = [torch.cat(self._decode(proj, tq, HH, WW, self._tab(H, Wd, HH, WW, (vx, vy))), 0)
                for vx in (-1, 1) for vy in (-1, 1)]
        out = self._empty(len(times), 3, HH, WW)
        ops.dec_blend4(decs, wts, out)
        return out

    def forward(self, x, times=None, scale=None, test=False, center=None, index=0):
        """LunaTokis.forward (:1222-1231): decoding, or decoding_test with test=True."""
        self.gen_feat(x)
        if test:
            return self.decoding_test(times, scale)
        return self.decoding(times, scale)
