"""LunaTokis host: the reference model API driving the gfx950 kernels.

Mirrors ``codes/models/modules/Sakuya_arch_test.py:LunaTokis`` -- constructor
``LunaTokis(nf, nframes, groups, front_RBs, back_RBs)`` (:268-311),
``forward(x, times, scale=None, test=False)`` (:1222-1231), ``gen_feat`` (:313-362),
``decoding`` (:364-459), ``load_state_dict(sd, strict=True)`` over the reference's
442 keys -- as an ``nn.Module`` whose parameters are those 442 tensors, but every layer
runs through libstif_hip.so on repacked copies (see ops.py); no torch.nn layer is on
the path.

Work is batched across everything the reference runs sequentially but that is
independent: both PCD_Align directions (different weights -> launch groups), both
ConvLSTM directions (BiDeformableConvLSTM runs the same net on x and reversed x,
:256-266), pcd_h and pcd_c, all pairs of a window, and all three latent steps of
the reconstruction trunk.  Per-frame encoder features are computed once per frame
(a sliding window shares each inner frame between two pairs).
"""
from __future__ import annotations

import contextlib
import math
import warnings
import threading
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from . import _lib as L
from . import ops
from . import weights as W
from .coords import ensemble_weights

_CONST_LOCK = threading.Lock()   # _const's dict is shared by DataParallel replicas (replicate() threads)


def _np(v):
    if isinstance(v, np.ndarray):
        return v.astype(np.float32, copy=False)
    return v.detach().cpu().numpy().astype(np.float32, copy=False)


def _drain(gen):
    """Run a stage generator (see LunaTokis._run_lanes) to completion; returns its return value."""
    while True:
        try:
            next(gen)
        except StopIteration as e:
            return e.value


class _Container(nn.Module):
    """A plain node of the reference's module tree (holds the reference parameters by their key)."""


class LunaTokis(nn.Module):
    """STIF LunaTokis (Sakuya_arch_test.py:268) on MI355X.

    An ``nn.Module`` whose parameters are exactly the reference's 442 state-dict tensors (same keys,
    shapes and registration order; ``requires_grad=False``: inference engine), so ``state_dict``,
    ``load_state_dict``, ``.to()`` / ``.cuda()`` and ``nn.DataParallel`` (VideoSR_base_model.py:29-32)
    behave as on the reference module.  The kernels read repacked copies of those weights
    (non-persistent buffers under ``_pk``, derived at ``load_state_dict``; they move and replicate with
    the module), never the parameters themselves."""

    def __init__(self, nf=64, nframes=3, groups=8, front_RBs=5, back_RBs=10, device="cuda", winograd=True,
                 mfma="f16x3", range_check="rerun", chunk_px=2 ** 21, lanes=1, dec_chunk_px=2 ** 25,
                 fused_dcn=True, trunk_lanes=2, dec_lanes=None, lstm_lanes=1, pcd_streams=1, const_shapes=2):
        super().__init__()
        if nf != 64 or groups != 8:
            raise ValueError("the gfx950 kernels implement nf=64, groups=8 (the shipped STIF configuration)")
        self.nf, self.groups = nf, groups
        self.in_frames = 1 + nframes // 2        # unused attributes kept for API parity (:272-273)
        self.ot_frames = nframes
        self.front_RBs, self.back_RBs = front_RBs, back_RBs
        self._spec = W.state_dict_spec(nf, front_RBs, back_RBs, groups)
        dev = torch.device(device)
        # the reference module tree: one parameter per state-dict key, registered in key order
        for key, shape in self._spec.items():
            *path, leaf = key.split(".")
            node = self
            for name in path:
                if name not in node._modules:
                    node.add_module(name, _Container())
                node = node._modules[name]
            node.register_parameter(leaf, nn.Parameter(torch.zeros(shape, device=dev), requires_grad=False))
        self._pk = _Container()                   # packed kernel weights (non-persistent buffers)
        self._meta = {}                           # layer name -> (buffer index, cout, cin, ks, mode)
        self._meta32 = None                       # fp32 re-packing of the f16x3 layers (range fallback)
        self.register_buffer("_range_status", torch.zeros(1, dtype=torch.int32, device=dev), persistent=False)
        self._host = None
        self._layers_key = None
        self.layers = {}
        self._feat = None
        self.inp = None
        self._tables = {}
        self.training = False
        # 3x3 convs by Winograd F(2x2,3x3) where the shape allows (fp32 throughout); False = direct
        self.winograd = bool(winograd)
        # operand arithmetic: "f32" (fp32 MFMA) or "f16x3" (fp32 products from three fp16 MFMAs on split
        # operands, ~22-bit operands, fp32 accumulation; stif.h)
        if mfma not in ("f32", "f16x3"):
            raise ValueError("mfma must be 'f32' or 'f16x3'")
        self.mfma = mfma
        # f16x3: DCN_sep as one kernel (offset/mask conv + sigmoid + deformable conv, k_dcn_sep); False =
        # the offset/mask conv (k_wino_om) and the deformable conv (k_dcn) as two launches
        self.fused_dcn = bool(fused_dcn)
        self._dec_flags = L.CONV_F16X3 if mfma == "f16x3" else 0   # decoder SIREN layers likewise
        # f16x3 activations outside the split range: "rerun" the call in fp32 (warning), "raise", or "off"
        if range_check not in ("rerun", "raise", "off"):
            raise ValueError("range_check must be 'rerun', 'raise' or 'off'")
        self.range_check = range_check
        self.range_reruns = 0
        # pairs per encoder pass: a window is processed in chunks of about chunk_px LR pixels, which
        # bounds the PCD / BiConvLSTM working set (~20 KB per pair-pixel) at large frames
        self.chunk_px = int(chunk_px)
        # HR pixels per decoder pass (decoding): bounds the decoder's scratch (~9 GB at the default)
        self.dec_chunk_px = int(dec_chunk_px)
        # independent pair ranges run as `lanes` concurrent HIP streams (_run_lanes), so one lane's kernels
        # could fill the others' tail waves and dispatch gaps; results do not depend on it.  Default 1:
        # at C0, 2 lanes measured 5 % slower (82.5 -> 76.7, 84.6 -> 80.4 Mpix/s, same box) -- the
        # persistent, XCD-mapped kernels lose more to sharing the CUs than the gaps cost
        if int(lanes) < 1:
            raise ValueError("lanes must be >= 1")
        self.lanes = int(lanes)
        # the recon trunk's items (3 latents per pair, independent chains of 80 convs) split over
        # `trunk_lanes` streams, block by block round-robin, so one half's tail waves overlap the other's.
        # At C0 (18 items = 2,304 tiles = 4.5 per persistent workgroup) 2 streams measured -0.1 to -0.5 ms
        # per step against 1, 3 streams +0.2 ms; splitting the 7-frame feature_extraction stack the same
        # way measured slower (profiles/r05_trunk_lanes_ab.log)
        if int(trunk_lanes) < 1:
            raise ValueError("trunk_lanes must be >= 1")
        self.trunk_lanes = int(trunk_lanes)
        # the BiConvLSTM's two directions on two streams (lstm_lanes=2): bit-identical, but measured
        # +0.9 ms per C0 step (17.2 vs 16.3 ms, profiles/r05_trunk_lanes_ab.log) -- half-size PCD launches
        # of two chains competing for the CUs; default 1
        if int(lstm_lanes) not in (1, 2):
            raise ValueError("lstm_lanes must be 1 or 2")
        self.lstm_lanes = int(lstm_lanes)
        # PCD alignment: the DCN / feature branch on a second stream (_pcd_align); bit-identical, measured
        # equal to one stream at C0 with either tile schedule (profiles/r05_dynamic_tiles_ab.log); default 1
        if int(pcd_streams) not in (1, 2):
            raise ValueError("pcd_streams must be 1 or 2")
        self.pcd_streams = int(pcd_streams)
        # decoding's pair ranges on their own streams (None: follow `lanes`)
        if dec_lanes is not None and int(dec_lanes) < 1:
            raise ValueError("dec_lanes must be >= 1")
        self.dec_lanes = None if dec_lanes is None else int(dec_lanes)
        self._lane_streams = {}
        self._active = False
        # weight-only constant maps (_const) are kept for this many (items, H, W) shapes per device
        if int(const_shapes) < 1:
            raise ValueError("const_shapes must be >= 1")
        self.const_shapes = int(const_shapes)

    # ------------------------------------------------------------------ nn.Module API
    @property
    def device(self):
        return self.conv_first.weight.device

    def train(self, mode=True):
        if mode:
            raise NotImplementedError("training (DCNv2 backward) is out of scope; inference only")
        return super().train(False)

    def to(self, *args, **kwargs):
        device, dtype, _, _ = torch._C._nn._parse_to(*args, **kwargs)
        if dtype is not None and dtype != torch.float32:
            raise NotImplementedError("LunaTokis (stif_amd) computes in fp32 (operand modes: mfma='f32'|'f16x3')")
        out = super().to(*args, **kwargs)
        with _CONST_LOCK:   # the constant maps of the device the module left are not used again
            consts = self.__dict__.get("_consts")
            if consts:
                for g in [g for g in consts if g[0] != str(self.device)]:
                    del consts[g]
        return out

    def half(self):
        raise NotImplementedError("LunaTokis (stif_amd) computes in fp32")

    bfloat16 = double = half

    def load_state_dict(self, state_dict, strict=True, assign=False):
        """Same key contract as nn.Module.load_state_dict on the reference module; a 'module.' prefix
        (DataParallel/DDP checkpoints) is stripped as base_model.py:93-98 does.  Repacks the kernel
        weights on the parameters' device."""
        sd = OrderedDict()
        for k, v in state_dict.items():
            sd[k[7:] if k.startswith("module.") else k] = v
        missing = [k for k in self._spec if k not in sd]
        unexpected = [k for k in sd if k not in self._spec]
        if strict and (missing or unexpected):
            raise RuntimeError("Error(s) in loading state_dict for LunaTokis:\n"
                               f"\tMissing key(s): {missing}\n\tUnexpected key(s): {unexpected}")
        params = dict(self.named_parameters())
        host = OrderedDict()
        for k, shape in self._spec.items():
            if k in sd:
                a = _np(sd[k])
                if tuple(a.shape) != tuple(shape):
                    raise RuntimeError(f"size mismatch for {k}: copying a param with shape {tuple(a.shape)}, "
                                       f"the shape in current model is {tuple(shape)}")
                host[k] = np.ascontiguousarray(a)
                params[k].data.copy_(torch.from_numpy(host[k]))
            elif self._host is not None:
                host[k] = self._host[k]
            else:
                host[k] = params[k].detach().cpu().numpy().astype(np.float32)
        self._host = host
        self._pack()
        return type("IncompatibleKeys", (), {"missing_keys": missing, "unexpected_keys": unexpected})()

    # ------------------------------------------------------------------ weight packing
    def _pack(self):
        """Pack every layer for the kernels into non-persistent buffers of ``_pk`` (on the parameters'
        device).  f16x3 packings whose weights leave the split range fall back to fp32 per layer."""
        h, dev = self._host, self.device
        meta = {}
        bufs = []

        def put(name, pc, extra=None):
            meta[name] = (len(bufs), pc.cout, pc.cin, pc.ks, pc.mode) if extra is None else (len(bufs),) + extra
            bufs.append(pc.w)
            bufs.append(pc.b if pc.b is not None else torch.zeros(1, device=dev))

        def conv(name, mode=L.PACK_PLAIN):
            put(name, ops.pack_conv(h[name + ".weight"], h[name + ".bias"], mode, dev))

        # 3x3 / stride-1 / 64-cout convs run by Winograd F(2x2,3x3) (stif_conv3x3_wino; the
        # cat(., up(.)) ones on a materialised x2-upsampled second input), as do the offset/mask
        # (64 -> 216) and ConvLSTMCell (128 -> 256, gate epilogue) convs; the strided convs keep the
        # direct kernel, the 1x1 cat convs (fusion, conv_1x1) run k_conv1x1 (f16x3) or the direct
        # kernel (f32).
        f16 = L.PACK_F16X3 if self.mfma == "f16x3" else 0
        wino = (L.PACK_WINO | f16) if self.winograd else L.PACK_PLAIN

        put("conv_first", ops.PackedConv(torch.from_numpy(h["conv_first.weight"]).to(dev),
                                         torch.from_numpy(h["conv_first.bias"]).to(dev), 64, 3, 3, L.PACK_PLAIN))
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
                        om = n + ".conv_offset_mask"
                        if f16 and self.fused_dcn:
                            # the fused DCN_sep kernel (k_dcn_sep); out of the split range -> the two-kernel path
                            try:
                                pom = ops.pack_conv(h[om + ".weight"], h[om + ".bias"], L.PACK_DCNSEP | L.PACK_F16X3,
                                                    dev, range_fallback=False)
                                pcore = ops.pack_conv(h[n + ".weight"], h[n + ".bias"], L.PACK_DCNPAIR | L.PACK_F16X3,
                                                      dev, range_fallback=False)
                                put(n, pcore)
                                put(om, pom)
                                continue
                            except L.StifError as e:
                                if e.code != L.E_RANGE:
                                    raise
                        conv(n, L.PACK_PLAIN | f16)     # the DCN core (k_dcn)
                        conv(om, (L.PACK_WINO_OFFMASK | f16) if self.winograd else L.PACK_OFFMASK)
                    else:
                        conv(n, wino)

        pcd("pcd_align.")
        conv("fusion", L.PACK_PLAIN | f16)
        conv("ConvBLSTM.forward_net.cell_list.0.conv", (L.PACK_WINO_LSTM | f16) if self.winograd else L.PACK_LSTM)
        for p in ("ConvBLSTM.forward_net.pcd_h.", "ConvBLSTM.forward_net.pcd_c."):
            for n in ("fea_L2_conv1", "fea_L3_conv1"):
                conv(p + n, L.PACK_PLAIN | f16)
            conv(p + "fusion", L.PACK_PLAIN | f16)
            for n in ("fea_L2_conv2", "fea_L3_conv2"):
                conv(p + n, wino)
            pcd(p + "pcd_align.")
        conv("ConvBLSTM.conv_1x1", L.PACK_PLAIN | f16)
        for i in range(self.back_RBs):
            conv(f"recon_trunk.{i}.conv1", wino)
            conv(f"recon_trunk.{i}.conv2", wino)
        # decoder: the SIREN MLPs, then the LR projections (their sine-layer scale follows the MLP's
        # operand mode: omega_0 / (2 pi) -- revolutions -- with f16x3, stif.h STIF_DEC_REVOLUTIONS)
        mlp, flags = self._pack_mlp(self._dec_flags)
        self._dec_flags = flags
        for lr_image in (True, False):
            put("dec.proj" if lr_image else "dec.proj_hrimg", self._pack_proj(lr_image, bool(flags & L.CONV_F16X3)))
        meta["dec.mlp"] = (len(bufs), flags)
        bufs.append(mlp)
        bufs.append(torch.zeros(1, device=dev))
        self._pk = _Container()
        for i, b in enumerate(bufs):
            self._pk.register_buffer(f"b{i}", b, persistent=False)
        self._meta = meta
        self._meta32 = None
        self._layers_key = None
        self._tables = {}
        self._consts = OrderedDict()

    def _pack_mlp(self, flags):
        """All SIREN layers (stif_pack_dec_mlp_ex); an out-of-range weight for f16x3 -> fp32 packing."""
        h, lib = self._host, L.lib()

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
        try:
            L.check(lib.stif_pack_dec_mlp_ex(fp, lp, ep, mlp.ctypes.data, flags), "stif_pack_dec_mlp_ex")
        except L.StifError as e:
            if e.code != L.E_RANGE or not flags:
                raise
            flags = 0
            L.check(lib.stif_pack_dec_mlp_ex(fp, lp, ep, mlp.ctypes.data, 0), "stif_pack_dec_mlp_ex")
        return torch.from_numpy(mlp).to(self.device), flags

    def _pack_proj(self, lr_image=True, revolutions=False):
        """LR projection of the decoder's first layers (stif_pack_dec_proj_ex); lr_image=False leaves
        the LR frames out of P2..P4 for decoding_test, which samples the x4-upsampled frames;
        revolutions: sine-layer scale omega_0 / (2 pi), matching an f16x3-packed MLP."""
        h, dev, lib = self._host, self.device, L.lib()

        def pack(mode):
            wd = np.empty(lib.stif_conv_weight_floats(256, 200, 1, mode), np.float32)
            bd = np.empty(lib.stif_conv_bias_floats(256, L.PACK_PLAIN), np.float32)
            L.check(lib.stif_pack_dec_proj_ex(h["feat_imnet.net.0.linear.weight"].ctypes.data,
                                              h["feat_imnet.net.0.linear.bias"].ctypes.data,
                                              h["flow_imnet.net.0.linear.weight"].ctypes.data,
                                              h["encode_imnet.net.0.linear.weight"].ctypes.data,
                                              int(lr_image) | (mode & L.PACK_F16X3) | (L.DEC_REVOLUTIONS if revolutions else 0),
                                              wd.ctypes.data, bd.ctypes.data),
                    "stif_pack_dec_proj_ex")
            return ops.PackedConv(torch.from_numpy(wd).to(dev), torch.from_numpy(bd).to(dev), 256, 200, 1, mode)

        if self.mfma == "f16x3":   # k_conv1x1; a weight outside the split range -> fp32 packing
            try:
                return pack(L.PACK_PLAIN | L.PACK_F16X3)
            except L.StifError as e:
                if e.code != L.E_RANGE:
                    raise
        return pack(L.PACK_PLAIN)

    def _build_layers(self, pk, meta):
        bufs = pk._buffers
        lay = {}
        for name, m in meta.items():
            w, b = bufs[f"b{m[0]}"], bufs[f"b{m[0] + 1}"]
            lay[name] = w if name == "dec.mlp" else ops.PackedConv(w, b, *m[1:])
        return lay

    def _layers_fp32(self):
        """The f16x3 layers re-packed in fp32 (range fallback), as non-persistent buffers of ``_pk32``."""
        if self._meta32 is None or self._pk32.b0.device != self.device:
            keep = (self.mfma, self._dec_flags, self._pk, self._meta)
            self.mfma, self._dec_flags = "f32", 0
            try:
                self._pack()
                self._pk32, self._meta32 = self._pk, self._meta
            finally:
                self.mfma, self._dec_flags, self._pk, self._meta = keep
                self._layers_key = None
        return self._build_layers(self._pk32, self._meta32)

    # ------------------------------------------------------------------ call wrapper
    def _call(self, fn, *args, **kwargs):
        """Run a public entry point on the module's device (its current stream), with the packed
        layers of this module (or replica).  With f16x3 operands the kernels report non-finite
        outputs in ``_range_status``; the call is then re-run in fp32 (range_check='rerun') or
        raises (range_check='raise')."""
        if self._host is None:
            raise RuntimeError("LunaTokis: call load_state_dict first")
        dev = self.device
        if dev.type != "cuda":
            raise L.StifError("LunaTokis (stif_amd) runs on the GPU only: move it with .to('cuda')")
        if self._active:                       # nested entry (e.g. decoding_fasttest -> decoding)
            return fn(*args, **kwargs)
        with torch.cuda.device(dev):
            key = self._pk.b0.data_ptr()
            if self._layers_key != key:
                self.layers = self._build_layers(self._pk, self._meta)
                self._layers_key = key
            check = self.range_check != "off" and (self.mfma == "f16x3")
            # inside a hipGraph capture the status word is still zeroed and written by the captured
            # kernels, but read by the caller after each replay (tools/graph_step.py), not here
            capturing = torch.cuda.is_current_stream_capturing()
            self._active = True
            try:
                if check:
                    self._range_status.zero_()
                out = fn(*args, **kwargs)
                if check and not capturing and int(self._range_status.item()):
                    if self.range_check == "raise":
                        raise L.StifError("f16x3 operand outside the split-fp16 range (|activation| >= 1024): "
                                          "use LunaTokis(mfma='f32') or range_check='rerun'", L.E_RANGE)
                    warnings.warn("LunaTokis: an f16x3 operand left the split-fp16 range; re-running this call "
                                  "with fp32 MFMA operands", RuntimeWarning, stacklevel=3)
                    self.range_reruns += 1
                    keep = (self.layers, self._dec_flags, self._layers_key)
                    self.layers, self._dec_flags = self._layers_fp32(), 0
                    try:
                        out = fn(*args, **kwargs)
                    finally:
                        self.layers, self._dec_flags, self._layers_key = keep
            finally:
                self._active = False
        return out

    @property
    def _status(self):
        return self._range_status if self.range_check != "off" else None

    # ------------------------------------------------------------------ encoder pieces
    def _conv(self, groups, **kw):
        ops.conv2d(groups, status=self._status, **kw)

    def _dcn(self, groups, **kw):
        ops.dcn(groups, status=self._status, **kw)

    def _dcn_sep(self, items, epi=L.EPI_NONE):
        """DCN_sep.forward (dcn_v2.py:127-140) for a launch group of items (layer name, fea, inp, out):
        the fused kernel where both layers are packed for it, else conv_offset_mask (OFFMASK epilogue)
        into a 216-channel map and the deformable conv."""
        lay = self.layers
        fused = [it for it in items if ops.dcn_sep_fusable(lay[it[0] + ".conv_offset_mask"], lay[it[0]])]
        rest = [it for it in items if not ops.dcn_sep_fusable(lay[it[0] + ".conv_offset_mask"], lay[it[0]])]
        if fused:
            ops.dcn_sep([dict(om_layer=lay[n + ".conv_offset_mask"], layer=lay[n], fea=f, inp=x, out=o)
                         for n, f, x, o in fused], epi=epi, status=self._status)
        if rest:
            n0, f0 = rest[0][0], rest[0][1]
            om = self._empty(len(rest), *f0.shape[:3], 216)
            self._conv([dict(layer=lay[n + ".conv_offset_mask"], in0=f, out=om[i]) for i, (n, f, x, o) in enumerate(rest)],
                       epi=L.EPI_OFFMASK)
            self._dcn([dict(layer=lay[n], inp=x, offmask=om[i], out=o) for i, (n, f, x, o) in enumerate(rest)], epi=epi)

    def _empty(self, *shape):
        return torch.empty(*shape, device=self.device, dtype=torch.float32)

    def _const(self, key, shape, make):
        """Maps that depend only on the packed weights and a shape (the all-zero initial state, its
        pyramids, the zero-state L1 DCN output), computed on first use and kept until the layers are
        re-packed.  Entries are grouped by (device, shape): the key holds the weight buffers' addresses
        (so the fp32 range re-run's layers get their own entries) and the device is part of every
        group, so DataParallel replicas -- which share this dict through replicate()'s shallow
        __dict__ copy -- and a module moved by .to() never receive another device's tensors.  At most
        ``const_shapes`` groups per device are kept (least recently used evicted): one C0 group is
        ~0.1 GB, a 720p / 1080p group ~1.7 / 2 GB, so a serving process that sees many resolutions
        holds at most two of them.  Not cached inside a hipGraph capture (computed in the graph)."""
        if self.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            return make()
        dev = str(self.device)
        grp = (dev,) + tuple(int(s) for s in shape)
        with _CONST_LOCK:
            consts = self.__dict__.get("_consts")
            if not isinstance(consts, OrderedDict):
                consts = self.__dict__["_consts"] = OrderedDict()
            ent = consts.get(grp)
            if ent is not None and key in ent:
                consts.move_to_end(grp)
                return ent[key]
        v = make()
        if self.device.type == "cuda":   # once: other streams (lanes) read it without an event
            torch.cuda.current_stream(self.device).synchronize()
        with _CONST_LOCK:
            consts.setdefault(grp, {})[key] = v
            consts.move_to_end(grp)
            mine = [g for g in consts if g[0] == dev]
            for g in mine[:max(0, len(mine) - max(1, self.const_shapes))]:
                del consts[g]
        return v

    def _zeros(self, *shape):
        # grouped with the other maps of the same (items, H, W)
        return self._const(("zeros",) + tuple(shape), shape[:3],
                           lambda: torch.zeros(*shape, device=self.device, dtype=torch.float32))

    def _frame_features(self, frames):
        """conv_first + feature_extraction + pyramid (:318-325) for frames [n,3,H,W] (NCHW)."""
        return _drain(self._frame_features_steps(frames))

    def _frame_features_steps(self, frames):
        n, _, H, Wd = frames.shape
        l1 = self._empty(n, H, Wd, 64)
        ops.conv_first(frames, self.layers["conv_first"].w, self.layers["conv_first"].b, l1)
        tmp = self._empty(n, H, Wd, 64)
        yield from self._resblocks(l1, tmp, [f"feature_extraction.{i}" for i in range(self.front_RBs)])
        l2, l3 = self._pyramid([(l1, "")])
        return l1, l2[0], l3[0]

    # ------------------------------------------------------------------ lanes
    def _streams(self, k, pool="lanes"):
        dev = self.device
        ss = self._lane_streams.setdefault((pool, str(dev)), [])
        while len(ss) < k:
            ss.append(torch.cuda.Stream(device=dev))
        return ss[:k]

    def _run_lanes(self, n, make, lanes=None, pool="lanes"):
        """Items [0, n) in up to ``self.lanes`` contiguous ranges; ``make(c0, c1)`` is a generator
        issuing one range's launches (each ``yield`` a point where another lane may issue).  Each
        range runs on its own stream, forked from and joined back into the current one, and the
        generators advance round-robin, so every stream has queued work from the start and the
        kernels of one lane fill the last waves and the dispatch gaps of the others.  Every kernel
        computes each item independently of the batch it is launched in, so the results are
        bit-identical for any lane count."""
        k = max(1, min(self.lanes if lanes is None else lanes, n))
        per = -(-n // k)
        ranges = [(c0, min(n, c0 + per)) for c0 in range(0, n, per)]
        if len(ranges) == 1:
            _drain(make(0, n))
            return
        main = torch.cuda.current_stream()
        streams = self._streams(len(ranges), pool)
        for s in streams:
            s.wait_stream(main)
        live = [(s, make(c0, c1)) for s, (c0, c1) in zip(streams, ranges)]
        while live:
            nxt = []
            for s, g in live:
                with torch.cuda.stream(s):
                    try:
                        next(g)
                        nxt.append((s, g))
                    except StopIteration:
                        pass
            live = nxt
        for s in streams:
            main.wait_stream(s)

    def _resblocks(self, x, tmp, names, lanes=1):
        """A stack of ResidualBlock_noBN on x [n, H, W, 64] in place (generator, one yield per block).
        The items are independent chains, so with ``lanes`` > 1 they are split into that many
        contiguous ranges on their own streams, issued block by block round-robin: one range's tail
        waves and dispatch gaps overlap the other's work.  Bit-identical for any split."""
        n = x.shape[0]
        k = max(1, min(lanes, n))
        if k == 1:
            for name in names:
                self._resblock(x, tmp, name)
                yield
            return
        per = -(-n // k)
        ranges = [(c0, min(n, c0 + per)) for c0 in range(0, n, per)]
        main = torch.cuda.current_stream()
        ss = self._streams(len(ranges), pool="trunk")
        for s in ss:
            s.wait_stream(main)
        for name in names:
            for s, (c0, c1) in zip(ss, ranges):
                with torch.cuda.stream(s):
                    self._resblock(x[c0:c1], tmp[c0:c1], name)
            yield
        for s in ss:
            main.wait_stream(s)

    def _resblock(self, x, tmp, name):
        """ResidualBlock_noBN (module_util.py:48-52), x updated in place."""
        self._conv([dict(layer=self.layers[name + ".conv1"], in0=x, out=tmp)], epi=L.EPI_RELU)
        self._conv([dict(layer=self.layers[name + ".conv2"], in0=tmp, out=x, res=x)], epi=L.EPI_RES)

    def _pyramid(self, srcs):
        """fea_L2_conv1/2, fea_L3_conv1/2 with lrelu for a list of (L1 map, weight prefix)."""
        G = len(srcs)
        n, H, Wd, _ = srcs[0][0].shape
        a2 = self._empty(G, n, H // 2, Wd // 2, 64)
        b2 = self._empty(G, n, H // 2, Wd // 2, 64)
        a3 = self._empty(G, n, H // 4, Wd // 4, 64)
        b3 = self._empty(G, n, H // 4, Wd // 4, 64)
        lay = self.layers
        self._conv([dict(layer=lay[p + "fea_L2_conv1"], in0=s, out=a2[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU, stride=2)
        self._conv([dict(layer=lay[p + "fea_L2_conv2"], in0=a2[i], out=b2[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU)
        self._conv([dict(layer=lay[p + "fea_L3_conv1"], in0=b2[i], out=a3[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU, stride=2)
        self._conv([dict(layer=lay[p + "fea_L3_conv2"], in0=a3[i], out=b3[i]) for i, (s, p) in enumerate(srcs)],
                   epi=L.EPI_LRELU)
        return b2, b3

    def _pcd_align(self, units, zero_l1=()):
        """PCD_Align.forward (:71-130) for up to 8 independent (module, direction) units.
        unit = (prefix, d, fa[L1,L2,L3], fb[L1,L2,L3], y_out).  ``zero_l1``: indices of units whose
        fa L1 map is all zeros (the ConvLSTM's initial state, convlstm.py:60-63, sampled by the
        reversed-direction alignment of the first step): their L1 DCN samples only zeros, so its output
        is its bias wherever the offsets land (DCN_sep, dcn_v2.py:127-140: sum of 0 * w + b), and the
        L1 offset branch that only steers it (L1_offset_conv1..3, conv_offset_mask) is not run for
        them -- bit-identical to running it (for finite offsets)."""
        G = len(units)
        n, H, Wd, _ = units[0][2][0].shape
        lay = self.layers
        lv = [(H, Wd), (H // 2, Wd // 2), (H // 4, Wd // 4)]

        def buf(level, c=64):
            h_, w_ = lv[level]
            return self._empty(G, n, h_, w_, c)

        def L_(u, name):
            return lay[f"{u[0]}{name}_{u[1]}"]

        conv = self._conv
        E = enumerate
        # pcd_streams = 2: the DCN / feature branch (L3 DCN; L2 DCN + fea conv; L1 DCN + fea conv) on a
        # side stream, each part forked when its offsets are ready, so it overlaps the offset convs of the
        # next level (which depend on the offsets only) -- the under-filled L3 launches and the tails of
        # every launch get work beside them
        main = torch.cuda.current_stream()
        side = self._streams(1, pool="pcd")[0] if self.pcd_streams > 1 else None

        def branch():
            if side is None:
                return contextlib.nullcontext()
            side.wait_stream(main)
            return torch.cuda.stream(side)

        def conv_up(make, coarse, scale, epi):
            """conv on cat(x, scale * up2(coarse)) for every unit, the x2 upsample fused into the
            conv's staging (Winograd: expanded from an LDS-staged coarse patch per tile; direct
            kernel: register-staged) -- the upsampled map never reaches HBM"""
            conv([make(i, u, coarse[i]) for i, u in E(units)], epi=epi, in1_mode=2, in1_scale=scale)
        # ---- L3
        o = buf(2)
        conv([dict(layer=L_(u, "L3_offset_conv1"), in0=u[2][2], in1=u[3][2], out=o[i]) for i, u in E(units)],
             epi=L.EPI_LRELU, in1_mode=1)
        l3off = buf(2)
        conv([dict(layer=L_(u, "L3_offset_conv2"), in0=o[i], out=l3off[i]) for i, u in E(units)], epi=L.EPI_LRELU)
        l3fea = buf(2)
        with branch():
            self._dcn_sep([(f"{u[0]}L3_dcnpack_{u[1]}", l3off[i], u[2][2], l3fea[i]) for i, u in E(units)],
                          L.EPI_LRELU)
        # ---- L2
        o1 = buf(1)
        conv([dict(layer=L_(u, "L2_offset_conv1"), in0=u[2][1], in1=u[3][1], out=o1[i]) for i, u in E(units)],
             epi=L.EPI_LRELU, in1_mode=1)
        o2 = buf(1)
        conv_up(lambda i, u, c: dict(layer=L_(u, "L2_offset_conv2"), in0=o1[i], in1=c, out=o2[i]),
                l3off, 2.0, L.EPI_LRELU)
        l2off = buf(1)
        conv([dict(layer=L_(u, "L2_offset_conv3"), in0=o2[i], out=l2off[i]) for i, u in E(units)], epi=L.EPI_LRELU)
        d2 = buf(1)
        l2fea = buf(1)
        with branch():
            self._dcn_sep([(f"{u[0]}L2_dcnpack_{u[1]}", l2off[i], u[2][1], d2[i]) for i, u in E(units)])
            conv_up(lambda i, u, c: dict(layer=L_(u, "L2_fea_conv"), in0=d2[i], in1=c, out=l2fea[i]),
                    l3fea, 1.0, L.EPI_LRELU)
        # ---- L1 (offset branch and DCN for the units whose fa L1 is not all zeros; k = their index)
        live = [(i, u) for i, u in E(units) if i not in zero_l1]
        d1 = buf(0)
        if live:
            o1 = self._empty(len(live), n, H, Wd, 64)
            conv([dict(layer=L_(u, "L1_offset_conv1"), in0=u[2][0], in1=u[3][0], out=o1[k])
                  for k, (i, u) in E(live)], epi=L.EPI_LRELU, in1_mode=1)
            o2 = self._empty(len(live), n, H, Wd, 64)
            conv([dict(layer=L_(u, "L1_offset_conv2"), in0=o1[k], in1=l2off[i], out=o2[k]) for k, (i, u) in E(live)],
                 epi=L.EPI_LRELU, in1_mode=2, in1_scale=2.0)
            l1off = self._empty(len(live), n, H, Wd, 64)
            conv([dict(layer=L_(u, "L1_offset_conv3"), in0=o2[k], out=l1off[k]) for k, (i, u) in E(live)],
                 epi=L.EPI_LRELU)
            del o1, o2
            with branch():
                self._dcn_sep([(f"{u[0]}L1_dcnpack_{u[1]}", l1off[k], u[2][0], d1[i]) for k, (i, u) in E(live)])
        # the zero-state units' L1 DCN output is its bias everywhere: a constant map, kept across calls
        d1z = {}
        for i in zero_l1:
            b = L_(units[i], "L1_dcnpack").b
            d1z[i] = self._const(("dcn_bias", b.data_ptr()), (n, H, Wd), lambda b=b: b.view(1, 1, 1, 64).expand(
                n, H, Wd, 64).contiguous())
        with branch():
            conv_up(lambda i, u, c: dict(layer=L_(u, "L1_fea_conv"), in0=d1z.get(i, d1[i]), in1=c, out=u[4]),
                    l2fea, 1.0, L.EPI_NONE)
        if side is not None:
            main.wait_stream(side)   # before any buffer of this call can be freed and reused on main

    def _bilstm(self, X):
        return _drain(self._bilstm_steps([X[0], X[1], X[2]]))

    def _bilstm_steps(self, X, feats=None):
        """BiDeformableConvLSTM.forward (:256-266) with DeformableConvLSTM.forward (:192-242) for
        both directions batched.  X: the 3 latent inputs [B, H, W, 64] (t-major; views with one common
        item stride).  Returns [3,B,H,W,64] (in ``feats`` when given)."""
        B, H, Wd, _ = X[0].shape
        lay = self.layers
        pf = "ConvBLSTM.forward_net."
        pcds = (pf + "pcd_h.", pf + "pcd_c.")
        hs = self._empty(2, 3, B, H, Wd, 64)            # h of (direction, step)
        cs = self._empty(2, B, H, Wd, 64)               # c of the last step (step 0 reads the zero state)
        zero = self._zeros(B, H, Wd, 64)                # the initial h and c (convlstm.py:60-63), never written
        # Easy_PCD pyramids (:148-160) of the inputs, once per (pcd, input): the forward direction reads
        # X[t] and the reversed one X[2 - t] with the same weights, so per-step pyramids of the inputs
        # would compute each of them twice (bit-identical results, half the work); groups (pcd, t)
        xp2, xp3 = self._pyramid([(X[t], pcds[p]) for p in range(2) for t in range(3)])

        def xpyr(p, level, fr):
            return (xp2 if level == 2 else xp3)[p * 3 + fr]

        # the step-0 state pyramids (zeros) once per pcd, depending on the weights only: kept across calls
        zkey = ("zero_pyr", lay[pcds[0] + "fea_L2_conv1"].w.data_ptr())
        z2, z3 = self._const(zkey, (B, H, Wd), lambda: self._pyramid([(zero, pcds[p]) for p in range(2)]))

        def step(t, ds):
            """Step t of the directions ds (0 forward, 1 reversed): state pyramids, PCD alignments,
            Easy_PCD fusion and the ConvLSTM cell, each one launch over (pcd, direction) groups."""
            fr = [t, 2 - t]                               # forward / reversed sequence
            xin = [X[f] for f in fr]
            pd = [(p, d) for p in range(2) for d in ds]
            st = {(p, d): zero if t == 0 else (hs[d, t - 1] if p == 0 else cs[d]) for p, d in pd}
            if t == 0:
                pyr = {(p, d): (z2[p], z3[p]) for p, d in pd}
            else:
                a2, a3 = self._pyramid([(st[p, d], pcds[p]) for p, d in pd])
                pyr = {k: (a2[i], a3[i]) for i, k in enumerate(pd)}
            nd = len(ds)
            Y = self._empty(2, nd, 2, B, H, Wd, 64)      # (pcd, dir, align direction)
            units = []
            for p in range(2):
                for j, d in enumerate(ds):
                    f1 = [xin[d], xpyr(p, 2, fr[d]), xpyr(p, 3, fr[d])]
                    f2 = [st[p, d], *pyr[p, d]]
                    units.append((pcds[p] + "pcd_align.", 1, f1, f2, Y[p, j, 0]))
                    units.append((pcds[p] + "pcd_align.", 2, f2, f1, Y[p, j, 1]))
            # step 0: the reversed alignments (odd units) sample the all-zero initial state at L1
            self._pcd_align(units, zero_l1=range(1, len(units), 2) if t == 0 else ())
            T = self._empty(2, nd, B, H, Wd, 64)         # Easy_PCD.fusion outputs: (pcd, dir)
            self._conv([dict(layer=lay[pcds[p] + "fusion"], in0=Y[p, j, 0], in1=Y[p, j, 1], out=T[p, j])
                        for p in range(2) for j in range(nd)], in1_mode=1)
            # ConvLSTMCell (convlstm.py:42-58): combined = cat(x, h~); c_next = f*c~ + i*g
            self._conv([dict(layer=lay[pf + "cell_list.0.conv"], in0=xin[d], in1=T[0, j], res=T[1, j],
                             out=hs[d, t], out2=cs[d]) for j, d in enumerate(ds)], epi=L.EPI_LSTM, in1_mode=1)

        if self.lstm_lanes < 2:
            for t in range(3):
                step(t, (0, 1))
                yield
        else:
            # the two directions are independent recurrences: one stream each, step by step round-robin
            main = torch.cuda.current_stream()
            ss = self._streams(2, pool="lstm")
            for s in ss:
                s.wait_stream(main)
            for t in range(3):
                for s, d in zip(ss, (0, 1)):
                    with torch.cuda.stream(s):
                        step(t, (d,))
                yield
            for s in ss:
                main.wait_stream(s)
        if feats is None:
            feats = self._empty(3, B, H, Wd, 64)
        self._conv([dict(layer=lay["ConvBLSTM.conv_1x1"], in0=hs[0, t], in1=hs[1, 2 - t], out=feats[t])
                    for t in range(3)], in1_mode=1)
        return feats

    def _gen_feat_core(self, fea1, fea2, out):
        """Everything after the per-frame features: PCD + fusion, BiConvLSTM, recon trunk, into
        out [3, B, H, W, 64] (generator: yields between stages, see _run_lanes).
        fea1 / fea2: [L1, L2, L3] of the pairs' first / second frames (item = pair)."""
        B, H, Wd, _ = fea1[0].shape
        X1 = self._empty(B, H, Wd, 64)                  # the fused middle latent input
        Y = self._empty(2, B, H, Wd, 64)
        self._pcd_align([("pcd_align.", 1, fea1, fea2, Y[0]), ("pcd_align.", 2, fea2, fea1, Y[1])])
        self._conv([dict(layer=self.layers["fusion"], in0=Y[0], in1=Y[1], out=X1)], in1_mode=1)
        del Y
        yield
        # the inputs X = [fea1 L1, fused, fea2 L1] as views (no copies) when their item strides agree (the
        # sliding-window path: consecutive frames); the batched pyramid of the inputs needs one stride
        X = [fea1[0], X1, fea2[0]]
        if not all(x.stride(0) == X1.stride(0) for x in X):   # (a [1, ...] view counts as contiguous in torch)
            X = [X1 if x is X1 else self._empty(B, H, Wd, 64).copy_(x) for x in X]
        # the latents go straight into `out` when it is one contiguous block (one chunk of pairs)
        feats = yield from self._bilstm_steps(X, out if out.is_contiguous() else None)
        del X, X1
        trunk = feats.view(3 * B, H, Wd, 64)
        tmp = self._empty(3 * B, H, Wd, 64)
        yield from self._resblocks(trunk, tmp, [f"recon_trunk.{i}" for i in range(self.back_RBs)], self.trunk_lanes)
        if feats is not out:
            out.copy_(feats)

    def _gen_feat_pairs(self, fea1, fea2, out):
        """_gen_feat_core over chunks of about ``chunk_px`` LR pixels of pairs (balanced), so the
        working set stays bounded at large frames; pairs are independent, so chunking does not
        change a bit of the result (generator)."""
        B, H, Wd, _ = fea1[0].shape
        per = max(1, self.chunk_px // (H * Wd))
        nch = math.ceil(B / per)
        per = math.ceil(B / nch)
        for c0 in range(0, B, per):
            c1 = min(B, c0 + per)
            yield from self._gen_feat_core([t[c0:c1] for t in fea1], [t[c0:c1] for t in fea2], out[:, c0:c1])

    # ------------------------------------------------------------------ reference API
    def _check_input(self, x):
        x = x.to(self.device, torch.float32).contiguous()
        if x.dim() != 5 or x.shape[1] != 2 or x.shape[2] != 3:
            raise ValueError(f"x must be [B, 2, 3, H, W], got {tuple(x.shape)}")
        if x.shape[3] % 4 or x.shape[4] % 4:
            raise ValueError("H and W must be multiples of 4 (custom_video_test.py:44-48 pads to 4)")
        return x

    def gen_feat(self, x):
        """LunaTokis.gen_feat (:313-362): x [B,2,3,H,W] -> self.feat (NHWC [3,B,H,W,64] on device)."""
        return self._call(self._gen_feat, x)

    def _gen_feat(self, x):
        x = self._check_input(x)
        self.inp = x
        B, N, C, H, Wd = x.shape
        out = self._empty(3, B, H, Wd, 64)

        def lane(c0, c1):
            l1, l2, l3 = yield from self._frame_features_steps(x[c0:c1].reshape((c1 - c0) * N, C, H, Wd))
            fea1 = [l1[0::2], l2[0::2], l3[0::2]]
            fea2 = [l1[1::2], l2[1::2], l3[1::2]]
            yield from self._gen_feat_pairs(fea1, fea2, out[:, c0:c1])
        self._run_lanes(B, lane)
        self._feat = out
        return None

    def frame_features(self, frames):
        """Per-frame encoder (conv_first + feature_extraction + pyramid, :318-325) of frames
        [F,3,H,W] -> NHWC (L1, L2, L3); used for sliding windows and the halo exchange."""
        return self._call(lambda f: self._frame_features(f.to(self.device, torch.float32).contiguous()), frames)

    def gen_feat_window(self, frames, last_frame_feats=None, frame_feats=None):
        """Sliding-window gen_feat: frames [F,3,H,W] -> latents of the F-1 adjacent pairs, with the
        per-frame encoder run once per frame (the reference harness runs it twice per inner frame,
        custom_video_test.py:81-97).  ``frame_feats`` = (L1, L2, L3) of all F frames computed
        beforehand (frame_features + parallel.halo_exchange); ``last_frame_feats`` = those of the
        last frame only (the others are computed here)."""
        return self._call(self._gen_feat_window, frames, last_frame_feats, frame_feats)

    def _gen_feat_window(self, frames, last_frame_feats=None, frame_feats=None):
        frames = frames.to(self.device, torch.float32).contiguous()
        x = torch.stack([frames[:-1], frames[1:]], dim=1).contiguous()
        self.inp = self._check_input(x)
        F_ = frames.shape[0]
        _, _, H, Wd = frames.shape
        out = self._empty(3, F_ - 1, H, Wd, 64)
        if frame_feats is None and last_frame_feats is None:
            # lanes of pairs [c0, c1) each run the encoder on their frames c0..c1 (the frame two lanes
            # share is encoded by both, so no lane waits for another)
            def lane(c0, c1):
                l1, l2, l3 = yield from self._frame_features_steps(frames[c0:c1 + 1])
                yield from self._gen_feat_pairs([l1[:-1], l2[:-1], l3[:-1]], [l1[1:], l2[1:], l3[1:]],
                                                out[:, c0:c1])
            self._run_lanes(F_ - 1, lane)
            self._feat = out
            return None
        if frame_feats is not None:
            l1, l2, l3 = frame_feats
            if l1.shape[0] != F_:
                raise ValueError(f"frame_feats hold {l1.shape[0]} frames, the window {F_}")
        else:
            a1, a2, a3 = self._frame_features(frames[:-1].contiguous())
            l1, l2, l3 = (torch.cat([a, b.reshape(1, *a.shape[1:]).to(a.device)])
                          for a, b in zip((a1, a2, a3), last_frame_feats))
        self._run_lanes(F_ - 1, lambda c0, c1: self._gen_feat_pairs(
            [l1[c0:c1], l2[c0:c1], l3[c0:c1]], [l1[c0 + 1:c1 + 1], l2[c0 + 1:c1 + 1], l3[c0 + 1:c1 + 1]],
            out[:, c0:c1]))
        self._feat = out
        return None

    @property
    def feat(self):
        """Latent video as the reference's [B, 3, 64, H, W] (a permuted view of the NHWC buffer)."""
        f = self.__dict__.get("_feat")
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
        key = (str(self.device), H, Wd, HH, WW, shift)
        if key not in self._tables:
            self._tables[key] = ops.DecTablesDev(H, Wd, HH, WW, self.device, shift)
        return self._tables[key]

    def _projection(self, lr_image=True, c0=0, c1=None):
        """LR projections P1..P4 of the current latent's items [c0, c1) (stage 0 of every decoder
        variant)."""
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        feats, x = self._feat, self.inp
        _, B, H, Wd, _ = feats.shape
        c1 = B if c1 is None else c1
        f, x, B = feats[:, c0:c1], x[c0:c1], c1 - c0
        src = self._empty(B, H, Wd, 200)
        ops.dec_pack_lr(f[0], f[1], f[2], x, src)
        proj = self._empty(B, H, Wd, 256)
        self._conv([dict(layer=self.layers["dec.proj" if lr_image else "dec.proj_hrimg"], in0=src, out=proj)])
        return proj

    def _decode_steps(self, proj, tvs, HH, WW, tab, outs, image=None):
        """Decoder stages 1-2 of every query time (time vectors ``tvs``) into ``outs`` (generator)."""
        B = proj.shape[0]
        mlp = self.layers["dec.mlp"]
        hrf = self._empty(B, HH, WW, 64)
        flow = self._empty(B, HH, WW, 4)
        for t, out in zip(tvs, outs):
            ops.dec_stage1(proj, mlp, tab, t, hrf, flow, image, flags=self._dec_flags, status=self._status)
            ops.dec_stage2(proj, mlp, hrf, flow, tab, t, out, image, flags=self._dec_flags, status=self._status)
            yield

    def _decode(self, proj, times, HH, WW, tab, image=None):
        B = proj.shape[0]
        outs = [self._empty(B, 3, HH, WW) for _ in times]
        _drain(self._decode_steps(proj, [self._time_vec(tq, B) for tq in times], HH, WW, tab, outs, image))
        return outs

    def decoding(self, times=None, scale=None):
        """LunaTokis.decoding (:364-459): list over times of [B,3,HH,WW] (unclamped)."""
        return self._call(self._decoding, times, scale)

    def _decoding(self, times=None, scale=None):
        if times is None:
            raise ValueError("times must be a list of query times")
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        _, B, H, Wd, _ = self._feat.shape
        HH, WW = (H * 4, Wd * 4) if scale is None else (int(scale[0]), int(scale[1]))
        tab = self._tab(H, Wd, HH, WW)
        tvs = [self._time_vec(tq, B) for tq in times]
        outs = [self._empty(B, 3, HH, WW) for _ in times]

        # items per decode pass: the LR projections (1 KB per LR pixel) and the HRfeat / flow scratch
        # (272 B per HR pixel) of at most dec_chunk_px HR pixels -- a 63-pair 720p sequence on one GPU
        # would otherwise need ~300 GB of scratch; every pixel is decoded independently, so chunking
        # does not change a bit
        per = max(1, self.dec_chunk_px // (HH * WW))

        def lane(c0, c1):
            for a in range(c0, c1, per):
                b = min(c1, a + per)
                proj = self._projection(True, a, b)
                yield
                yield from self._decode_steps(proj, [t[a:b] for t in tvs], HH, WW, tab, [o[a:b] for o in outs])
                del proj
        self._run_lanes(B, lane, self.dec_lanes, pool="dec")
        return outs

    def decoding_test(self, times=None, scale=None):
        """LunaTokis.decoding_test (:461-598), what forward(test=True) returns: the flow and encode
        stages sample HRinp = F.upsample(inp, x4, bilinear) instead of the LR frames; HH = H * scale
        (integer scale, default 4).  The reference's q/3 chunking only bounds its memory."""
        return self._call(self._decoding_test, times, scale)

    def _decoding_test(self, times=None, scale=None):
        if times is None:
            raise ValueError("times must be a list of query times")
        proj = self._projection(lr_image=False)
        _, H, Wd, _ = proj.shape
        s = 4 if scale is None else int(scale)
        HH, WW = H * s, Wd * s
        image = ops.DecImageDev(self.inp, 4, HH, WW)
        return self._decode(proj, times, HH, WW, self._tab(H, Wd, HH, WW), image)

    def decoding_fasttest(self, times=None, scale=None):
        """LunaTokis.decoding_fasttest (:863-960): `times` is a list of floats, the latent a batch of
        one; all times come back as one batch [len(times), 3, HH, WW]."""
        return self._call(self._decoding_fasttest, times, scale)

    def _decoding_fasttest(self, times=None, scale=None):
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        if self._feat.shape[1] != 1:
            raise ValueError("decoding_fasttest batches the query times: the latent must have batch 1")
        tq = [torch.tensor([[float(t)]]) for t in times]
        return torch.cat(self._decoding(tq, scale), 0)

    def decoding_localensemble(self, times=None, scale=None):
        """LunaTokis.decoding_localensemble (:962-1085): four decodes with the query shifted by
        (+-1/H, +-1/W), blended per HR pixel by the diagonally opposite |rel_y rel_x| area; batch-1
        latent, `times` a list of floats -> [len(times), 3, HH, WW]."""
        return self._call(self._decoding_localensemble, times, scale)

    def _decoding_localensemble(self, times=None, scale=None):
        if self._feat is None:
            raise RuntimeError("decoding needs gen_feat first")
        if self._feat.shape[1] != 1:
            raise ValueError("decoding_localensemble batches the query times: the latent must have batch 1")
        proj = self._projection()
        _, H, Wd, _ = proj.shape
        HH, WW = (H * 4, Wd * 4) if scale is None else (int(scale[0]), int(scale[1]))
        key = ("ens", str(self.device), H, Wd, HH, WW)
        if key not in self._tables:
            self._tables[key] = [torch.from_numpy(a).to(self.device) for a in ensemble_weights(H, Wd, HH, WW)]
        wts = self._tables[key]
        tq = [torch.tensor([[float(t)]]) for t in times]
        decs = [torch.cat(self._decode(proj, tq, HH, WW, self._tab(H, Wd, HH, WW, (vx, vy))), 0)
                for vx in (-1, 1) for vy in (-1, 1)]
        out = self._empty(len(times), 3, HH, WW)
        ops.dec_blend4(decs, wts, out)
        return out

    def forward(self, x, times=None, scale=None, test=False, center=None, index=0):
        """LunaTokis.forward (:1222-1231): decoding, or decoding_test with test=True."""
        return self._call(self._forward, x, times, scale, test)

    def _forward(self, x, times, scale, test):
        self._gen_feat(x)
        if test:
            return self._decoding_test(times, scale)
        return self._decoding(times, scale)
