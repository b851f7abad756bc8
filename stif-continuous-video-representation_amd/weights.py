"""State-dict layout of STIF ``LunaTokis`` and a deterministic weight generator.

The reference's trained checkpoint ``latest_G.pth`` is not in the tree
(``.MISSING_LARGE_BLOBS:1``), so parity and benchmarking use weights drawn by
this generator.  The key names, order and shapes are exactly the reference
``state_dict`` (442 keys, 11,312,698 parameters); ``tests/golden`` pins them
against a dump taken from the reference module itself.

Key order follows module registration in
``codes/models/modules/Sakuya_arch_test.py:268-311`` (LunaTokis),
``:20-67`` (PCD_Align), ``:132-142`` (Easy_PCD), ``:168-190``
(DeformableConvLSTM, whose ``ConvLSTM.__init__`` registers ``cell_list`` first,
``convlstm.py:66-100``), ``codes/models/modules/DCNv2/dcn_v2.py:53-125``
(DCNv2 params then ``conv_offset_mask``) and ``SIREN.py:49-79``.

The generator mirrors the reference init *families*:
  * ResidualBlock_noBN convs: kaiming-normal(fan_in) x 0.1 (``module_util.py:7-24,46``)
  * other ``nn.Conv2d``: PyTorch default U(+-1/sqrt(fan_in))
  * SIREN: first layer U(+-1/in), later layers U(+-sqrt(6/in)/30) (``SIREN.py:35-42,66-67``)
but, unlike the reference, gives every bias a small random value and gives
``conv_offset_mask`` a non-zero draw: the reference zero-initialises it
(``dcn_v2.py:123-125``), which would collapse every deformable conv to 0.5*conv
and leave the bilinear sampling path untested.
"""
from __future__ import annotations

import zlib
from collections import OrderedDict

import numpy as np

NF = 64

_PCD_LAYERS = [
    # (name, cin, cout) in registration order of PCD_Align.__init__ for one direction
    ("L3_offset_conv1", 2 * NF, NF),
    ("L3_offset_conv2", NF, NF),
    ("L3_dcnpack", None, None),
    ("L2_offset_conv1", 2 * NF, NF),
    ("L2_offset_conv2", 2 * NF, NF),
    ("L2_offset_conv3", NF, NF),
    ("L2_dcnpack", None, None),
    ("L2_fea_conv", 2 * NF, NF),
    ("L1_offset_conv1", 2 * NF, NF),
    ("L1_offset_conv2", 2 * NF, NF),
    ("L1_offset_conv3", NF, NF),
    ("L1_dcnpack", None, None),
    ("L1_fea_conv", 2 * NF, NF),
]


def _conv(spec, name, cout, cin, k):
    spec[name + ".weight"] = (cout, cin, k, k)
    spec[name + ".bias"] = (cout,)


def _pcd_align(spec, prefix, groups=8):
    for d in (1, 2):
        for lname, cin, cout in _PCD_LAYERS:
            n = f"{prefix}{lname}_{d}"
            if cin is None:
                spec[n + ".weight"] = (NF, NF, 3, 3)
                spec[n + ".bias"] = (NF,)
                _conv(spec, n + ".conv_offset_mask", groups * 3 * 9, NF, 3)
            else:
                _conv(spec, n, cout, cin, 3)


def _easy_pcd(spec, prefix, groups=8):
    for n, s in (("fea_L2_conv1", 2), ("fea_L2_conv2", 1), ("fea_L3_conv1", 2), ("fea_L3_conv2", 1)):
        _conv(spec, prefix + n, NF, NF, 3)
    _pcd_align(spec, prefix + "pcd_align.", groups)
    _conv(spec, prefix + "fusion", NF, 2 * NF, 1)


def _siren(spec, prefix, fin, hidden, fout):
    dims = [fin] + list(hidden)
    for i in range(len(hidden)):
        spec[f"{prefix}net.{i}.linear.weight"] = (dims[i + 1], dims[i])
        spec[f"{prefix}net.{i}.linear.bias"] = (dims[i + 1],)
    spec[f"{prefix}net.{len(hidden)}.weight"] = (fout, hidden[-1])
    spec[f"{prefix}net.{len(hidden)}.bias"] = (fout,)


FEAT_IMNET = (201, (64, 64, 256), 64)      # Sakuya_arch_test.py:306-307
FLOW_IMNET = (263, (64, 64, 256), 4)       # :308-309
ENCODE_IMNET = (525, (64, 64, 256, 256), 3)  # :310-311


def state_dict_spec(nf: int = 64, front_RBs: int = 5, back_RBs: int = 40, groups: int = 8):
    """Ordered {key: shape} of ``LunaTokis(nf, nframes, groups, front_RBs, back_RBs).state_dict()``."""
    if nf != NF:
        raise ValueError("STIF decoder widths are hard-wired to nf=64 (Sakuya_arch_test.py:306-311)")
    spec: "OrderedDict[str, tuple]" = OrderedDict()
    _conv(spec, "conv_first", NF, 3, 3)
    for i in range(front_RBs):
        _conv(spec, f"feature_extraction.{i}.conv1", NF, NF, 3)
        _conv(spec, f"feature_extraction.{i}.conv2", NF, NF, 3)
    for n in ("fea_L2_conv1", "fea_L2_conv2", "fea_L3_conv1", "fea_L3_conv2"):
        _conv(spec, n, NF, NF, 3)
    _pcd_align(spec, "pcd_align.", groups)
    _conv(spec, "fusion", NF, 2 * NF, 1)
    _conv(spec, "ConvBLSTM.forward_net.cell_list.0.conv", 4 * NF, 2 * NF, 3)
    _easy_pcd(spec, "ConvBLSTM.forward_net.pcd_h.", groups)
    _easy_pcd(spec, "ConvBLSTM.forward_net.pcd_c.", groups)
    _conv(spec, "ConvBLSTM.conv_1x1", NF, 2 * NF, 1)
    for i in range(back_RBs):
        _conv(spec, f"recon_trunk.{i}.conv1", NF, NF, 3)
        _conv(spec, f"recon_trunk.{i}.conv2", NF, NF, 3)
    # upsampling head: registered (so strict loading needs it) but never run (Sakuya_arch_test.py:295-299)
    _conv(spec, "upconv1", NF * 4, NF, 3)
    _conv(spec, "upconv2", 64 * 4, NF, 3)
    _conv(spec, "HRconv", 64, 64, 3)
    _conv(spec, "conv_last", 3, 64, 3)
    _siren(spec, "feat_imnet.", *FEAT_IMNET)
    _siren(spec, "flow_imnet.", *FLOW_IMNET)
    _siren(spec, "encode_imnet.", *ENCODE_IMNET)
    return spec


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng(np.random.SeedSequence([seed, zlib.crc32(key.encode())]))


# std of the offset/mask conv weights: chosen so that DCN offsets are a few
# pixels (fractional, some pointing outside the frame) on random inputs.
OFFSET_W_STD = 1.0
OFFSET_B_STD = 0.5


def make_weight(key: str, shape, seed: int = 0) -> np.ndarray:
    """Deterministic fp32 tensor for one state-dict key (independent of the other keys)."""
    g = _rng(seed, key)
    shape = tuple(shape)
    is_w = key.endswith(".weight")
    if ".conv_offset_mask." in key:
        std = OFFSET_W_STD if is_w else OFFSET_B_STD
        return (g.standard_normal(shape) * std).astype(np.float32)
    if "_imnet." in key:
        fin = shape[-1] if is_w else None
        if is_w:
            first = ".net.0." in key
            bound = 1.0 / fin if first else np.sqrt(6.0 / fin) / 30.0
            return g.uniform(-bound, bound, shape).astype(np.float32)
        # nn.Linear default bias U(+-1/sqrt(fan_in)); fan_in is not in the bias shape, use a fixed scale
        return g.uniform(-0.05, 0.05, shape).astype(np.float32)
    if ("feature_extraction." in key or "recon_trunk." in key):
        if is_w:
            fan_in = int(np.prod(shape[1:]))
            return (g.standard_normal(shape) * np.sqrt(2.0 / fan_in) * 0.1).astype(np.float32)
        return g.uniform(-0.01, 0.01, shape).astype(np.float32)
    if is_w:
        fan_in = int(np.prod(shape[1:]))
        bound = 1.0 / np.sqrt(fan_in)
        return g.uniform(-bound, bound, shape).astype(np.float32)
    return g.uniform(-0.05, 0.05, shape).astype(np.float32)


def make_state_dict(seed: int = 0, nf: int = 64, front_RBs: int = 5, back_RBs: int = 40, groups: int = 8):
    """Ordered {key: np.float32 array} with the reference's 442 keys."""
    spec = state_dict_spec(nf, front_RBs, back_RBs, groups)
    return OrderedDict((k, make_weight(k, s, seed)) for k, s in spec.items())
