"""a training step through the `_ext` drop-in.

A DCN_sep-bearing module (dcn_v2.py:110-140: conv_offset_mask, chunk / cat / sigmoid, the _DCNv2
autograd wiring of dcn_v2.py:15-47 on `_ext.dcn_v2_forward` / `_ext.dcn_v2_backward`) takes one
VideoSRBaseModel.optimize_parameters step (VideoSR_base_model.py:113-134): the Charbonnier loss
(loss.py:7-17, sum of sqrt(d^2 + 1e-6)), backward, Adam with the shipped options (train_zsm.yml:56-59:
lr 2e-5, betas (0.9, 0.99), no weight decay).  GPU: integration/_ext.py (stif_dcn_v2_forward /
stif_dcn_v2_backward).  Oracle: the same step in float64 on the CPU with the DCN op restated
(oracle dcn_v2_forward / dcn_v2_backward); conv, sigmoid, loss and Adam by torch (float64).
"""
import importlib.util
import os

import numpy as np
import pytest
import torch
from torch import nn

from oracle import stif_oracle as O

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ext():
    spec = importlib.util.spec_from_file_location("_ext", os.path.join(REPO, "integration", "_ext.py"))
    ext = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ext)
    return ext


class _OracleBackend:
    """the oracle as an `_ext` (float64 numpy in, torch float64 out)"""

    @staticmethod
    def dcn_v2_forward(inp, w, b, off, msk, *dims):
        n = lambda t: t.detach().cpu().numpy()
        return torch.from_numpy(O.dcn_v2_forward(n(inp), n(w), n(b), n(off), n(msk), *dims))

    @staticmethod
    def dcn_v2_backward(inp, w, b, off, msk, go, *dims):
        n = lambda t: t.detach().cpu().numpy()
        return [torch.from_numpy(np.asarray(g, np.float64)) for g in
                O.dcn_v2_backward(n(inp), n(w), n(b), n(off), n(msk), n(go), *dims)]


def make_dcn_conv(backend):
    class _DCNv2(torch.autograd.Function):   # dcn_v2.py:15-47 wiring
        @staticmethod
        def forward(ctx, inp, offset, mask, weight, bias, dg):
            ctx.dg = dg
            ctx.save_for_backward(inp, offset, mask, weight, bias)
            return backend.dcn_v2_forward(inp, weight, bias, offset, mask, 3, 3, 1, 1, 1, 1, 1, 1, dg)

        @staticmethod
        def backward(ctx, go):
            inp, offset, mask, weight, bias = ctx.saved_tensors
            gi, goff, gm, gw, gb = backend.dcn_v2_backward(inp, weight, bias, offset, mask, go.contiguous(),
                                                           3, 3, 1, 1, 1, 1, 1, 1, ctx.dg)
            return gi, goff, gm, gw, gb, None
    return _DCNv2.apply


class DcnSep(nn.Module):
    """DCN_sep(64, 64, 3, stride=1, padding=1, deformable_groups=8) (dcn_v2.py:110-140)"""

    def __init__(self, conv_fn, dtype, device):
        super().__init__()
        self.conv_fn = conv_fn
        kw = dict(dtype=dtype, device=device)
        self.weight = nn.Parameter(torch.empty(64, 64, 3, 3, **kw))
        self.bias = nn.Parameter(torch.empty(64, **kw))
        self.conv_offset_mask = nn.Conv2d(64, 216, 3, 1, 1, bias=True, **kw)

    def forward(self, inp, fea):
        out = self.conv_offset_mask(fea)
        o1, o2, mask = torch.chunk(out, 3, dim=1)
        offset = torch.cat((o1, o2), dim=1)
        return self.conv_fn(inp, offset.contiguous(), torch.sigmoid(mask).contiguous(), self.weight, self.bias, 8)


def charbonnier(x, y, eps=1e-6):   # loss.py:14-17
    d = x - y
    return torch.sum(torch.sqrt(d * d + eps))


def _step(net, inp, fea, gt):
    opt = torch.optim.Adam(net.parameters(), lr=2e-5, weight_decay=0, betas=(0.9, 0.99))
    opt.zero_grad()
    loss = charbonnier(net(inp, fea), gt)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in net.named_parameters()}
    opt.step()
    return float(loss.detach()), grads, {k: p.detach().clone() for k, p in net.named_parameters()}


def test_training_step_through_ext_shim_matches_oracle(sd):
    rng = np.random.default_rng(21)
    B, H, W = 2, 12, 17
    p = "pcd_align.L1_dcnpack_1"
    init = {"weight": sd[p + ".weight"], "bias": sd[p + ".bias"],
            "conv_offset_mask.weight": sd[p + ".conv_offset_mask.weight"] * 0.2,   # offsets of a few pixels
            "conv_offset_mask.bias": sd[p + ".conv_offset_mask.bias"]}
    inp = rng.standard_normal((B, 64, H, W)).astype(np.float32)
    fea = rng.standard_normal((B, 64, H, W)).astype(np.float32)

    def make(backend, dt, dev):
        net = DcnSep(make_dcn_conv(backend), dt, dev)
        with torch.no_grad():
            for k, v in net.named_parameters():
                v.copy_(torch.from_numpy(np.asarray(init[k])))
        return net

    # the target sits 1-2 away from the output everywhere: the Charbonnier gradient d / sqrt(d^2 + 1e-6)
    # is then ~sign(d) and well conditioned (near d = 0 it amplifies a 1e-6 forward difference ~350x,
    # which would test the loss's conditioning, not the DCN op)
    with torch.no_grad():
        out0 = make(_OracleBackend, torch.float64, "cpu")(torch.from_numpy(inp).double(),
                                                          torch.from_numpy(fea).double()).numpy()
    gt = (out0 + np.where(rng.random(out0.shape) < 0.5, -1.0, 1.0) * (1.0 + rng.random(out0.shape))).astype(np.float32)
    res = {}
    for name, backend, dt, dev in (("gpu", _ext(), torch.float32, "cuda"), ("oracle", _OracleBackend, torch.float64, "cpu")):
        net = make(backend, dt, dev)
        T = lambda a: torch.from_numpy(a).to(dev, dt)
        res[name] = _step(net, T(inp), T(fea), T(gt))
    (lg, gg, pg), (lo, go, po) = res["gpu"], res["oracle"]
    assert abs(lg - lo) <= 1e-5 * abs(lo), (lg, lo)
    for k in go:
        g, r = gg[k].double().cpu(), go[k]
        err, tol = float((g - r).abs().max()), 2e-5 * float(r.abs().max())
        assert err <= tol, (k, err, tol)
        # Adam's first step moves each parameter by ~lr * sign(grad): equal wherever the gradient's sign
        # is not decided by rounding
        d = (pg[k].double().cpu() - po[k]).abs()
        firm = r.abs() > 1e-3 * r.abs().max()
        e_firm, e_all = float(d[firm].max()), float(d.max())
        assert e_firm <= 1e-6, (k, e_firm)
        assert e_all <= 2 * 2e-5 + 1e-6, (k, e_all)


def test_training_loop_with_restart_schedule_matches_oracle(sd):
    """Six iterations of the reference's training loop (VideoSRBaseModel: update_learning_rate -- the
    CosineAnnealingLR_Restart schedule of train.py, base_model.py:51-63 -- then optimize_parameters,
    VideoSR_base_model.py:113-134, Charbonnier + Adam) on the DCN_sep module through the `_ext` drop-in, vs the
    same loop on the oracle in float64: the losses agree every iteration, the schedule's learning rates are the
    ones the run used, and every parameter whose gradient is firm at every iteration ends where the oracle's
    does (Adam normalises each update, so only entries whose gradient sign rounding could flip may differ, by
    at most one lr-sized step per iteration)."""
    import stif_pkg
    T = stif_pkg.load().train
    rng = np.random.default_rng(22)
    B, H, W = 2, 10, 13
    p = "pcd_align.L2_dcnpack_1"
    init = {"weight": sd[p + ".weight"], "bias": sd[p + ".bias"],
            "conv_offset_mask.weight": sd[p + ".conv_offset_mask.weight"] * 0.2,
            "conv_offset_mask.bias": sd[p + ".conv_offset_mask.bias"]}
    inp = rng.standard_normal((B, 64, H, W)).astype(np.float32)
    fea = rng.standard_normal((B, 64, H, W)).astype(np.float32)

    def make(backend, dt, dev):
        net = DcnSep(make_dcn_conv(backend), dt, dev)
        with torch.no_grad():
            for k, v in net.named_parameters():
                v.copy_(torch.from_numpy(np.asarray(init[k])))
        return net

    with torch.no_grad():
        out0 = make(_OracleBackend, torch.float64, "cpu")(torch.from_numpy(inp).double(),
                                                          torch.from_numpy(fea).double()).numpy()
    gt = (out0 + np.where(rng.random(out0.shape) < 0.5, -1.0, 1.0) * (1.0 + rng.random(out0.shape))).astype(np.float32)
    opts = dict(lr_G=2e-5, beta1=0.9, beta2=0.99, weight_decay_G=0, lr_scheme="CosineAnnealingLR_Restart",
                T_period=[3, 3], restarts=[3], restart_weights=[0.5], eta_min=1e-7)
    runs = {}
    for name, backend, dt, dev in (("gpu", _ext(), torch.float32, "cuda"), ("oracle", _OracleBackend, torch.float64, "cpu")):
        net = make(backend, dt, dev)
        opt, sch = T.make_optimizer(net, opts)
        X = [torch.from_numpy(a).to(dev, dt) for a in (inp, fea)]
        G = torch.from_numpy(gt).to(dev, dt)
        crit = T.CharbonnierLoss()
        losses, lrs, grads = [], [], []
        for it in range(1, 7):
            T.update_learning_rate([sch], [opt], it)
            lrs.append(opt.param_groups[0]["lr"])
            losses.append(T.optimize_step(net, opt, crit, X, G))
            grads.append({k: v.grad.detach().double().cpu().clone() for k, v in net.named_parameters()})
        runs[name] = (losses, lrs, grads, {k: v.detach().double().cpu() for k, v in net.named_parameters()})
    (lg, rg, gg, pg), (lo, ro, go, po) = runs["gpu"], runs["oracle"]
    assert rg == ro
    # cosine from 2e-5 over 3 steps, restart at 3 to 1e-5, then down again
    assert abs(ro[2] - 1e-5) < 1e-18 and ro[0] < 2e-5 and ro[1] < ro[0] and ro[3] < ro[2], ro
    for a, b in zip(lg, lo):
        assert abs(a - b) <= 1e-5 * abs(b), (lg, lo)
    for k in po:
        firm = torch.ones_like(po[k], dtype=torch.bool)
        for gi in go:
            firm &= gi[k].abs() > 1e-3 * gi[k].abs().max()
        d = (pg[k] - po[k]).abs()
        assert float(d[firm].max()) <= 6e-6, (k, float(d[firm].max()))
        assert float(d.max()) <= 6 * 2 * 2e-5 + 1e-6, (k, float(d.max()))
