"""Training-side pieces of the reference's VideoSRBaseModel (training only):
the Charbonnier pixel loss and the two learning-rate schedules its option files select, as drop-ins with
the reference's names, arguments and step semantics.

* ``CharbonnierLoss`` -- loss.py:7-17: sum(sqrt((x - y)^2 + eps)).
* ``CosineAnnealingLR_Restart`` -- lr_scheduler.py:34-64, selected by ``lr_scheme: CosineAnnealingLR_Restart``
  (VideoSR_base_model.py:77-82; train_zsm.yml:57-65): cosine annealing from the group's lr to ``eta_min``
  over ``T_period[k]`` steps, restarted at ``restarts[k]`` to ``initial_lr * weights[k]``.
* ``MultiStepLR_Restart`` -- lr_scheduler.py:8-31 (``lr_scheme: MultiStepLR``, VideoSR_base_model.py:70-76):
  lr x gamma^(multiplicity) at each milestone, restarts as above, optionally clearing the optimizer state.

Both schedules are recurrences on the group's current lr (each step scales the previous lr), exactly as the
reference evaluates them, so a resumed optimizer continues the same sequence; ``tests/test_train.py`` checks
them step for step against sequences recorded from the reference's own classes (tests/golden/make_golden.py
sched).  ``optimize_step`` is VideoSRBaseModel.optimize_parameters (VideoSR_base_model.py:113-134) for a
module and one target.  The HIP forward (``LunaTokis``) is inference-only; training runs a torch module whose
DCN_sep layers call the ``_ext`` drop-in (integration/_ext.py: stif_dcn_v2_forward / _backward).
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict

import torch
from torch import nn
from torch.optim.lr_scheduler import LRScheduler


class CharbonnierLoss(nn.Module):
    """loss.py:7-17 (``pixel_criterion: cb``)"""

    def __init__(self, eps: float = 1e-6):
        super().__init__()
        self.eps = eps

    def forward(self, x, y):
        d = x - y
        return torch.sum(torch.sqrt(d * d + self.eps))


def _restart_lists(restarts, weights):
    r = list(restarts) if restarts else [0]
    w = list(weights) if weights else [1]
    if len(r) != len(w):
        raise ValueError("restarts and their weights do not match")
    return r, w


class CosineAnnealingLR_Restart(LRScheduler):
    """lr_scheduler.py:34-64.  Step e of the current period (k = e - last restart, period T):
    lr_e = eta_min + (lr_{e-1} - eta_min) * (1 + cos(pi k / T)) / (1 + cos(pi (k - 1) / T)); at a restart
    lr = initial_lr * weight and T becomes the next T_period entry; at k = T + 1 (mod 2T) the ratio's
    denominator vanishes and the schedule adds (base_lr - eta_min) (1 - cos(pi / T)) / 2 instead."""

    def __init__(self, optimizer, T_period, restarts=None, weights=None, eta_min=0, last_epoch=-1):
        self.T_period = list(T_period)
        self.T_max = self.T_period[0]
        self.eta_min = eta_min
        self.restarts, self.restart_weights = _restart_lists(restarts, weights)
        self.last_restart = 0
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        e, groups, eta = self.last_epoch, self.optimizer.param_groups, self.eta_min
        if e == 0:
            return list(self.base_lrs)
        if e in self.restarts:
            i = self.restarts.index(e)
            self.last_restart, self.T_max = e, self.T_period[i + 1]
            return [g["initial_lr"] * self.restart_weights[i] for g in groups]
        T, k = self.T_max, e - self.last_restart
        if (k - 1 - T) % (2 * T) == 0:
            return [g["lr"] + (b - eta) * (1 - math.cos(math.pi / T)) / 2 for b, g in zip(self.base_lrs, groups)]
        ratio = (1 + math.cos(math.pi * k / T)) / (1 + math.cos(math.pi * (k - 1) / T))
        return [ratio * (g["lr"] - eta) + eta for g in groups]


class MultiStepLR_Restart(LRScheduler):
    """lr_scheduler.py:8-31: at step e, a restart sets lr = initial_lr * weight (and, with ``clear_state``,
    drops the optimizer's moments); otherwise lr *= gamma ** (how often e appears in ``milestones``)."""

    def __init__(self, optimizer, milestones, restarts=None, weights=None, gamma=0.1, clear_state=False,
                 last_epoch=-1):
        self.milestones = Counter(milestones)
        self.gamma = gamma
        self.clear_state = clear_state
        self.restarts, self.restart_weights = _restart_lists(restarts, weights)
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        e, groups = self.last_epoch, self.optimizer.param_groups
        if e in self.restarts:
            if self.clear_state:
                self.optimizer.state = defaultdict(dict)
            w = self.restart_weights[self.restarts.index(e)]
            return [g["initial_lr"] * w for g in groups]
        n = self.milestones.get(e, 0)
        if n == 0:
            return [g["lr"] for g in groups]
        return [g["lr"] * self.gamma ** n for g in groups]


def make_optimizer(net: nn.Module, train_opt: dict):
    """VideoSR_base_model.py:56-83: Adam over the trainable parameters and the configured schedule."""
    wd = train_opt.get("weight_decay_G") or 0
    opt = torch.optim.Adam([p for p in net.parameters() if p.requires_grad], lr=train_opt["lr_G"],
                           weight_decay=wd, betas=(train_opt["beta1"], train_opt["beta2"]))
    scheme = train_opt["lr_scheme"]
    if scheme == "CosineAnnealingLR_Restart":
        sched = CosineAnnealingLR_Restart(opt, train_opt["T_period"], eta_min=train_opt["eta_min"],
                                          restarts=train_opt.get("restarts"), weights=train_opt.get("restart_weights"))
    elif scheme == "MultiStepLR":
        sched = MultiStepLR_Restart(opt, train_opt["lr_steps"], restarts=train_opt.get("restarts"),
                                    weights=train_opt.get("restart_weights"), gamma=train_opt["lr_gamma"],
                                    clear_state=train_opt.get("clear_state", False))
    else:
        raise NotImplementedError(f"lr_scheme {scheme!r}")
    return opt, sched


def update_learning_rate(schedulers, optimizers, cur_iter: int, warmup_iter: int = -1):
    """base_model.py:51-63: step every schedule, then during warm-up (cur_iter < warmup_iter) override each
    group's lr with initial_lr / warmup_iter * cur_iter."""
    for sch in schedulers:
        sch.step()
    if cur_iter < warmup_iter:
        for opt in optimizers:
            for g in opt.param_groups:
                g["lr"] = g["initial_lr"] / warmup_iter * cur_iter


def optimize_step(net: nn.Module, opt, criterion, inputs, gt, weight: float = 1.0) -> float:
    """VideoSR_base_model.py:113-134 for one output: zero_grad, forward, weight * criterion, backward,
    optimizer step; returns the loss (the caller steps the schedule, as train.py does per iteration)."""
    opt.zero_grad()
    loss = weight * criterion(net(*inputs), gt)
    loss.backward()
    opt.step()
    return float(loss.detach())
