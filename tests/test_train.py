"""SURVEY section 8 (f4), the training drop-ins of train.py on the CPU: the two restart LR schedules step for
step against sequences recorded from the reference's own classes (lr_scheduler.py:8-64, driven as
base_model.py:51-63 update_learning_rate drives them; tests/golden/make_golden.py sched), the Charbonnier loss
(loss.py:7-17) and the Adam / schedule set-up of VideoSR_base_model.py:56-83 from train_zsm.yml's options."""
import json
import math
import os

import pytest
import torch

import stif_pkg

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lr_schedules.json")


@pytest.fixture(scope="module")
def T():
    return stif_pkg.load().train


@pytest.mark.parametrize("case", ["cosine_zsm", "cosine_wrap", "cosine_weighted", "multistep"])
def test_schedule_matches_reference_sequence(T, case):
    g = json.load(open(GOLD))[case]
    c = g["case"]
    p = torch.zeros(3, requires_grad=True)
    opt = torch.optim.Adam([p], lr=c["lr"], weight_decay=0, betas=(0.9, 0.99))
    if c["kind"] == "cos":
        sch = T.CosineAnnealingLR_Restart(opt, c["T_period"], eta_min=c["eta_min"], restarts=c["restarts"],
                                          weights=c["weights"])
    else:
        sch = T.MultiStepLR_Restart(opt, c["milestones"], restarts=c["restarts"], weights=c["weights"],
                                    gamma=c["gamma"])
    lrs = [opt.param_groups[0]["lr"]]
    for it in range(1, c["iters"] + 1):
        T.update_learning_rate([sch], [opt], it, c["warmup"])
        lrs.append(opt.param_groups[0]["lr"])
    # the same recurrence in the same operation order: equal to the last bit
    assert lrs == g["lr"], [(i, a, b) for i, (a, b) in enumerate(zip(lrs, g["lr"])) if a != b][:5]


def test_cosine_restart_closed_form(T):
    """Between restarts the recurrence telescopes to eta + (lr0 - eta) (1 + cos(pi k / T)) / 2."""
    p = torch.zeros(1, requires_grad=True)
    opt = torch.optim.Adam([p], lr=1e-3)
    sch = T.CosineAnnealingLR_Restart(opt, [8, 8], restarts=[8], weights=[0.5], eta_min=1e-5)
    for e in range(1, 16):
        sch.step()
        k, lr0 = (e, 1e-3) if e < 8 else (e - 8, 0.5e-3)
        want = 1e-5 + (lr0 - 1e-5) * (1 + math.cos(math.pi * k / 8)) / 2
        assert abs(opt.param_groups[0]["lr"] - want) <= 1e-15, (e, opt.param_groups[0]["lr"], want)


def test_multistep_clear_state_drops_moments(T):
    p = torch.nn.Parameter(torch.ones(4))
    opt = torch.optim.Adam([p], lr=1e-2)
    sch = T.MultiStepLR_Restart(opt, [2], restarts=[0, 3], weights=[1, 1], gamma=0.1, clear_state=True)
    for _ in range(3):
        opt.zero_grad()
        (p * p).sum().backward()
        opt.step()
        sch.step()
    assert len(opt.state) == 0 and abs(opt.param_groups[0]["lr"] - 1e-2) < 1e-18


def test_charbonnier_and_optimizer_setup(T):
    x, y = torch.randn(2, 3, 5, 7, dtype=torch.float64), torch.randn(2, 3, 5, 7, dtype=torch.float64)
    assert torch.allclose(T.CharbonnierLoss()(x, y), torch.sqrt((x - y) ** 2 + 1e-6).sum(), rtol=0, atol=1e-12)
    net = torch.nn.Conv2d(3, 4, 3)
    # train_zsm.yml:53-65
    opt, sch = T.make_optimizer(net, dict(lr_G=2e-4, beta1=0.9, beta2=0.99, weight_decay_G=0,
                                          lr_scheme="CosineAnnealingLR_Restart", T_period=[150000] * 4,
                                          restarts=[150000, 300000, 450000], restart_weights=[1, 1, 1],
                                          eta_min=1e-7))
    assert isinstance(opt, torch.optim.Adam) and opt.param_groups[0]["betas"] == (0.9, 0.99)
    assert isinstance(sch, T.CosineAnnealingLR_Restart) and sch.T_max == 150000
    with pytest.raises(NotImplementedError):
        T.make_optimizer(net, dict(lr_G=1e-4, beta1=0.9, beta2=0.99, lr_scheme="Plateau"))
