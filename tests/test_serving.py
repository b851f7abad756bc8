"""Checkpoint / option-file drop-in (serving.py) on CPU: option parsing, define_G, load_network
with DataParallel prefixes, create_model's pretrain loading; the GPU test runs VideoSRModel.test."""
import os

import numpy as np
import pytest
import torch

OPT_YML = """
name: stif_engine_test
model: VideoSR_base
distortion: sr
scale: 4
gpu_ids: [0]
datasets:
  test_1:
    name: synthetic
    mode: video_test
network_G:
  which_model_G: LIIF
  nf: 64
  nframes: 6
  groups: 8
  front_RBs: 5
  mid_RBs: 0
  back_RBs: 40
path:
  pretrain_model_G: {ckpt}
  strict_load: true
train:
  lr_G: !!float 2e-5
"""


@pytest.fixture()
def ckpt(tmp_path, sd):
    p = tmp_path / "latest_G.pth"
    torch.save({"module." + k: torch.from_numpy(v) for k, v in sd.items()}, p)
    return str(p)


@pytest.fixture()
def opt_file(tmp_path, ckpt):
    p = tmp_path / "test.yml"
    p.write_text(OPT_YML.format(ckpt=ckpt))
    return str(p)


def test_parse_and_define_G(stif, opt_file):
    S = stif.serving
    opt = S.parse_options(opt_file)
    assert opt["is_train"] is False and opt["datasets"]["test_1"]["scale"] == 4
    assert opt["train"]["lr_G"] == 2e-5
    net = S.define_G(opt, device="cpu")
    assert (net.front_RBs, net.back_RBs, net.ot_frames) == (5, 40, 6)
    opt["network_G"]["which_model_G"] = "TMNet"
    with pytest.raises(NotImplementedError):
        S.define_G(opt, device="cpu")


def test_load_network_strips_module_prefix(stif, sd, ckpt):
    S = stif.serving
    net = stif.LunaTokis(64, 6, 8, 5, 40, device="cpu")
    S.load_network(ckpt, net, strict=True)
    back = net.state_dict()
    assert list(back) == list(sd)
    assert np.array_equal(back["fusion.weight"].numpy(), sd["fusion.weight"])


def test_create_model_loads_pretrain(stif, sd, opt_file):
    S = stif.serving
    opt = S.parse_options(opt_file)
    m = S.create_model(opt, device="cpu")
    assert np.array_equal(m.netG.state_dict()["recon_trunk.3.conv1.bias"].numpy(), sd["recon_trunk.3.conv1.bias"])
    with pytest.raises(NotImplementedError):
        S.create_model(dict(opt, is_train=True), device="cpu")
    with pytest.raises(NotImplementedError):
        S.create_model(dict(opt, model="VideoSR_other"), device="cpu")


@pytest.mark.gpu
def test_video_sr_model_test_matches_reference(stif, opt_file, golden):
    """feed_data + test (VideoSR_base_model.py:90-149) against the reference outputs."""
    S = stif.serving
    m = S.create_model(S.parse_options(opt_file))
    g = golden["model_16x20"]
    times = [torch.tensor([[float(t)]]) for t in g["times"]]
    m.feed_data({"LQs": torch.from_numpy(g["x"]), "time": times}, need_GT=False)
    out = m.test(output=True)
    vis = m.get_current_visuals(need_GT=False)
    assert tuple(vis["restore"].shape) == (4, 3, 64, 80)
    ref = g["out"]
    assert np.abs(vis["restore"].numpy() - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6
    assert len(out) == 4
