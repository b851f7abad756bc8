"""Checkpoint + option-file drop-in for the reference's inference entry points.

Mirrors, for inference, what a user of the reference reaches the LunaTokis path through:
  * ``options.parse`` (codes/options/options.py:9-60): YAML option files (``yaml.safe_load``);
  * ``networks.define_G`` (codes/models/networks.py:7-26) for ``which_model_G: LIIF`` -- the
    reference's branch calls ``Sakuya_arch_test.LunaTokis`` without importing the module, so it
    cannot run as shipped; here it builds the MI355X LunaTokis;
  * ``BaseModel.load_network`` (codes/models/base_model.py:89-99): state dict file, ``module.``
    prefixes stripped, ``load_state_dict(strict)``;
  * ``create_model`` / ``VideoSRBaseModel`` (codes/models/__init__.py:5-13,
    codes/models/VideoSR_base_model.py:17-180): ``feed_data``, ``test``, ``get_current_visuals``,
    ``load`` from ``path.pretrain_model_G``.
Training (losses, optimizers, schedulers, DataParallel) is out of scope: ``is_train`` raises.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

from .model import LunaTokis


def parse_options(opt_path: str, is_train: bool = False) -> dict:
    """options.parse (options.py:9-60) for the keys inference uses: YAML (safe loader), ``is_train``,
    ``~``-expanded paths, the network scale copied to every dataset entry."""
    import yaml

    with open(opt_path) as f:
        opt = yaml.safe_load(f)
    opt["is_train"] = is_train
    scale = opt.get("scale")
    for phase, dataset in (opt.get("datasets") or {}).items():
        dataset["phase"] = phase.split("_")[0]
        if opt.get("distortion") in ("sr", "isr"):
            dataset["scale"] = scale
    for key, path in (opt.get("path") or {}).items():
        if path and key != "strict_load" and isinstance(path, str):
            opt["path"][key] = os.path.expanduser(path)
    return opt


def define_G(opt: dict, device="cuda") -> LunaTokis:
    """networks.define_G (networks.py:7-26): the LIIF generator = LunaTokis(nf, nframes, groups,
    front_RBs, back_RBs).  The reference's other generators (LunaTokis of Sakuya_arch_o, TMNet)
    are different model families, outside this engine."""
    opt_net = opt["network_G"]
    which = opt_net["which_model_G"]
    if which == "LIIF":
        return LunaTokis(nf=opt_net["nf"], nframes=opt_net["nframes"], groups=opt_net["groups"],
                         front_RBs=opt_net["front_RBs"], back_RBs=opt_net["back_RBs"], device=device)
    if which in ("LunaTokis", "TMNet"):
        raise NotImplementedError(f"Generator model [{which}] is not part of the MI355X engine (LIIF only)")
    raise NotImplementedError("Generator model [{:s}] not recognized".format(which))


def load_network(load_path: str, network: LunaTokis, strict: bool = True):
    """BaseModel.load_network (base_model.py:89-99).  The file is read with
    ``torch.load(weights_only=True)`` (tensors only, nothing executed); ``module.`` prefixes of a
    DataParallel checkpoint are stripped."""
    load_net = torch.load(load_path, map_location="cpu", weights_only=True)
    clean = OrderedDict()
    for k, v in load_net.items():
        clean[k[7:] if k.startswith("module.") else k] = v
    return network.load_state_dict(clean, strict=strict)


class VideoSRModel:
    """Inference side of VideoSRBaseModel (VideoSR_base_model.py:17-180) for the LIIF generator."""

    def __init__(self, opt: dict, device="cuda"):
        if opt.get("is_train"):
            raise NotImplementedError("training (DCN backward, losses, optimizers) is out of scope of the engine")
        self.opt = opt
        self.device = torch.device(device)
        self.netG = define_G(opt, device)
        self.net_opt = opt["network_G"]
        self.net_base = self.net_opt["which_model_G"]
        self.times = None
        self.scale = None
        self.testmode = False
        self.load()

    def load(self):
        """VideoSRBaseModel.load (:174-178): path.pretrain_model_G with path.strict_load."""
        path = (self.opt.get("path") or {}).get("pretrain_model_G")
        if path is not None:
            load_network(path, self.netG, bool(self.opt["path"].get("strict_load", True)))

    def feed_data(self, data: dict, need_GT: bool = True):
        """VideoSRBaseModel.feed_data (:90-107)."""
        self.var_L = data["LQs"].to(self.device)
        self.times = [t.to(self.device) for t in data["time"]] if "time" in data else None
        self.scale = data.get("scale")
        self.testmode = data.get("test", False)
        if need_GT:
            self.real_H = data["GT"].to(self.device)

    def test(self, output: bool = False):
        """VideoSRBaseModel.test (:135-149): netG(LQs, times, scale, test) under no_grad."""
        if self.times is None:
            raise ValueError("LIIF needs query times: feed_data with a 'time' entry")
        with torch.no_grad():
            self.fake_H = self.netG(self.var_L, self.times, self.scale, self.testmode)
        if output:
            return self.fake_H

    def get_current_visuals(self, need_GT: bool = True) -> OrderedDict:
        """VideoSRBaseModel.get_current_visuals (:154-161); the LIIF output (a list over times, or a
        tensor for decoding_test) is stacked time-major for item 0."""
        fake = self.fake_H
        if isinstance(fake, (list, tuple)):
            fake = torch.stack(list(fake), 1)
        out = OrderedDict()
        out["LQ"] = self.var_L.detach()[0].float().cpu()
        out["restore"] = fake.detach()[0].float().cpu()
        if need_GT:
            out["GT"] = self.real_H.detach()[0].float().cpu()
        return out


def create_model(opt: dict, device="cuda") -> VideoSRModel:
    """models.create_model (models/__init__.py:5-13) for model: VideoSR_base."""
    if opt.get("model") != "VideoSR_base":
        raise NotImplementedError("Model [{}] not recognized.".format(opt.get("model")))
    return VideoSRModel(opt, device)
