"""stif_amd: MI355X-native (gfx950) engine for the STIF LunaTokis forward.

Import through ``stif_pkg.load()`` (the directory name is not a Python identifier).
Layout:
  csrc/       HIP kernels (conv, DCN, decoder) + C ABI (include/stif.h) + host packing
  _lib.py     ctypes binding of libstif_hip.so (no fallback: missing library -> error)
  ops.py      torch-buffer wrappers of the C ABI
  model.py    LunaTokis host (reference API: forward / gen_feat / decoding / load_state_dict)
  coords.py   fp32 query-grid tables of the decoder
  weights.py  state-dict spec + deterministic weight generator
  video.py    custom_video_test-style sliding-window driver
(integration/_ext.py at the repo root is the DCNv2 `_ext` shim over ops.dcn_v2_forward)
  parallel.py frame-pair sharding over ranks
  serving.py  option files, define_G / load_network / VideoSRModel (checkpoint drop-in)
  train.py    Charbonnier loss, the two restart LR schedules, Adam set-up (training drop-ins)
"""
from . import weights  # noqa: F401
from . import coords  # noqa: F401


def __getattr__(name):
    # torch-dependent parts load lazily so that weight/coords utilities work without torch/GPU
    if name in ("ops", "model", "video", "parallel", "_lib", "serving", "train"):
        import importlib
        return importlib.import_module(f"{__name__}.{name}")
    if name == "LunaTokis":
        from .model import LunaTokis
        return LunaTokis
    raise AttributeError(name)
