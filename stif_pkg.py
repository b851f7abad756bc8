"""Import helper: the package directory ``stif-continuous-video-representation_amd/``
has a name Python cannot ``import`` directly, so it is registered as ``stif_amd``."""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stif-continuous-video-representation_amd")


def load():
    mod = sys.modules.get("stif_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "stif_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["stif_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
