"""stif_amd: MI355X-native (gfx950) engine for the STIF LunaTokis forward.

Import through ``stif_pkg.load()`` (the directory name is not a Python identifier).
"""
from . import weights  # noqa: F401
