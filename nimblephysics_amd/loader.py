"""nimble.loadWorld (python/nimblephysics/loader.py:12): resolve `path`
relative to the running script and load it through the universal loader
(.skel -> SkelParser, nimblephysics_amd/skel.py; .urdf -> urdf.py).

The GPU box carries no model files of the reference, so the benchmark worlds
are also bundled as JSON exports (nimblephysics_amd/assets/, made by
tools/export_assets.py); a path whose file does not exist falls back to the
bundled export of the same name (e.g. "half_cheetah.skel" ->
assets/half_cheetah_world.json).
"""
from __future__ import annotations

import os
import sys

from . import assets
from .simulation import World

_BUNDLED = {"half_cheetah.skel": "half_cheetah_world"}


def loadWorld(path: str) -> World:
    root = os.path.join(os.getcwd(), sys.argv[0]) if sys.argv and sys.argv[0] else os.getcwd()
    absolute = os.path.join(os.path.dirname(root), path)
    for cand in (absolute, path):
        if os.path.exists(cand):
            return World.loadFrom(cand)
    name = _BUNDLED.get(os.path.basename(path))
    if name is not None:
        return assets.load_world(name)
    raise FileNotFoundError(path)
