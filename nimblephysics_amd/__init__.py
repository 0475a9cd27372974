"""nimblephysics_amd -- MI355X-native differentiable timestep.

Drop-in for the reference's ``nimble.timestep`` hot path
(python/nimblephysics/timestep.py) with the model API subset it needs:
``nimblephysics_amd.simulation.World``, ``nimblephysics_amd.dynamics``.
"""
from . import dynamics, neural, simulation  # noqa: F401
from .simulation import World  # noqa: F401
from .timestep import TimestepLayer, timestep  # noqa: F401
from .loader import loadWorld  # noqa: F401

__all__ = ["dynamics", "neural", "simulation", "World", "timestep", "TimestepLayer", "loadWorld"]
