"""MI355X-native N-body hot path: SEGNN / PONITA / EGNN-MC self-feed rollout and the
GravitySim ground-truth integrator, behind the reference's plugin registry.

The directory name is not a Python identifier; import it through the alias that
``nbody_amd.py`` at the repository root registers (``import nbody_amd``).
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
