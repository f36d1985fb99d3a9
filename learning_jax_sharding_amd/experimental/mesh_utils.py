"""``jax.experimental.mesh_utils`` equivalent (``case1a.py:6,15``)."""
from ..mesh import create_device_mesh  # noqa: F401

__all__ = ["create_device_mesh"]
