"""``jax.experimental.mesh_utils`` equivalent (``case1a.py:6,15``; ``case5_attention_dense.py:82``,
``case6_attention.py:151``): ``create_device_mesh`` for one node, ``create_hybrid_device_mesh``
for an xGMI-inside / network-across node layout (see :mod:`..mesh`)."""
from ..mesh import create_device_mesh, create_hybrid_device_mesh  # noqa: F401

__all__ = ["create_device_mesh", "create_hybrid_device_mesh"]
