from . import mesh_utils  # noqa: F401
