"""Device mesh: an n-d array of devices with named axes.

Reference usage: ``Mesh(devices=device_mesh, axis_names=('data','model'))``
(``case6_attention.py:155-156``) and ``with mesh:`` (``case6_attention.py:219,234``).
The context manager sets the ambient mesh that ``with_logical_constraint``
needs; the stack is thread-local.
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from typing import Optional, Sequence, Tuple

import numpy as np

from .runtime.devices import Device, process_index

__all__ = ["Mesh", "current_mesh", "create_device_mesh", "create_hybrid_device_mesh", "node_of"]

_TLS = threading.local()


def _stack():
    s = getattr(_TLS, "stack", None)
    if s is None:
        s = _TLS.stack = []
    return s


class Mesh:
    def __init__(self, devices, axis_names: Sequence[str]):
        arr = np.asarray(devices, dtype=object)
        if isinstance(axis_names, str):
            axis_names = (axis_names,)
        axis_names = tuple(axis_names)
        if arr.ndim != len(axis_names):
            raise ValueError(
                f"Mesh devices have rank {arr.ndim} but {len(axis_names)} axis names were given")
        if len(set(axis_names)) != len(axis_names):
            raise ValueError(f"duplicate mesh axis names {axis_names}")
        flat = list(arr.flat)
        if not all(isinstance(d, Device) for d in flat):
            raise TypeError("Mesh devices must be Device objects (see ljs.devices())")
        if len({d.id for d in flat}) != len(flat):
            raise ValueError("a device appears twice in the mesh")
        self.devices = arr
        self.axis_names = axis_names
        self.device_ids = np.vectorize(lambda d: d.id, otypes=[np.int64])(arr) if arr.size else arr.astype(np.int64)

    @property
    def shape(self) -> "OrderedDict[str, int]":
        return OrderedDict(zip(self.axis_names, self.devices.shape))

    @property
    def axis_sizes(self) -> Tuple[int, ...]:
        return tuple(self.devices.shape)

    @property
    def size(self) -> int:
        return int(self.devices.size)

    @property
    def empty(self) -> bool:
        return self.devices.size == 0

    @property
    def local_devices(self):
        pi = process_index()
        return [d for d in self.devices.flat if d.process_index == pi]

    @property
    def device_set(self):
        return set(self.devices.flat)

    def axis_index(self, name: str) -> int:
        return self.axis_names.index(name)

    def __enter__(self):
        _stack().append(self)
        return self

    def __exit__(self, *exc):
        _stack().pop()
        return False

    def __eq__(self, other):
        return (isinstance(other, Mesh) and self.axis_names == other.axis_names
                and np.array_equal(self.device_ids, other.device_ids))

    def __hash__(self):
        return hash((self.axis_names, self.device_ids.tobytes(), self.device_ids.shape))

    def __repr__(self):
        return f"Mesh(device_ids={self.device_ids.tolist()}, axis_names={self.axis_names})"


def current_mesh() -> Optional[Mesh]:
    s = _stack()
    return s[-1] if s else None


def create_device_mesh(mesh_shape: Sequence[int], devices: Optional[Sequence[Device]] = None,
                       *, contiguous_submeshes: bool = False) -> np.ndarray:
    """Arrange devices into an n-d array (``mesh_utils.create_device_mesh``, ``case1a.py:15``).

    MI355X nodes connect all 8 GPUs point-to-point over xGMI (7 links per GPU),
    so there is no torus topology to respect: every ordering gives the same
    link count between any pair.  The row-major order is kept so device ids
    match the reference's printed layouts (``(2,4)`` -> ``[[0,1,2,3],[4,5,6,7]]``).
    """
    from .runtime.devices import devices as _all

    mesh_shape = tuple(int(s) for s in mesh_shape)
    devs = list(_all() if devices is None else devices)
    n = int(np.prod(mesh_shape)) if mesh_shape else 1
    if n > len(devs):
        raise ValueError(f"mesh shape {mesh_shape} needs {n} devices, only {len(devs)} available")
    arr = np.empty(n, dtype=object)
    for i, d in enumerate(devs[:n]):
        arr[i] = d
    return arr.reshape(mesh_shape)


def node_of(d: Device) -> int:
    """The node (host) a device sits on: ranks are grouped ``LOCAL_WORLD_SIZE`` per node (torchrun's
    launch order, one process per GPU), a single-controller process owns one node's GPUs."""
    import os
    lws = int(os.environ.get("LJS_LOCAL_WORLD_SIZE", os.environ.get("LOCAL_WORLD_SIZE", "0")) or 0)
    if lws <= 0:
        return 0
    return d.process_index // lws


def create_hybrid_device_mesh(mesh_shape: Sequence[int], dcn_mesh_shape: Sequence[int],
                              devices: Optional[Sequence[Device]] = None) -> np.ndarray:
    """``mesh_utils.create_hybrid_device_mesh``: a mesh of shape ``mesh_shape * dcn_mesh_shape``
    (elementwise) whose ``dcn_mesh_shape`` factor spans nodes and whose ``mesh_shape`` factor
    spans the GPUs of one node.  On MI355X the in-node factor rides the point-to-point xGMI links
    (7 per GPU, ~153 GB/s each) and the cross-node factor the network, so an axis that carries the
    step's large or frequent collectives (tensor / sequence parallel) belongs in ``mesh_shape``
    and data parallelism - one bucketed gradient all-reduce per step - in ``dcn_mesh_shape``.
    Nodes are ordered by their lowest device id, and a node's GPUs fill its sub-mesh row-major."""
    mesh_shape = tuple(int(s) for s in mesh_shape)
    dcn_mesh_shape = tuple(int(s) for s in dcn_mesh_shape)
    if len(mesh_shape) != len(dcn_mesh_shape):
        raise ValueError(f"mesh_shape {mesh_shape} and dcn_mesh_shape {dcn_mesh_shape} need the same rank")
    from .runtime.devices import devices as _all
    devs = list(_all() if devices is None else devices)
    per_node = int(np.prod(mesh_shape)) if mesh_shape else 1
    n_nodes = int(np.prod(dcn_mesh_shape)) if dcn_mesh_shape else 1
    groups: "OrderedDict[int, list]" = OrderedDict()
    for d in sorted(devs, key=lambda d: d.id):
        groups.setdefault(node_of(d), []).append(d)
    nodes = [g for g in groups.values()]
    if len(nodes) == 1 and n_nodes > 1 and len(nodes[0]) >= per_node * n_nodes:
        # one node's devices standing in for several (host / virtual devices): consecutive blocks
        flat = nodes[0]
        nodes = [flat[i * per_node:(i + 1) * per_node] for i in range(n_nodes)]
    if len(nodes) < n_nodes or any(len(g) < per_node for g in nodes[:n_nodes]):
        raise ValueError(f"hybrid mesh {mesh_shape} x dcn {dcn_mesh_shape} needs {n_nodes} nodes of {per_node} "
                         f"devices; have {[len(g) for g in nodes]}")
    nd = len(mesh_shape)
    # [dcn_0, .., dcn_{k-1}, ici_0, .., ici_{k-1}] -> interleave (dcn_i, ici_i) -> merge each pair
    blocks = np.empty(dcn_mesh_shape + mesh_shape, dtype=object)
    for ni, node in enumerate(nodes[:n_nodes]):
        sub = np.empty(per_node, dtype=object)
        for i, d in enumerate(node[:per_node]):
            sub[i] = d
        blocks[np.unravel_index(ni, dcn_mesh_shape)] = sub.reshape(mesh_shape)
    order = [a for i in range(nd) for a in (i, nd + i)]
    out = blocks.transpose(order).reshape(tuple(a * b for a, b in zip(dcn_mesh_shape, mesh_shape)))
    return out
