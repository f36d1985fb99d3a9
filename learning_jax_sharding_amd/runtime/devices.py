"""Device model and backend selection.

The reference fakes N in-process CPU devices by setting
``XLA_FLAGS=--xla_force_host_platform_device_count=N`` *before* importing JAX
(``case1a.py:2-3`` uses 8, ``case6_attention.py:4-5`` uses 4).  Here the same
idea is a small device factory with three personalities:

* ``cpu``  - N host devices in one process (torch CPU tensors).  Honours the
  reference's ``XLA_FLAGS`` variable for drop-in fidelity, or
  ``LJS_NUM_DEVICES``.
* ``gpu``  - MI355X devices.  Single process: every physical GPU is a device,
  and ``LJS_NUM_DEVICES=N`` larger than the physical count creates *virtual*
  devices mapped round-robin onto the physical GPUs (used to run a 2x2 or 2x4
  mesh on one MI355X).  Multi process (``torchrun``, one rank per GPU, RCCL):
  one device per process, device id == global rank.
* multi-process CPU (gloo) - one host device per rank; used by the CPU test
  suite to exercise the exact code path the 8-GPU RCCL run takes.

Environment variables (read once, at first use):
  LJS_PLATFORM     cpu | gpu  (default: gpu if a GPU is visible else cpu)
  LJS_NUM_DEVICES  number of devices in single-process mode
  XLA_FLAGS        ``--xla_force_host_platform_device_count=N`` (cpu only)
"""
from __future__ import annotations

import os
import re
import threading
from typing import List, Optional

import torch

__all__ = [
    "Device",
    "devices",
    "local_devices",
    "device_count",
    "local_device_count",
    "process_index",
    "process_count",
    "default_backend",
    "is_distributed",
    "reset_backend",
    "initialize_distributed",
]


class Device:
    """One SPMD device.  ``id`` is global; ``torch_device`` is where its shards live."""

    __slots__ = ("id", "platform", "process_index", "torch_device", "physical_index")

    def __init__(self, id: int, platform: str, process_index: int, torch_device: torch.device,
                 physical_index: int):
        self.id = int(id)
        self.platform = platform
        self.process_index = int(process_index)
        self.torch_device = torch_device
        self.physical_index = int(physical_index)

    @property
    def device_kind(self) -> str:
        return "MI355X" if self.platform == "gpu" else "cpu"

    @property
    def label(self) -> str:
        return self.platform.upper()

    def is_addressable(self) -> bool:
        return self.process_index == process_index()

    def __repr__(self) -> str:
        if self.platform == "cpu":
            return f"CpuDevice(id={self.id})"
        return f"RocmDevice(id={self.id})"

    def __hash__(self):
        return hash(("ljs-device", self.id))

    def __eq__(self, other):
        return isinstance(other, Device) and other.id == self.id

    def __lt__(self, other):
        return self.id < other.id


_XLA_COUNT_RE = re.compile(r"--xla_force_host_platform_device_count=(\d+)")


def _xla_flag_count() -> Optional[int]:
    m = _XLA_COUNT_RE.search(os.environ.get("XLA_FLAGS", ""))
    return int(m.group(1)) if m else None


class _Backend:
    def __init__(self):
        platform = os.environ.get("LJS_PLATFORM", "").strip().lower()
        if platform not in ("", "cpu", "gpu"):
            raise ValueError(f"LJS_PLATFORM must be cpu or gpu, got {platform!r}")
        if not platform:
            platform = "gpu" if torch.cuda.is_available() else "cpu"
        if platform == "gpu" and not torch.cuda.is_available():
            raise RuntimeError("LJS_PLATFORM=gpu but no GPU is visible to torch")
        self.platform = platform
        dist = torch.distributed
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if self.distributed:
            world = dist.get_world_size()
            rank = dist.get_rank()
            self.process_index = rank
            self.process_count = world
            devs = []
            for r in range(world):
                if platform == "gpu":
                    local_rank = _local_gpu(r)
                    td = torch.device("cuda", local_rank if r == rank else 0)
                    phys = local_rank if r == rank else -1
                else:
                    td = torch.device("cpu")
                    phys = 0
                devs.append(Device(r, platform, r, td, phys))
            self.devices = devs
        else:
            self.process_index = 0
            self.process_count = 1
            n_env = os.environ.get("LJS_NUM_DEVICES")
            if platform == "cpu":
                n = int(n_env) if n_env else (_xla_flag_count() or 1)
                self.devices = [Device(i, "cpu", 0, torch.device("cpu"), 0) for i in range(n)]
            else:
                phys = torch.cuda.device_count()
                n = int(n_env) if n_env else phys
                self.devices = [
                    Device(i, "gpu", 0, torch.device("cuda", i % phys), i % phys) for i in range(n)
                ]
        self.by_id = {d.id: d for d in self.devices}

    @property
    def local_devices(self) -> List[Device]:
        return [d for d in self.devices if d.process_index == self.process_index]


_LOCK = threading.Lock()
_BACKEND: Optional[_Backend] = None


def _local_gpu(rank: Optional[int] = None) -> int:
    """This process's GPU: LOCAL_RANK, wrapped onto the visible devices (several ranks may
    share one GPU in tests; ``torch.cuda.device_count`` does not initialise the GPU)."""
    n = max(1, torch.cuda.device_count())
    r = int(os.environ.get("LOCAL_RANK", rank if rank is not None else 0))
    return r % n


def initialize_distributed(backend: Optional[str] = None) -> None:
    """Initialise ``torch.distributed`` from the torchrun environment.

    One process per GPU; backend ``nccl`` is RCCL over xGMI on ROCm.  CPU runs
    use ``gloo``.  Safe to call more than once.  Must run before the first
    call to :func:`devices` for the multi-process device map to be used.
    """
    global _BACKEND
    dist = torch.distributed
    if dist.is_initialized():
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return
    platform = os.environ.get("LJS_PLATFORM", "").lower() or ("gpu" if torch.cuda.is_available() else "cpu")
    if backend is None:
        # LJS_DIST_BACKEND=gloo runs GPU ranks over gloo (e.g. several ranks sharing one GPU in
        # tests, which RCCL does not allow)
        backend = os.environ.get("LJS_DIST_BACKEND") or ("nccl" if platform == "gpu" else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import datetime
    # torch's own collectives (barriers, gloo fallbacks) give up after the job's comm timeout too
    kwargs = {"timeout": datetime.timedelta(seconds=float(os.environ.get("LJS_COMM_TIMEOUT_S", "300")))}
    if platform == "gpu":
        torch.cuda.set_device(_local_gpu())
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", _local_gpu())
    if backend == "fake":
        # rehearsal: ONE process plays rank RANK of WORLD_SIZE and every collective completes
        # at once without moving data - the whole multi-rank code path (process groups, grad
        # buckets, segmented graphs, side-stream joins) runs, so its overhead is measurable on
        # one GPU with the network taken out (numerics are NOT those of a real run)
        from torch.testing._internal.distributed.fake_pg import FakeStore
        kwargs.update(store=FakeStore(), rank=int(os.environ.get("RANK", "0")), world_size=world)
    dist.init_process_group(backend=backend, **kwargs)
    with _LOCK:
        _BACKEND = None


def _backend() -> _Backend:
    global _BACKEND
    if _BACKEND is None:
        if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and torch.distributed.is_available()
                and not torch.distributed.is_initialized()
                and os.environ.get("LJS_AUTO_DISTRIBUTED", "1") == "1"):
            # torchrun launch: join the process group before building the device map.
            initialize_distributed()
        with _LOCK:
            if _BACKEND is None:
                _BACKEND = _Backend()
    return _BACKEND


def reset_backend() -> None:
    """Forget the device map (tests use this after changing the environment)."""
    global _BACKEND
    with _LOCK:
        _BACKEND = None
    from ..comm import backend as _cb  # local import: avoid a cycle at import time
    _cb.reset_comm()


def devices() -> List[Device]:
    return list(_backend().devices)


def local_devices() -> List[Device]:
    return _backend().local_devices


def device_count() -> int:
    return len(_backend().devices)


def local_device_count() -> int:
    return len(_backend().local_devices)


def process_index() -> int:
    return _backend().process_index


def process_count() -> int:
    return _backend().process_count


def default_backend() -> str:
    return _backend().platform


def is_distributed() -> bool:
    return _backend().distributed


def get_device(dev_id: int) -> Device:
    return _backend().by_id[int(dev_id)]
