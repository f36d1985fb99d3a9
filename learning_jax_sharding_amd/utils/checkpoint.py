"""Sharded checkpoint / resume (the reference builds a TrainState at
``case6_attention.py:171-178`` but never saves it).

Layout of a checkpoint directory::

    meta.json                 format version, step, one record per leaf: path, shape, dtype,
                              partition spec (when named), tile grid; plain (non-array) leaves
    shards_p{k}.safetensors   the tiles process k is the FIRST holder of (replicas are
                              written once), keyed "<leaf>/<tile index>"
    index_p{k}.json           global slice (start, stop per dim) of every saved tile

Every process writes only its own tiles (no gather, no host copy of remote data); a restore
reads the tile files, assembles each leaf on the host and places it with the TARGET's
sharding - so a run may resume on a different mesh or device count.  Files are written with
``safetensors`` (no pickling anywhere; loading executes nothing from the files).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional

import numpy as np
import torch
from safetensors.torch import load_file, save_file

from ..array import ShardedArray
from ..runtime.devices import process_count, process_index
from . import tree as T

__all__ = ["save_checkpoint", "restore_checkpoint", "latest_step", "checkpoint_dir"]

FORMAT = 1


def _is_arr(x):
    return isinstance(x, ShardedArray)


def _path_str(path) -> str:
    return "/".join(str(p) for p in path)


def _spec_str(sh) -> Optional[List]:
    spec = getattr(sh, "spec", None)
    if spec is None:
        return None
    return [list(e) if isinstance(e, tuple) else e for e in spec]


def checkpoint_dir(root: str, step: int) -> str:
    return os.path.join(root, f"step_{int(step):08d}")


def latest_step(root: str) -> Optional[int]:
    if not os.path.isdir(root):
        return None
    steps = [int(d[5:]) for d in os.listdir(root) if d.startswith("step_") and
             os.path.exists(os.path.join(root, d, "meta.json"))]
    return max(steps) if steps else None


def save_checkpoint(directory: str, tree: Any, step: Optional[int] = None) -> str:
    """Write ``tree`` (e.g. a TrainState) under ``directory`` (created); returns it."""
    os.makedirs(directory, exist_ok=True)
    me = process_index()
    items = T.tree_leaves_with_path(tree, is_leaf=_is_arr)
    tensors: Dict[str, torch.Tensor] = {}
    index: Dict[str, List] = {}
    records = []
    for li, (path, leaf) in enumerate(items):
        if _is_arr(leaf):
            ta = leaf.tile
            records.append({"path": _path_str(path), "kind": "array", "shape": list(leaf.shape),
                            "dtype": str(leaf.dtype).replace("torch.", ""), "spec": _spec_str(leaf.sharding),
                            "tiles": list(ta.tile_shape)})
            for d, t in leaf.local.items():
                tile = ta.coords[d]
                if min(ta.holders(tile)) != d:
                    continue                      # replicas are written once, by the first holder
                sl = ta.indices(d, leaf.shape)
                key = f"{li}/{'_'.join(str(i) for i in tile) or '0'}"
                # own copy: leaves may alias (TrainState.step IS the optimizer's count)
                tensors[key] = t.detach().to("cpu", copy=True).contiguous()
                index[key] = [[s.start or 0, s.stop if s.stop is not None else leaf.shape[k]]
                              for k, s in enumerate(sl)]
        else:
            val = leaf
            if isinstance(val, torch.Tensor):
                val = val.item() if val.numel() == 1 else val.tolist()
            elif isinstance(val, np.generic):
                val = val.item()
            records.append({"path": _path_str(path), "kind": "value", "value": val})
    save_file(tensors, os.path.join(directory, f"shards_p{me}.safetensors"))
    with open(os.path.join(directory, f"index_p{me}.json"), "w") as f:
        json.dump(index, f)
    if me == 0:
        with open(os.path.join(directory, "meta.json"), "w") as f:
            json.dump({"format": FORMAT, "step": step, "processes": process_count(), "leaves": records}, f, indent=1)
    if process_count() > 1 and torch.distributed.is_initialized():
        torch.distributed.barrier()
    return directory


def restore_checkpoint(directory: str, target: Any) -> Any:
    """Load a checkpoint into the structure (and shardings) of ``target``: array leaves of
    ``target`` give the placement, other leaves are replaced by the saved values."""
    with open(os.path.join(directory, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"unsupported checkpoint format {meta.get('format')}")
    records = meta["leaves"]
    items = T.tree_leaves_with_path(target, is_leaf=_is_arr)
    if len(items) != len(records):
        raise ValueError(f"checkpoint has {len(records)} leaves, target has {len(items)}")
    shards: Dict[str, torch.Tensor] = {}
    index: Dict[str, List] = {}
    for k in range(meta["processes"]):
        shards.update(load_file(os.path.join(directory, f"shards_p{k}.safetensors")))
        with open(os.path.join(directory, f"index_p{k}.json")) as f:
            index.update(json.load(f))
    from ..array import device_put
    out_leaves = []
    for li, ((path, leaf), rec) in enumerate(zip(items, records)):
        if _path_str(path) != rec["path"]:
            raise ValueError(f"leaf {li}: checkpoint path {rec['path']!r} != target path {_path_str(path)!r}")
        if rec["kind"] == "value":
            out_leaves.append(rec["value"] if not isinstance(leaf, torch.Tensor) else torch.tensor(rec["value"]))
            continue
        dtype = getattr(torch, rec["dtype"])
        full = torch.empty(rec["shape"], dtype=dtype)
        for key, t in shards.items():
            if key.split("/")[0] != str(li):
                continue
            sl = tuple(slice(a, b) for a, b in index[key])
            full[sl] = t
        if _is_arr(leaf):
            if tuple(leaf.shape) != tuple(rec["shape"]):
                raise ValueError(f"{rec['path']}: saved shape {rec['shape']} != target {tuple(leaf.shape)}")
            out_leaves.append(device_put(full.to(leaf.dtype), leaf.sharding))
        else:
            out_leaves.append(device_put(full))
    td = T.tree_structure(target, is_leaf=_is_arr)
    return T.tree_unflatten(td, out_leaves)
