"""dtype helpers: the framework uses torch dtypes; numpy/JAX-style names are accepted."""
from __future__ import annotations

import numpy as np
import torch

float32 = torch.float32
float16 = torch.float16
bfloat16 = torch.bfloat16
float64 = torch.float64
int32 = torch.int32
int64 = torch.int64
uint32 = torch.uint32 if hasattr(torch, "uint32") else torch.int64
int8 = torch.int8
uint8 = torch.uint8
bool_ = torch.bool
float8_e4m3fn = torch.float8_e4m3fn
float8_e5m2 = torch.float8_e5m2

_NAME = {
    "float32": torch.float32, "f32": torch.float32, "float": torch.float32,
    "float16": torch.float16, "f16": torch.float16, "half": torch.float16,
    "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
    "float64": torch.float64, "f64": torch.float64, "double": torch.float64,
    "int32": torch.int32, "int64": torch.int64, "int8": torch.int8, "uint8": torch.uint8,
    "bool": torch.bool, "float8_e4m3fn": torch.float8_e4m3fn, "float8_e5m2": torch.float8_e5m2,
}


def canonicalize(dtype) -> torch.dtype:
    if dtype is None:
        return None
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(getattr(dtype, "dtype", None), torch.dtype):  # jnp.bfloat16-style scalar types
        return dtype.dtype
    if isinstance(dtype, str):
        return _NAME[dtype]
    if dtype is float:
        return torch.float32
    if dtype is int:
        return torch.int32
    if dtype is bool:
        return torch.bool
    try:
        npd = np.dtype(dtype)
    except TypeError:
        raise TypeError(f"unsupported dtype {dtype!r}")
    if npd.name == "bfloat16":
        return torch.bfloat16
    return _NAME.get(npd.name) or torch.from_numpy(np.zeros(0, npd)).dtype


def to_numpy_dtype(dtype: torch.dtype):
    if dtype == torch.bfloat16:
        return np.float32  # numpy has no bf16; host copies are upcast (exact)
    if dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
        return np.float32
    return torch.empty(0, dtype=dtype).numpy().dtype


def itemsize(dtype: torch.dtype) -> int:
    return torch.empty(0, dtype=dtype).element_size()


def is_floating(dtype: torch.dtype) -> bool:
    return dtype.is_floating_point


def result_type(*dtypes) -> torch.dtype:
    ds = [canonicalize(d) for d in dtypes if d is not None]
    out = ds[0]
    for d in ds[1:]:
        out = torch.promote_types(out, d)
    return out
