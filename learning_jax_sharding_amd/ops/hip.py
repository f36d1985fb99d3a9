"""ctypes bindings of the gfx950 HIP kernel library + autograd wrappers.

The library (``_lib/libljs_kernels.so``, built by ``csrc/build.py``) exposes a plain C
ABI; every launcher takes the current torch HIP stream, so kernels interleave with torch
ops, RCCL collectives and HIP-graph capture.  There is no fallback: if the library is
missing on a GPU machine every op raises (``LJS_ALLOW_TORCH_FALLBACK=1`` is a debugging
escape hatch that routes to the torch reference implementations instead).
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from typing import Dict, List, Optional, Sequence

import torch

__all__ = ["lib", "available", "gemm", "bmm_nt", "linear", "attention", "cast", "sum_all", "softmax_lastdim",
           "adam", "rng_fill", "colsum", "supports_cast"]

_HERE = os.path.dirname(os.path.abspath(__file__))
# LJS_KERNELS_LIB: an alternative build of the library (A/B timing of kernel variants)
_LIBPATH = os.environ.get("LJS_KERNELS_LIB") or os.path.join(os.path.dirname(_HERE), "_lib", "libljs_kernels.so")
_LIB = None
_LOCK = threading.Lock()

c_void_p, c_int, c_long, c_float, c_uint = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_uint
_LP = ctypes.POINTER(ctypes.c_long)

_SIGS = {
    "ljs_pack_rows": [c_void_p, c_int, c_void_p, c_long, c_long, c_long, c_int, c_void_p, c_void_p],
    "ljs_gemm_group_end": [c_void_p],
    "ljs_gemm_bf16": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_long, c_long, c_long, c_long,
                      c_long, c_long, c_long, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_void_p,
                      ctypes.POINTER(c_int), c_void_p, c_long, c_long, c_void_p],
    "ljs_sum_partials": [c_void_p, c_int, c_void_p, c_int, c_void_p],
    "ljs_mse_colsum_ws_bytes": [c_int, c_int],
    "ljs_gemm_f32": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_long, c_long, c_long, c_long, c_long,
                     c_long, c_long, c_long, c_int, c_void_p],
    "ljs_attn_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, _LP, _LP, _LP, _LP,
                     c_float, c_int, c_int, c_void_p],
    "ljs_attn_set_trace": [c_void_p],
    "ljs_qkv_attn_fwd": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                         c_void_p, c_void_p],
    "ljs_attn_fwd_acc": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, _LP, _LP, _LP,
                         _LP, c_float, c_int, c_int, c_void_p, _LP, c_int, c_void_p],
    "ljs_attn_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_int, c_int, c_int, c_int, _LP, _LP, _LP, _LP, _LP, _LP, _LP, _LP, c_float, c_int,
                     c_int, c_void_p],
    "ljs_cast_f32_bf16": [c_void_p, c_void_p, c_long, c_void_p],
    "ljs_cast_bf16_f32": [c_void_p, c_void_p, c_long, c_void_p],
    "ljs_swap01_bf16": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p],
    "ljs_transpose_bf16": [c_void_p, c_void_p, c_int, c_int, c_long, c_long, c_void_p],
    "ljs_sum_n": [ctypes.POINTER(c_void_p), c_int, c_int, c_long, c_void_p, c_void_p],
    "ljs_rows_sum_f32": [c_void_p, c_int, c_int, c_long, c_void_p, c_void_p],
    "ljs_cast_transpose_f32_bf16": [c_void_p, c_void_p, c_int, c_int, c_long, c_long, c_void_p],
    "ljs_sum_all": [c_void_p, c_int, c_long, c_void_p, c_int, c_void_p, c_void_p],
    "ljs_colsum": [c_void_p, c_int, c_int, c_int, c_long, c_void_p, c_int, c_void_p, c_void_p],
    "ljs_fill_row_bf16": [c_void_p, c_int, c_void_p, c_long, c_void_p],
    "ljs_relu_bwd_colsum": [c_void_p, c_void_p, c_int, c_int, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p],
    "ljs_relu_bwd": [c_void_p, c_void_p, c_int, c_int, c_long, c_long, c_void_p, c_void_p],
    "ljs_bcast_scalar": [c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "ljs_pad_box": [c_void_p, c_void_p, c_int, _LP, _LP, _LP, _LP,
                    c_int, c_void_p],
    "ljs_slab_reduce": [c_void_p, c_int, c_long, c_int, c_int, c_void_p, c_int, c_long, c_int, c_void_p, c_void_p,
                        c_void_p, c_int, c_float, c_int, c_void_p],
    "ljs_softmax_rows_f32": [c_void_p, c_void_p, c_long, c_int, c_void_p],
    "ljs_adam_f32": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long,
                     c_float, c_float, c_float, c_float, c_float, c_void_p],
    "ljs_adam_multi": [_LP, c_int, c_void_p, c_int, c_void_p, c_float, c_float, c_float, c_float, c_float,
                       c_void_p, c_void_p, c_long, c_void_p],
    "ljs_step_add": [c_void_p, c_int, c_void_p],
    "ljs_adam_set_rows": [c_int],
    "ljs_clock_probe": [c_void_p, c_void_p, c_uint, c_uint, c_void_p],
    "ljs_mse_loss": [c_void_p, c_void_p, c_int, c_long, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "ljs_mse_colsum": [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_void_p],
    "ljs_rng_fill": [c_void_p, c_int, c_int, _LP, _LP, _LP, c_uint, c_uint, c_int, c_float, c_float, c_float,
                     c_float, c_void_p],
    "ljs_dropout": [c_void_p, c_void_p, c_int, c_int, _LP, _LP, _LP, c_uint, c_uint, c_float, c_void_p],
}


def lib():
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                if not os.path.exists(_LIBPATH):
                    raise RuntimeError(
                        f"HIP kernel library not found at {_LIBPATH}: build it with "
                        "`python -m learning_jax_sharding_amd.csrc.build` (or __graft_entry__.build())")
                L = ctypes.CDLL(_LIBPATH)
                for name, argt in _SIGS.items():
                    fn = getattr(L, name)
                    fn.argtypes = argt
                    fn.restype = c_int
                L.ljs_mse_colsum_ws_bytes.restype = c_long
                _LIB = L
    return _LIB


def set_attention_fwd_resident(waves: int):
    """Forward kernel for key lengths <= 256: 0 = tiled (K/V tiles through registers), 4 or 8 =
    K/V-resident (whole K/V of a head in LDS by one LDS-DMA burst; waves x 16 queries per block),
    -1 = the default (8, or 4 below 256 blocks)."""
    fn = lib().ljs_attn_set_fwd_res
    fn.argtypes = [c_int]
    fn.restype = None
    fn(int(waves))


def set_attention_bwd_kv_dma(enabled: Optional[bool]):
    """Fused short-key backward: K / V land in LDS by LDS-DMA in flight with the first query block
    (True) or through registers (False); None = automatic (LDS-DMA when a block sweeps at most
    128 queries).  Bit-identical either way."""
    fn = lib().ljs_attn_set_bwd_kv_dma
    fn.argtypes = [c_int]
    fn.restype = None
    fn(-1 if enabled is None else int(bool(enabled)))


def set_attention_vst(enabled: Optional[bool]):
    """Attention output row tiles (forward O, backward dK / dV) stored through an LDS image as
    whole 128-byte rows with 16-byte stores (True, the default via None), or per lane as 8-byte
    pieces (False).  Bit-identical either way."""
    fn = lib().ljs_attn_set_vst
    fn.argtypes = [c_int]
    fn.restype = None
    fn(-1 if enabled is None else int(bool(enabled)))


def set_attention_bwd_fused(enabled: Optional[bool]):
    """Select the attention backward for key lengths <= 256: the single-pass fused kernel
    (True), the split dQ + dK/dV kernels (False; always used above 256 keys), or None for the
    automatic choice by grid size (the default)."""
    fn = lib().ljs_attn_set_bwd_fused
    fn.argtypes = [c_int]
    fn.restype = None
    fn(2 if enabled is None else (1 if enabled else 0))


def set_attention_dkv32(enabled: Optional[bool]):
    """Split attention backward with 128-key dK/dV blocks (4 waves x 32 keys): True / None (the
    default) or False (64-key blocks)."""
    fn = lib().ljs_attn_set_dkv32
    fn.argtypes = [c_int]
    fn.restype = None
    fn(-1 if enabled is None else (1 if enabled else 0))


def set_attention_dq32(enabled: Optional[bool]):
    """With 128-key dK/dV blocks: 128-query dQ blocks (True / None, the default) or 64 (False)."""
    fn = lib().ljs_attn_set_dq32
    fn.argtypes = [c_int]
    fn.restype = None
    fn(1 if enabled is None or enabled else 0)


def set_attention_bwd_pair(enabled: Optional[bool]):
    """Split attention backward as ONE launch of dQ and dK/dV blocks (True, the default via
    None) or as two launches ordered by the dQ kernel's delta output (False)."""
    fn = lib().ljs_attn_set_bwd_pair
    fn.argtypes = [c_int]
    fn.restype = None
    fn(1 if enabled is None or enabled else 0)


def available() -> bool:
    try:
        lib()
        return True
    except (RuntimeError, OSError):
        return False


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


_DEBUG_SYNC = os.environ.get("LJS_DEBUG_SYNC", "0") == "1"


def _ck(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    if _DEBUG_SYNC or os.environ.get("LJS_DEBUG_SYNC") == "1":
        from ..profiler import after_kernel
        after_kernel(name)


_WS = {}


def _workspace(dev: torch.device, name: str, nbytes: int) -> torch.Tensor:
    """Persistent zero-initialised per-device scratch for in-launch last-arriver reductions:
    its ticket words are re-armed by the kernels themselves, so no per-call memset.  (Keyed
    by device only: a HIP graph captures on a side stream, and a workspace first created
    inside a capture would replay its zero-fill every step.  The kernels using one
    workspace are never run concurrently on two streams.)"""
    key = (dev.index, name)
    t = _WS.get(key)
    if t is None or t.numel() * 4 < nbytes:
        t = torch.zeros((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        _WS[key] = t
    return t


_COLSUM_WS_BYTES = 4 << 20  # = ljs_colsum_ws_floats() * 4


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _longs(vals) -> ctypes.Array:
    arr = (ctypes.c_long * len(vals))(*[int(v) for v in vals])
    return arr


# ============================================================================ GEMM
# output stores with sc1 (drop the written lines from L2 so the output stream does not evict the
# operand panels that neighbouring blocks re-read)
_GEMM_SC1 = True


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, M: int, N: int, K: int, lda: int, ldb: int, ldc: int,
         a_kc: bool, b_kc: bool, batch: int = 1, sA: int = 0, sB: int = 0, sC: int = 0,
         bias: Optional[torch.Tensor] = None, sBias: int = 0, relu: bool = False, alpha: float = 1.0,
         accumulate: bool = False, splitk: int = 1, tile: Optional[int] = None, a_off: int = 0, b_off: int = 0,
         c_off: int = 0, zero_c: bool = False, psum: Optional[torch.Tensor] = None,
         res: Optional[torch.Tensor] = None, res_ld: int = 0, res_mode: str = "add", sR: int = 0,
         slabs: bool = False, b_list: Optional[Sequence[torch.Tensor]] = None) -> int:
    """Raw launcher.  A/B bf16; C bf16 or f32 (split-K/accumulate need f32 C).

    ``lda``/``ldb`` may be 0 for an operand that repeats one row (a broadcast gradient).
    ``zero_c`` zeroes C inside the launch sequence (needed before split-K accumulation).
    ``psum`` (f32, >= :func:`psum_slots` floats): the LDS-DMA kernels with bf16 output also write
    per-(tile, wave) sums of the stored values there.  Returns the number of partials written
    (0 when the chosen kernel does not produce them).
    ``res`` (bf16 or f32, element [row][col] at ``row * res_ld + col``; ``res_ld`` 0 = one
    broadcast row; bf16 C only) is an epilogue operand: ``res_mode="add"`` adds it as a residual
    (``bf16(bf16(y) + bf16(res))``, bit-exact with the unfused add), ``"mask"`` keeps the outputs
    where ``res > 0`` (a ReLU backward fused into the dX GEMM).
    ``b_list`` (slab mode, batch <= 4): batch b's B operand is ``b_list[b]`` (separate tensors).
    ``slabs`` (f32 C, m/n-contiguous operands, an LDS-DMA tile): split s of batch b's K range
    writes its own slab ``C + (s * batch + b) * sC``; ``splitk`` must be :func:`slab_count`-consistent (the
    last split may run past K, where it reads zeros), so the split need not divide the K-tiles.
    """
    assert A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16, (A.dtype, B.dtype)
    assert not slabs or C.dtype == torch.float32, "split-K slabs are f32"
    out_f32 = C.dtype == torch.float32
    if tile is None:
        tile = pick_tile(M, N, K, batch, a_kc, b_kc, out_f32, splitk, ldc, A.dtype, bias, sBias, relu, accumulate,
                         zero_c, psum, res, slabs, sA, sB, sC, ldb)
    flags = (1 if relu else 0) | (2 if bias is not None else 0) | \
        (4 if (bias is not None and bias.dtype == torch.float32) else 0) | (8 if accumulate else 0) | \
        (16 if zero_c else 0) | (32 if _GEMM_SC1 else 0) | (512 if slabs else 0) | \
        (8192 if (slabs and _SLAB_VST) else 0)
    if res is not None:
        assert not out_f32 and res.dtype in (torch.bfloat16, torch.float32), (C.dtype, res.dtype)
        flags |= (64 if res_mode == "add" else 128) | (256 if res.dtype == torch.float32 else 0)
    if tile is None:
        tile = pick_tile(M, N, K, batch, a_kc, b_kc, out_f32, splitk, ldc)
    eA = A.element_size()
    cnt = c_int(0)
    b_arg = ctypes.c_void_p(B.data_ptr() + b_off * eA)
    if b_list is not None:
        # slab mode over a batch of separate B tensors (each laid out like B): pointers by value
        assert slabs and len(b_list) == batch <= 4 and all(t.dtype == torch.bfloat16 for t in b_list)
        flags |= 4096
        b_keep = (c_void_p * len(b_list))(*[t.data_ptr() + b_off * eA for t in b_list])
        b_arg = ctypes.cast(b_keep, c_void_p)
    rc = lib().ljs_gemm_bf16(ctypes.c_void_p(A.data_ptr() + a_off * eA), b_arg,
                             ctypes.c_void_p(C.data_ptr() + c_off * C.element_size()), _p(bias), M, N, K, lda, ldb,
                             ldc, sA, sB, sC, sBias, batch, int(a_kc), int(b_kc), int(out_f32), flags, alpha,
                             splitk, tile, _p(psum), ctypes.byref(cnt), _p(res), res_ld, sR, _stream(C))
    _ck(rc, "ljs_gemm_bf16")
    return cnt.value


def gemm_group_begin():
    """Open a grouped launch: the plain f32 slab GEMMs (weight gradients) that :func:`gemm` is
    asked for until :func:`gemm_group_end` are recorded instead of launched."""
    fn = lib().ljs_gemm_group_begin
    fn.argtypes = []
    fn.restype = None
    fn()


def gemm_group_end(dev_tensor: torch.Tensor):
    """Launch what the open group recorded on ``dev_tensor``'s current stream: two GEMMs of one
    kernel instance as ONE grid (one block per work item of either; the same kernel body per
    item, so bit-identical to separate launches), anything else one by one."""
    rc = lib().ljs_gemm_group_end(_stream(dev_tensor))
    _ck(rc, "ljs_gemm_group_end")


_LEAN_REQ = 100000  # tile code + _LEAN_REQ: force the lean K-loop kernel (gemm.hip gemm_lean_kernel; A/B),
                    # + 2 * _LEAN_REQ: force the general LDS-DMA kernel


def psum_slots(M: int, N: int, batch: int = 1) -> int:
    """Upper bound on the fused output-sum partials of one bf16 GEMM (128-row tiles, 8 waves)."""
    return -(-M // 128) * -(-N // 128) * batch * 8


# Fused output sums: a bf16 GEMM output registered here (weakly) carries the per-wave sums of
# its values computed in the GEMM epilogue, so a following whole-array sum (the loss y.sum())
# reduces a few thousand partials in one tiny kernel instead of re-reading the output.  The
# entry is used only while the output tensor is alive, unmodified (version counter) and
# summed whole (same storage, numel, contiguous).
_PSUM = {}


def _register_psum(y: torch.Tensor, partials: torch.Tensor, count: int) -> None:
    import weakref
    key = y.data_ptr()
    ref = weakref.ref(y, lambda _r, k=key: _PSUM.pop(k, None) if _PSUM.get(k, (None,))[0] is _r else None)
    _PSUM[key] = (ref, y._version, partials, count, y.numel())


def _psum_for(t: torch.Tensor):
    ent = _PSUM.get(t.data_ptr())
    if ent is None:
        return None
    ref, ver, partials, count, numel = ent
    y = ref()
    if y is None or count <= 0 or t.numel() != numel or not t.is_contiguous() or t._version != ver \
            or y.data_ptr() != t.data_ptr():
        return None
    return partials, count


# 256x128 tile for large k-contiguous bf16 GEMMs: with the DMA pieces issued after each k-step's
# fragment reads it beats the 128x128 x 2/CU kernel at the QKV projection (37.9 vs 40.4 us) and
# the FF up-projection (60.7 vs 65.2 us; scripts/gemm_tiles_out.py)
_TILE_2561 = True
# 256x192 tile (8 waves of 64x96, 2 stages; a weight-major batch folded into one GEMM): fewer DMA
# pieces and fragment reads per MFMA than 256x128, one stage less in flight.  On by default with the
# lean K-loop kernel (round 5: QKV 33.5 vs 39.2 us isolated, B=64 step 0.2124 / 0.2159 vs 0.2250 /
# 0.2189 ms, gpurun_out/r5g)
_TILE_2562 = True
# slab-mode GEMMs: the last item's f32 tile leaves through LDS as whole rows (kSlabVst; the GPU
# tests switch it off to check the per-lane form bit-exact)
_SLAB_VST = True


# 128x160 tiles when they (and not 128x128 tiles) fill whole rounds of 512 resident blocks
_TILE_1602 = True


def pick_tile(M: int, N: int, K: int, batch: int, a_kc: bool, b_kc: bool, out_f32: bool, splitk: int = 1,
              ldc: int = 0, a_dtype=None, bias=None, sBias: int = 0, relu: bool = False, accumulate: bool = False,
              zero_c: bool = False, psum=None, res=None, slabs: bool = False, sA: int = 0, sB: int = 0,
              sC: int = 0, ldb: int = 0) -> int:
    """Kernel/tile choice (measured on MI355X at the bench shapes, ``scripts/gemm_one.py``): the
    LDS-DMA kernels (codes 2562 = 256x192 8 waves, 2561 = 256x128 8 waves, 1602 = 128x160 4 waves,
    1282 = 128x128 4 waves x 2 blocks/CU, ...; the k-contiguous ones run the lean K-loop kernel)
    whenever K is a multiple of 64, else the register-staged 128/64 tiles."""
    tiles128 = -(-M // 128) * -(-N // 128) * batch * max(1, splitk)
    if (_TILE_1602 and K % 64 == 0 and a_kc and b_kc and not out_f32 and splitk <= 1 and N % 160 == 0
            and ldc % 8 == 0 and tiles128 % 512 and (-(-M // 128) * (N // 160) * batch) % 512 == 0):
        return 1602
    if K % 64 == 0 and tiles128 >= 96 and (out_f32 or (N % 8 == 0 and ldc % 8 == 0)):
        if (_TILE_2562 and a_kc and b_kc and not out_f32 and res is None and M >= 4096 and splitk <= 1
                and (N * batch) % 192 == 0 and (batch == 1 or (bias is None and sA == 0 and sB == N * ldb
                                                                and sC == N and ldc == N * batch))):
            return 2562
        if _TILE_2561 and a_kc and b_kc and not out_f32 and M >= 4096 and N * batch >= 1024 and N % 128 == 0:
            return 2561
        if a_kc and b_kc and not out_f32 and tiles128 < 256 and splitk <= 1:
            # under one round of 128x128 blocks (the 2048-token QKV projection: 192 tiles): the
            # 8-wave, 3-stage tile (qkv3 10.3 -> 9.5 us; scripts/gemm_small.py)
            return 12883
        return 1282
    if K % 64 == 0 and a_kc and b_kc and (out_f32 or (N % 8 == 0 and ldc % 8 == 0)):
        # few 128x128 tiles (the 2048-token reference shape): the 64x64 LDS-DMA tile, 4 stages
        # (out-projection 7.8 -> 7.0 us, its dX 8.0 -> 6.3 us vs the register-staged 64x64 tile;
        # scripts/gemm_small.py)
        return 644
    return 128 if tiles128 >= 160 else 64


# ... the slab traffic's weight in the split count of a weight-gradient GEMM launched on its own
# (not paired): its slabs are then always read back by a separate slab_reduce (a data-parallel
# step) or a lone deferred combine, so they weigh more -- dW_o at 16384 tokens 16 splits instead
# of 24: fake-4 dp rehearsal 0.2147-0.2172 vs 0.2211-0.2224 ms x3
# (profiles/r5bm_dw_single_traffic_lines.txt); the pair's model weighs them 1
_DW_SINGLE_TRAFFIC_W = 4.0
_DW_TRAFFIC_W = 1.0


def slab_count(nkt: int, S: int) -> int:
    """Splits actually launched for ``S`` requested over ``nkt`` K-tiles (ceil-sized splits)."""
    kps = -(-nkt // max(1, S))
    return -(-nkt // kps)


def _cus() -> int:
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    except Exception:
        return 256


def _dw_single(K: int, N: int, T: int, traffic_w: Optional[float] = None):
    """(tile, K-chunks, slab mode) of a weight-gradient slab GEMM [K, N] = X^T dY over T tokens.

    T > 4096: 128x128 tiles (2 blocks per CU) in slab mode, the split count chosen by a cost
    model -- rounds of resident blocks x K-tiles per split, plus the slab reduction's extra f32
    traffic -- instead of a power of two dividing the K-tiles: the FF weight gradients (100
    tiles) ran 400 items on 512 block slots (78 %), now 5 x 52 K-tiles = 500 items; dW_o (20
    tiles) 16 x 16 -> 24 x 11.  At T <= 4096 the 8-wave 128x128 tile (one block per CU) in slab
    mode."""
    w = _DW_SINGLE_TRAFFIC_W if traffic_w is None else traffic_w
    if K % 64 or N % 64 or T % 64:
        return 1282, pick_splitk_dma(K, N, T, 1), False, None
    nkt, tiles = T // 64, -(-K // 128) * -(-N // 128)
    best, best_cost = 1, None
    if T > 4096:
        slots = 2 * _cus()
        for S in range(1, min(64, nkt) + 1):
            if slab_count(nkt, S) != S:
                continue
            kps = -(-nkt // S)
            # ~1.2 us per K-tile round of a full chip of 128x128 blocks, ~1 us per round of
            # prologue/epilogue, and the reduction reads each f32 slab once (~5 TB/s)
            rounds = -(-tiles * S // slots)
            cost = rounds * (kps * 1.2 + 1.0) + w * S * K * N * 4 / 5e6
            if best_cost is None or cost < best_cost - 1e-9:
                best, best_cost = S, cost
        return 1282, best, True, best_cost
    # T <= 4096: 8-wave 128x128, 4 stages, one block per CU, uneven slab splits (0.1033-0.1053 ms
    # vs 0.1071-0.1076 for the 64x64 tile with power-of-two batched slabs at B = 8)
    for S in range(1, min(32, nkt) + 1):
        if slab_count(nkt, S) != S:
            continue
        cost = -(-tiles * S // _cus()) * (-(-nkt // S) * 1.2 + 1.0) + w * S * K * N * 4 / 5e6
        if best_cost is None or cost < best_cost - 1e-9:
            best, best_cost = S, cost
    return 12884, best, True, best_cost


def pick_dw_slabs(K: int, N: int, T: int):
    """(tile, K-chunks, slab mode) of a weight-gradient slab GEMM (see :func:`_dw_single`, which
    also returns the cost model's estimate in us, or None where no model applies)."""
    return _dw_single(K, N, T)[:3]


_PAIR_PICKS: Dict[tuple, Optional[tuple]] = {}
# "S0,S1[,tile]": force the pair's split counts (tests)
_DW_PAIR = ""


def pick_dw_pair(K0: int, N0: int, K1: int, N1: int, T: int):
    """(tile, S0, S1) for two weight-gradient slab GEMMs [K, N] over the same T tokens launched
    as ONE grid (ops.linear._hold_dw), or None when no pair of split counts fits one round of
    resident blocks or the two separate launches' estimate (:func:`_dw_single`) is lower.

    The 128x128 tile at 2 blocks per CU; the pair's items all start together, so the grid takes
    about its LONGEST item (~1.2 us per K-tile + ~1 us prologue / epilogue) plus the slab traffic
    (written here, read back by the combine or the fused Adam, ~5 TB/s) -- minimised over split
    pairs with tiles0 * S0 + tiles1 * S1 <= resident slots.  At the step shapes (dW_o 20 tiles,
    dW_qkv 60): 6 + 6 splits, 480 items of 43 K-tiles at T = 16384: 52.1 us for the pair vs 59.7
    for the 24 + 8-split launches back to back, and half the slab bytes
    (profiles/r5ah_dw_pair_probe.txt).  The FF block's pair (two 100-tile GEMMs) would need
    items of 128 K-tiles for one round and stays separate (bf16 layer 0.6475 / 0.6503 ms paired vs
    0.6314 / 0.6333, profiles/r5an_layer_pair_lines.txt)."""
    tiles0, size0 = -(-K0 // 128) * -(-N0 // 128), K0 * N0
    tiles1, size1 = -(-K1 // 128) * -(-N1 // 128), K1 * N1
    key = (K0, N0, K1, N1, T, _cus())
    if key in _PAIR_PICKS:
        return _PAIR_PICKS[key]
    nkt = T // 64
    # T <= 4096: the 8-wave 128x128 tile at one block per CU, as for a single weight gradient there
    # (B = 8 pair at 3 + 3 splits: 12.66 us vs 14.49 for the 1282 pair at 6 + 6, and half the slabs;
    # at T = 16384 72.0 vs 53.8, profiles/r5au_dw_pair_8w_probe.txt)
    tile, slots = (12884, _cus()) if T <= 4096 else (1282, 2 * _cus())
    best, best_cost = None, None
    if _DW_PAIR:
        v = [int(t) for t in _DW_PAIR.split(",")]
        best = (v[2] if len(v) > 2 else tile, slab_count(nkt, v[0]), slab_count(nkt, v[1]))
    else:
        for s0 in range(1, min(64, nkt) + 1):
            if tiles0 * s0 > slots:
                break
            if slab_count(nkt, s0) != s0:
                continue
            for s1 in range(1, min(64, nkt) + 1):
                if tiles0 * s0 + tiles1 * s1 > slots:
                    break
                if slab_count(nkt, s1) != s1:
                    continue
                kps = max(-(-nkt // s0), -(-nkt // s1))
                cost = kps * 1.2 + 1.0 + _DW_TRAFFIC_W * (s0 * size0 + s1 * size1) * 4 / 5e6
                if best_cost is None or cost < best_cost - 1e-9:
                    best, best_cost = (tile, s0, s1), cost
        c0, c1 = _dw_single(K0, N0, T, _DW_TRAFFIC_W)[3], _dw_single(K1, N1, T, _DW_TRAFFIC_W)[3]
        if best is not None and c0 is not None and c1 is not None and c0 + c1 <= best_cost:
            best = None
    _PAIR_PICKS[key] = best
    return best


def pick_splitk_dma(M: int, N: int, K: int, batch: int) -> int:
    """Split of the reduction for the 128x128 LDS-DMA kernel (weight-grad GEMMs): a divisor of
    the K-tiles giving ~512 work items (2 resident blocks per CU on 256 CUs), >= 4 K-tiles each."""
    if K % 64:
        return 1
    nkt = K // 64
    tiles = -(-M // 128) * -(-N // 128) * batch
    if tiles >= 384:
        return 1
    best, score = 1, None
    for s in range(1, min(16, nkt // 4) + 1):
        if nkt % s:
            continue
        sc = abs(tiles * s - 512)
        if score is None or sc < score:
            best, score = s, sc
    return best


def _choose_splitk(M: int, N: int, K: int, batch: int) -> int:
    """Split the reduction when the output tiles cannot fill MI355X's 256 CUs (weight-grad GEMMs)."""
    tiles = -(-M // 64) * -(-N // 64) * batch
    if tiles >= 256:
        return 1
    s = max(1, min(16, 512 // max(1, tiles), K // 512))
    return s


def _bmm_raw(A, B, out_dtype, a_kc, b_kc, M, N, K, batch, lda, ldb, sA, sB):
    C = torch.empty((batch, M, N), dtype=out_dtype, device=A.device)
    gemm(A, B, C, M, N, K, lda, ldb, N, a_kc, b_kc, batch, sA, sB, M * N)
    return C


def _gemm_f32(A, B, C, M, N, K, a_rs, a_cs, b_rs, b_cs, c_rs, sA, sB, sC, batch):
    rc = lib().ljs_gemm_f32(_p(A), _p(B), _p(C), M, N, K, a_rs, a_cs, b_rs, b_cs, c_rs, sA, sB, sC, batch,
                            _stream(C))
    _ck(rc, "ljs_gemm_f32")


class _BmmNT(torch.autograd.Function):
    """C[b] = A[b] @ Bt[b]^T for A (B,M,K), Bt (B,N,K)."""

    @staticmethod
    def forward(ctx, A, Bt, out_dtype):
        ctx.save_for_backward(A, Bt)
        ctx.out_dtype = out_dtype
        return _bmm_nt_fwd(A, Bt, out_dtype)

    @staticmethod
    def backward(ctx, dC):
        A, Bt = ctx.saved_tensors
        dC = dC.contiguous()
        dA = dB = None
        if ctx.needs_input_grad[0]:
            dA = _bmm_nn(dC.to(A.dtype) if A.dtype != dC.dtype else dC, Bt, A.dtype)       # dC @ Bt
        if ctx.needs_input_grad[1]:
            dB = _bmm_tn(dC.to(Bt.dtype) if Bt.dtype != dC.dtype else dC, A, Bt.dtype)     # dC^T @ A
        return dA, dB, None


def _bmm_nt_fwd(A, Bt, out_dtype):
    Bn, M, K = A.shape
    N = Bt.shape[1]
    if A.dtype == torch.float32 and Bt.dtype == torch.float32:
        A = A.contiguous()
        Bt = Bt.contiguous()
        C = torch.empty((Bn, M, N), dtype=torch.float32, device=A.device)
        _gemm_f32(A, Bt, C, M, N, K, K, 1, 1, K, N, M * K, N * K, M * N, Bn)
        return C.to(out_dtype)
    A = A.to(torch.bfloat16).contiguous()
    Bt = Bt.to(torch.bfloat16).contiguous()
    if K % 8:
        # pad the contraction to the kernel's 16-byte granularity
        pad = 8 - K % 8
        A = torch.nn.functional.pad(A, (0, pad))
        Bt = torch.nn.functional.pad(Bt, (0, pad))
        K += pad
    od = out_dtype if out_dtype in (torch.bfloat16, torch.float32) else torch.float32
    C = _bmm_raw(A, Bt, od, True, True, M, N, K, Bn, K, K, M * K, N * K)
    return C.to(out_dtype)


def _bmm_nn(dC, Bt, out_dtype):
    """(B,M,N) @ (B,N,K) -> (B,M,K)."""
    Bn, M, N = dC.shape
    K = Bt.shape[2]
    if dC.dtype == torch.float32:
        out = torch.empty((Bn, M, K), dtype=torch.float32, device=dC.device)
        _gemm_f32(dC, Bt.contiguous(), out, M, K, N, N, 1, K, 1, K, M * N, N * K, M * K, Bn)
        return out.to(out_dtype)
    if N % 8 == 0 and K % 8 == 0:
        # B[k=n][n'=k] = Bt[n][k] is n'-contiguous: read in place through the transposing LDS read
        dC = dC.to(torch.bfloat16).contiguous()
        od = out_dtype if out_dtype in (torch.bfloat16, torch.float32) else torch.float32
        out = torch.empty((Bn, M, K), dtype=od, device=dC.device)
        gemm(dC, Bt.to(torch.bfloat16).contiguous(), out, M, K, N, N, K, K, True, False, Bn, M * N, N * K, M * K)
        return out.to(out_dtype)
    return _bmm_nt_fwd(dC, Bt.transpose(1, 2).contiguous(), out_dtype)


def _bmm_tn(dC, A, out_dtype):
    """(B,M,N)^T @ (B,M,K) -> (B,N,K)."""
    Bn, M, N = dC.shape
    K = A.shape[2]
    if dC.dtype == torch.float32:
        out = torch.empty((Bn, N, K), dtype=torch.float32, device=dC.device)
        _gemm_f32(dC, A.contiguous(), out, N, K, M, 1, N, K, 1, K, M * N, M * K, N * K, Bn)
        return out.to(out_dtype)
    if N % 8 == 0 and K % 8 == 0 and M % 8 == 0:
        out = torch.empty((Bn, N, K), dtype=torch.float32 if out_dtype == torch.float32 else torch.bfloat16,
                          device=dC.device)
        gemm(dC.to(torch.bfloat16).contiguous(), A.to(torch.bfloat16).contiguous(), out, N, K, M, N, K, K, False,
             False, Bn, M * N, M * K, N * K)
        return out.to(out_dtype)
    return _bmm_nt_fwd(dC.transpose(1, 2).contiguous(), A.transpose(1, 2).contiguous(), out_dtype)


def bmm_nt(A: torch.Tensor, Bt: torch.Tensor, out_dtype: torch.dtype) -> torch.Tensor:
    return _BmmNT.apply(A, Bt, out_dtype)


# ============================================================================ casts
def supports_cast(src: torch.dtype, dst: torch.dtype) -> bool:
    return (src, dst) in ((torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32))


class _Cast(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dtype):
        ctx.src = t.dtype
        return _cast_raw(t, dtype)

    @staticmethod
    def backward(ctx, g):
        return _cast_raw(g.contiguous(), ctx.src) if supports_cast(g.dtype, ctx.src) else g.to(ctx.src), None


def _cast_raw(t: torch.Tensor, dtype: torch.dtype, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``t`` in ``dtype`` by one HIP launch (into ``out``, a contiguous tensor of t's shape, when
    given: a persistent buffer - e.g. a weight's bf16 shadow - is refreshed in place)."""
    if out is not None and not (t.dtype != dtype and supports_cast(t.dtype, dtype) and t.is_contiguous()
                                and out.is_contiguous() and out.dtype == dtype and out.shape == t.shape):
        out.copy_(t)
        return out
    if t.dtype == dtype:
        return t
    if not supports_cast(t.dtype, dtype) or not t.is_contiguous():
        return t.to(dtype)
    if out is None:
        out = torch.empty(t.shape, dtype=dtype, device=t.device)
    n = t.numel()
    if n == 0:
        return out
    if t.dtype == torch.float32:
        rc = lib().ljs_cast_f32_bf16(_p(t), _p(out), n, _stream(t))
    else:
        rc = lib().ljs_cast_bf16_f32(_p(t), _p(out), n, _stream(t))
    _ck(rc, "cast")
    return out


def swap01_bf16(x: torch.Tensor) -> torch.Tensor:
    """bf16 [S][B][K] (contiguous) from a contiguous f32 / bf16 [B][S][K]: the seq-major copy of
    an activation, rounded in the same pass (one HIP launch)."""
    B, S, K = x.shape
    out = torch.empty((S, B, K), dtype=torch.bfloat16, device=x.device)
    rc = lib().ljs_swap01_bf16(_p(x), int(x.dtype == torch.bfloat16), _p(out), B, S, K, _stream(x))
    _ck(rc, "swap01_bf16")
    return out


def sum_n(ts: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Elementwise sum of same-shape dense f32 / bf16 tensors on one GPU (f32 accumulation) in one
    launch - the loopback reduction over virtual devices.  Falls back to torch adds otherwise."""
    t0 = ts[0]
    ok = (t0.is_cuda and t0.dtype in (torch.float32, torch.bfloat16) and 1 <= len(ts) <= 128
          and all(t.shape == t0.shape and t.dtype == t0.dtype and t.device == t0.device and is_dense(t)
                  and t.stride() == t0.stride() and t.data_ptr() % 16 == 0 for t in ts))
    if not ok:
        acc = None
        for t in ts:
            v = t.float()
            acc = v if acc is None else acc + v
        return acc.to(t0.dtype)
    if out is None:
        out = torch.empty_like(t0)
    arr = (c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    rc = lib().ljs_sum_n(arr, len(ts), int(t0.dtype == torch.bfloat16), t0.numel(), _p(out), _stream(t0))
    _ck(rc, "sum_n")
    return out


def rows_sum(t2d: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """f32 [C] = sum over the rows of a SHORT f32 [R][C] (e.g. per-row-tile partial column sums a
    GEMM epilogue wrote): one memory round trip (rows_sum_f32_kernel); torch on the CPU."""
    R, C = t2d.shape
    if not t2d.is_cuda:
        s = t2d.float().sum(0)
        return s if out is None else out.copy_(s)
    assert t2d.dtype == torch.float32 and t2d.stride(1) == 1
    if out is None:
        out = torch.empty((C,), dtype=torch.float32, device=t2d.device)
    rc = lib().ljs_rows_sum_f32(_p(t2d), R, C, t2d.stride(0), _p(out), _stream(t2d))
    _ck(rc, "rows_sum_f32")
    return out


def sum_ptrs(ptrs: Sequence[int], out: torch.Tensor) -> torch.Tensor:
    """out (dense f32 / bf16) = sum of ``len(ptrs)`` <= 128 dense arrays of out's dtype and element
    count at the given device addresses (16-byte aligned) - e.g. every device's split-K weight
    gradient slabs, summed in one pass (parallel/weight_gather.py)."""
    assert 1 <= len(ptrs) <= 128 and out.is_cuda and is_dense(out) and all(p % 16 == 0 for p in ptrs)
    arr = (c_void_p * len(ptrs))(*ptrs)
    rc = lib().ljs_sum_n(arr, len(ptrs), int(out.dtype == torch.bfloat16), out.numel(), _p(out), _stream(out))
    _ck(rc, "sum_n")
    return out


def transpose_bf16(t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[C][R] bf16 transpose of a bf16 [R][C] matrix (unit column stride), one HIP launch."""
    R, C = t.shape
    assert t.dtype == torch.bfloat16 and t.stride(1) == 1
    if out is None:
        out = torch.empty((C, R), dtype=torch.bfloat16, device=t.device)
    rc = lib().ljs_transpose_bf16(_p(t), _p(out), R, C, t.stride(0), out.stride(0), _stream(t))
    _ck(rc, "transpose_bf16")
    return out


def cast_into(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst[...] = src converted to dst.dtype (f32 <-> bf16 on the HIP kernel; both contiguous)."""
    assert src.numel() == dst.numel() and dst.is_contiguous(), (src.shape, dst.shape)
    if src.dtype == dst.dtype:
        dst.copy_(src)
        return dst
    if not supports_cast(src.dtype, dst.dtype) or not src.is_contiguous() or not dst.is_cuda:
        dst.copy_(src.reshape(dst.shape))
        return dst
    n = src.numel()
    if n:
        fn = lib().ljs_cast_f32_bf16 if src.dtype == torch.float32 else lib().ljs_cast_bf16_f32
        _ck(fn(_p(src), _p(dst), n, _stream(dst)), "cast")
    return dst


def cast(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if t.requires_grad and torch.is_grad_enabled():
        return _Cast.apply(t, dtype)
    return _cast_raw(t, dtype)


def cast_transpose_bf16(w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 W^T ([N][K]) from an f32 [K][N] matrix (row stride w.stride(0))."""
    K, N = w.shape
    assert w.dtype == torch.float32 and w.stride(1) == 1
    if out is None:
        out = torch.empty((N, K), dtype=torch.bfloat16, device=w.device)
    rc = lib().ljs_cast_transpose_f32_bf16(_p(w), _p(out), K, N, w.stride(0), out.stride(0), _stream(w))
    _ck(rc, "cast_transpose")
    return out


# ============================================================================ reductions
def _sum_all_raw(t: torch.Tensor, out_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    t = t.contiguous()
    out_bf16 = out_dtype == torch.bfloat16 and t.data_ptr() % 16 == 0
    out = torch.empty((), dtype=torch.bfloat16 if out_bf16 else torch.float32, device=t.device)
    ps = _psum_for(t)
    if ps is not None:  # the producing GEMM already summed its output tile by tile
        rc = lib().ljs_sum_partials(_p(ps[0]), ps[1], _p(out), int(out_bf16), _stream(t))
        _ck(rc, "sum_partials")
        return out
    ws = _workspace(t.device, "sum_all", 1089 * 4)
    rc = lib().ljs_sum_all(_p(t), int(t.dtype == torch.bfloat16), t.numel(), _p(out), int(out_bf16), _p(ws),
                           _stream(t))
    _ck(rc, "sum_all")
    return out


# constant f32 gradient seeds (spmd.api._seed) -> their bf16 rounding, so the backward of a bf16
# sum fed by a cached seed needs no cast kernel
_SEEDS_BF16 = {}


def register_seed_bf16(seed: torch.Tensor, seed_bf16: torch.Tensor, value: Optional[float] = None) -> None:
    _SEEDS_BF16[seed.data_ptr()] = (seed, seed_bf16)
    if value is not None:
        bv = float(torch.tensor(value, dtype=torch.float32).to(torch.bfloat16).float())
        _SEED_CONST[seed.data_ptr()] = (seed, bv)
        _SEED_CONST[seed_bf16.data_ptr()] = (seed_bf16, bv)


def register_seed_const(seed: torch.Tensor, value: float) -> None:
    """A cached 1-element bf16 seed holding bf16(value) (spmd.api._seed)."""
    assert seed.dtype == torch.bfloat16 and seed.numel() == 1
    _SEED_CONST[seed.data_ptr()] = (seed, float(torch.tensor(value, dtype=torch.float32).to(torch.bfloat16).float()))


# constant seeds -> bf16(value) known on the host: a dense layer fed by one (the cotangent of a
# loss sum) takes its broadcast dY row from a cached constant and writes its bias gradient
# R * bf16(g) inside the weight-gradient combine -- no launch of its own (bcast_scalar)
_SEED_CONST = {}
_CONST_ROWS = {}


def seed_constant(g: torch.Tensor) -> Optional[float]:
    """bf16(value) of ``g`` when it is (a 1-element view of) a registered constant seed."""
    ent = _SEED_CONST.get(g.data_ptr())
    if ent is not None and ent[0].data_ptr() == g.data_ptr() and ent[0].dtype == g.dtype and ent[0].numel() == 1:
        return ent[1]
    return None


def const_row_bf16(value: float, n: int, device) -> Optional[torch.Tensor]:
    """A cached bf16 [n] row filled with ``value`` (None while a graph capture is running and
    the row does not exist yet: it is never allocated from a capture's private pool)."""
    key = (value, n, str(device))
    row = _CONST_ROWS.get(key)
    if row is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        row = torch.full((n,), value, dtype=torch.bfloat16, device=device)
        _CONST_ROWS[key] = row
    return row


def _seed_bf16(g: torch.Tensor) -> torch.Tensor:
    ent = _SEEDS_BF16.get(g.data_ptr())
    if ent is not None and ent[0].data_ptr() == g.data_ptr() and ent[0].numel() == 1:
        return ent[1].reshape(())
    return _cast_raw(g.reshape(1), torch.bfloat16).reshape(())


class _SumAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, acc_dtype):
        ctx.shape, ctx.dtype = t.shape, t.dtype
        r = _sum_all_raw(t, acc_dtype)
        return r if r.dtype == acc_dtype else r.to(acc_dtype)

    @staticmethod
    def backward(ctx, g):
        if ctx.dtype == torch.bfloat16 and g.dtype in (torch.bfloat16, torch.float32) and g.is_cuda \
                and g.numel() == 1 and len(ctx.shape) >= 1:
            # the scalar itself, broadcast with all strides 0: a dense layer's backward turns it
            # into its bf16 row + bias gradient in one launch (bcast_scalar).  An f32 seed (the
            # f32 partial sum of a sharded loss) is rounded to bf16 first (one 1-element cast).
            gb = g.reshape(()) if g.dtype == torch.bfloat16 else _seed_bf16(g)
            return gb.expand(ctx.shape), None
        if ctx.dtype == torch.bfloat16 and g.dtype in (torch.float32, torch.bfloat16) and g.is_cuda \
                and len(ctx.shape) >= 1:
            # one bf16 row holding g, broadcast (stride 0) over every leading dim: the consumers
            # (GEMMs, column sums) read it with ld = 0 and nothing of the full shape is written
            n = ctx.shape[-1]
            row = torch.empty((n,), dtype=torch.bfloat16, device=g.device)
            rc = lib().ljs_fill_row_bf16(_p(g), int(g.dtype == torch.bfloat16), _p(row), n, _stream(g))
            _ck(rc, "fill_row")
            return row.expand(ctx.shape), None
        return g.to(ctx.dtype).expand(ctx.shape), None


def sum_all(t: torch.Tensor, acc_dtype: torch.dtype) -> torch.Tensor:
    if t.dtype not in (torch.float32, torch.bfloat16):
        return t.sum(dtype=acc_dtype)
    return _SumAll.apply(t, acc_dtype)


# gradients whose column sums a producer already computed (the fused MSE): data_ptr ->
# (weakref, version, f32 [C] sums); the dense backward takes its bias gradient from here
_COLSUMS = {}


def register_colsum(g: torch.Tensor, sums: torch.Tensor) -> None:
    import weakref
    key = g.data_ptr()
    ref = weakref.ref(g, lambda _r, k=key: _COLSUMS.pop(k, None) if _COLSUMS.get(k, (None,))[0] is _r else None)
    _COLSUMS[key] = (ref, g._version, sums, g.numel())


def colsum_for(t: torch.Tensor, C: int) -> Optional[torch.Tensor]:
    """Precomputed column sums of the [R][C] gradient ``t`` (any view of the registered storage
    with the same element count), or None."""
    ent = _COLSUMS.get(t.data_ptr())
    if ent is None:
        return None
    g = ent[0]()
    if g is None or g._version != ent[1] or ent[3] != t.numel():
        return None
    sums = ent[2]() if callable(ent[2]) else ent[2]   # (a lazy reduction, computed on first use)
    return sums if sums.numel() == C else None


class _MSELoss(torch.autograd.Function):
    """scale * sum((y - t)^2) of one shard (bf16 y, f32 / bf16 t).  When y needs a gradient the
    SAME kernel pass writes dY = bf16(2 * scale * (y - t)) and dY's column sums - the bias gradient
    of the dense layer that produced y (csrc/kernels/loss.hip): the loss's backward is then free
    for the constant seed grad() feeds it, a scalar multiply otherwise."""

    @staticmethod
    def forward(ctx, y, t, scale):
        want_dy = ctx.needs_input_grad[0]
        order = storage_order(y)
        if order is None or order[-1] != y.dim() - 1:
            y, order = y.contiguous(), tuple(range(y.dim()))
        yp = y.permute(order)                                    # contiguous: y's storage order
        tp = t.permute(order).contiguous()                       # the target in the same order
        out = torch.empty((), dtype=torch.float32, device=y.device)
        dy = torch.empty_like(yp).permute(_inv(order)) if want_dy else None
        C = y.shape[-1]
        R = y.numel() // max(1, C)
        sums = None
        if want_dy and C % 64 == 0 and y.dim() >= 2:
            sums = torch.empty((C,), dtype=torch.float32, device=y.device)
            nb = lib().ljs_mse_colsum_ws_bytes(R, C)
            # keyed by geometry: the ticket words sit at an offset that depends on (R, C), so a
            # workspace shared across geometries could hand a call a non-zero "ticket" left in
            # another call's partial-sum area (the last arriver would never be found)
            ws = _workspace(y.device, f"mse_colsum/{R}x{C}", nb)
            rc = lib().ljs_mse_colsum(_p(yp), _p(tp), int(tp.dtype == torch.bfloat16), R, C, float(scale), _p(dy),
                                      _p(sums), _p(out), _p(ws), _stream(y))
            _ck(rc, "mse_colsum")
        else:
            ws = _workspace(y.device, "mse", (1024 + 33) * 4)
            rc = lib().ljs_mse_loss(_p(yp), _p(tp), int(tp.dtype == torch.bfloat16), y.numel(), float(scale),
                                    _p(dy), _p(out), _p(ws), _stream(y))
            _ck(rc, "mse_loss")
        ctx.save_for_backward(dy, sums)
        ctx.t_dtype = t.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        dy, sums = ctx.saved_tensors
        if dy is None:
            return None, None, None
        if seed_constant(g) == 1.0:
            gy = dy
            if sums is not None:
                register_colsum(gy, sums)
        else:
            gy = (dy.float() * g.float()).to(dy.dtype)
        gt = (-gy).to(ctx.t_dtype) if ctx.needs_input_grad[1] else None
        return gy, gt, None


def mse_loss(y: torch.Tensor, t: torch.Tensor, scale: float) -> torch.Tensor:
    ok = (y.dtype == torch.bfloat16 and t.dtype in (torch.float32, torch.bfloat16) and y.shape == t.shape
          and y.data_ptr() % 16 == 0 and t.data_ptr() % 16 == 0 and y.shape[-1] % 8 == 0)
    if not ok:
        return ((y.float() - t.float()) ** 2).sum() * scale
    return _MSELoss.apply(y, t, scale)


def colsum(t2d: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    R, C = t2d.shape
    if t2d.stride(1) != 1:
        t2d = t2d.contiguous()
    if out is None:
        out = torch.empty((C,), dtype=torch.float32, device=t2d.device)
    ws = _workspace(t2d.device, "colsum", _COLSUM_WS_BYTES)
    rc = lib().ljs_colsum(_p(t2d), int(t2d.dtype == torch.bfloat16), R, C, t2d.stride(0), _p(out), int(accumulate),
                          _p(ws), _stream(t2d))
    _ck(rc, "colsum")
    return out


class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        L = x.shape[-1]
        rc = lib().ljs_softmax_rows_f32(_p(x), _p(y), x.numel() // L, L, _stream(x))
        _ck(rc, "softmax")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return y * (dy - (dy * y).sum(-1, keepdim=True))


def softmax_lastdim(x: torch.Tensor) -> torch.Tensor:
    return _Softmax.apply(x)


# ============================================================================ dense / linear
def linear(x: torch.Tensor, ws: List[torch.Tensor], b: Optional[torch.Tensor], compute_dtype: torch.dtype,
           relu: bool, out_dtype: torch.dtype, residual: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    """Fused dense layer (see :mod:`.linear`).  Every GPU shape runs on a HIP GEMM:

    * bf16 compute, K and N multiples of 8, f32 row-major kernels: the fused MFMA path;
    * bf16 compute otherwise: the same path on zero-padded operands (rows M, K and N up to the
      next multiple of 8; zero rows/columns change no sum), result sliced back;
    * f32 compute: the MFMA ``v_mfma_f32_16x16x4f32`` GEMM (:class:`_MatmulF32`, strided
      operands, its own backward), bias and ReLU as elementwise epilogues.

    ``residual`` (same shape as the output) is added after the activation - in the GEMM
    epilogue on the fused path.

    Anything else raises unless ``LJS_ALLOW_TORCH_FALLBACK=1`` (debugging only)."""
    from . import linear as _lin
    if compute_dtype == torch.bfloat16 and _lin.supported(x, ws, b):
        return _lin.linear(x, list(ws), b, relu, out_dtype, residual=residual)
    from . import shadow
    if any(shadow.is_proxy(w) for w in ws):
        # a gathered-weight proxy holds no f32 values; a shape the fused path does not take (M, K
        # or N not a multiple of 8) reads the f32 values bf16(w) recovered from the gathered bf16
        # copy - exactly what a bf16-compute GEMM would round the f32 weight to
        ws = [_ProxyValues.apply(w) if shadow.is_proxy(w) else w for w in ws]
    outs = _linear_any(x, ws, b, compute_dtype, relu, out_dtype)
    if residual is not None:
        outs = [outs[0] + residual.to(outs[0].dtype)] + outs[1:]
    return outs


class _ProxyValues(torch.autograd.Function):
    """f32 values of a gathered-weight proxy (``parallel/weight_gather.py``) from its gathered bf16
    copy (the "T" shadow, [N][K]); the gradient passes through unchanged to the proxy, whose
    backward reduce-scatters it onto the shards."""

    @staticmethod
    def forward(ctx, w):
        from . import shadow
        return shadow.get(w, "T").t().float().contiguous()

    @staticmethod
    def backward(ctx, g):
        return g


def _linear_any(x, ws, b, compute_dtype, relu, out_dtype):
    from . import linear as _lin
    if compute_dtype == torch.bfloat16:
        if all(w.dim() == 2 and w.shape == ws[0].shape and w.dtype == torch.float32 for w in ws) \
                and (b is None or len(ws) == 1):
            return _linear_padded(x, ws, b, relu, out_dtype)
    elif compute_dtype == torch.float32:
        outs = []
        for w in ws:
            lead = x.shape[:-1]
            y = _MatmulF32.apply(x.reshape(-1, x.shape[-1]).float(), w.float())
            if b is not None and len(ws) == 1:
                y = y + b.float()
            if relu:
                y = torch.relu(y)
            outs.append(y.to(out_dtype).reshape(tuple(lead) + (w.shape[-1],)))
        return outs
    if os.environ.get("LJS_ALLOW_TORCH_FALLBACK", "0") != "1":
        raise NotImplementedError(f"no HIP dense path for compute dtype {compute_dtype}, x {tuple(x.shape)}, "
                                  f"w {[tuple(w.shape) for w in ws]} (LJS_ALLOW_TORCH_FALLBACK=1 to use torch)")
    return [_torch_linear(x, w, b if len(ws) == 1 else None, compute_dtype, relu, out_dtype) for w in ws]


def _linear_padded(x, ws, b, relu, out_dtype):
    """bf16 MFMA dense on operands zero-padded to M, K, N multiples of 8 (autograd flows through
    the pads and slices, so the gradients of x, w and b are those of the unpadded layer)."""
    from . import linear as _lin
    K, N = ws[0].shape
    lead = x.shape[:-1]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    pm, pk, pn = (-M) % 8, (-K) % 8, (-N) % 8
    xp = torch.nn.functional.pad(x2, (0, pk, 0, pm)) if (pk or pm) else x2
    wps = [torch.nn.functional.pad(w, (0, pn, 0, pk)).contiguous() if (pk or pn) else w.contiguous() for w in ws]
    bp = torch.nn.functional.pad(b, (0, pn)) if (b is not None and pn) else b
    outs = _lin.linear(xp, wps, bp, relu, out_dtype)
    return [o[:M, :N].reshape(tuple(lead) + (N,)) for o in outs]


class _MatmulF32(torch.autograd.Function):
    """``x [M, K] @ w [K, N]`` in f32 on the MFMA f32 GEMM; backward dx = dy w^T, dw = x^T dy on
    the same kernel through transposed strides (nothing is copied)."""

    @staticmethod
    def forward(ctx, x, w):
        x = x.contiguous()
        w = w.contiguous()
        M, K = x.shape
        N = w.shape[1]
        ctx.save_for_backward(x, w)
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        _gemm_f32(x, w, y, M, N, K, K, 1, N, 1, N, 0, 0, 0, 1)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous().float()
        M, K = x.shape
        N = w.shape[1]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), dtype=torch.float32, device=x.device)
            _gemm_f32(dy, w, dx, M, K, N, N, 1, 1, N, K, 0, 0, 0, 1)       # B[n][k] = w[k][n]
        if ctx.needs_input_grad[1]:
            dw = torch.empty((K, N), dtype=torch.float32, device=x.device)
            _gemm_f32(x, dy, dw, K, N, M, 1, K, N, 1, N, 0, 0, 0, 1)        # A[k][m] = x[m][k]
        return dx, dw


def slab_reduce(slabs: torch.Tensor, out: torch.Tensor, cb: int, out_bs: int, accumulate: bool = False,
                out_bf16: Optional[torch.Tensor] = None, tail: Optional[torch.Tensor] = None,
                tail_bf16: Optional[torch.Tensor] = None, tail_val: float = 0.0) -> None:
    """out = sum over the leading dim of f32 ``slabs`` [S][R][C], written as C/cb column blocks of
    width ``cb`` stored ``out_bs`` floats apart (the split-K combine of the weight-grad GEMMs).
    ``out_bf16`` (same layout as ``out``) also receives the sums rounded to bf16.  ``tail`` (f32,
    and ``tail_bf16``) is filled with the constant ``tail_val`` by the same launch."""
    S, R, C = slabs.shape
    assert slabs.dtype in (torch.float32, torch.bfloat16) and out.dtype == torch.float32 and slabs.is_contiguous()
    assert out_bf16 is None or (out_bf16.dtype == torch.bfloat16 and out_bf16.numel() == out.numel())
    tn = 0
    if tail is not None:
        assert tail.dtype == torch.float32 and tail.is_contiguous() and tail.device == out.device
        assert tail_bf16 is None or (tail_bf16.dtype == torch.bfloat16 and tail_bf16.numel() == tail.numel()
                                     and tail_bf16.is_contiguous())
        tn = tail.numel()
    rc = lib().ljs_slab_reduce(_p(slabs), S, R * C, R, C, _p(out), cb, out_bs, int(accumulate), _p(out_bf16),
                               _p(tail), _p(tail_bf16 if tn else None), tn, float(tail_val),
                               int(slabs.dtype == torch.bfloat16), _stream(out))
    _ck(rc, "slab_reduce")


# ============================================================================ collective pack / unpack
def _pack_launch(srcs, dst: torch.Tensor, A: int, B: int, inner: int, mode: int, perm) -> None:
    arr = (c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    pa = (c_int * B)(*[int(p) for p in perm]) if perm is not None else None
    rc = lib().ljs_pack_rows(arr, len(srcs), _p(dst), A, B, inner, mode, pa, _stream(dst))
    _ck(rc, "pack_rows")


def _pack_ok(*ts) -> bool:
    return all(t.is_cuda for t in ts)


def storage_order(t: torch.Tensor):
    """The permutation of ``t``'s dims from outermost to innermost in memory when ``t`` is DENSE
    (a permutation of a contiguous tensor: no gaps, no overlap), else None.  Size-1 dims keep
    their logical position.  Activations whose sharded sequence dim is kept outermost in
    storage (``seq-major``: (batch, seq, features) stored [seq][batch][features]) gather and
    scatter over that dim as whole contiguous blocks - no pack / unpack kernels."""
    if t.dim() == 0:
        return ()
    order = sorted(range(t.dim()), key=lambda d: (-t.stride(d) if t.shape[d] > 1 else 0, d))
    # size-1 dims anywhere: move them to their logical slot (their stride is irrelevant)
    big = [d for d in order if t.shape[d] > 1]
    one = [d for d in range(t.dim()) if t.shape[d] <= 1]
    order = sorted(one + big, key=lambda d: (big.index(d) if d in big else -1, d)) if one else big
    exp = 1
    for d in reversed(big):
        if t.stride(d) != exp:
            return None
        exp *= t.shape[d]
    return tuple(order)


def is_dense(t: torch.Tensor) -> bool:
    return storage_order(t) is not None


def dense(t: torch.Tensor) -> torch.Tensor:
    """``t`` itself when dense (any dim order), else a contiguous copy."""
    return t if is_dense(t) else t.contiguous()


def flat(t: torch.Tensor) -> torch.Tensor:
    """1-D view of a dense tensor's storage (in memory order)."""
    assert is_dense(t), "flat() needs a dense tensor"
    return t.as_strided((t.numel(),), (1,))


def _in_order(t: torch.Tensor):
    """(view of t with dims in storage order - contiguous, the order) for a dense t; else
    (t.contiguous(), identity)."""
    o = storage_order(t)
    if o is None or list(o) == list(range(t.dim())):
        return t.contiguous(), tuple(range(t.dim()))
    return t.permute(o), o


def _inv(order):
    inv = [0] * len(order)
    for i, d in enumerate(order):
        inv[d] = i
    return inv


def rank_major(x: torch.Tensor, dim: int, n: int, perm=None) -> torch.Tensor:
    """[.., n*s (dim), ..] -> [n][.., s, ..], chunk ``perm[k]`` in first-axis slot k (the send
    buffer of a reduce-scatter / all-to-all): dense, the chunks in x's own dim order.  When
    ``dim`` is outermost in x's storage (and no perm) this is a VIEW - no kernel; otherwise one
    HIP launch on GPU tensors."""
    if perm is not None and list(perm) == list(range(n)):
        perm = None
    xs, order = _in_order(x)
    pdim = order.index(dim)
    shp = tuple(xs.shape)
    s = shp[pdim] // n
    pshape = (n,) + shp[:pdim] + (s,) + shp[pdim + 1:]
    back = [0] + [1 + i for i in _inv(order)]
    if all(v == 1 for v in shp[:pdim]) and perm is None:
        return xs.reshape(pshape).permute(back)
    if not _pack_ok(x) or n > 64:
        v = xs.reshape(shp[:pdim] + (n, s) + shp[pdim + 1:]).movedim(pdim, 0)
        return (v[list(perm)] if perm is not None else v).contiguous().permute(back)
    A = math.prod(shp[:pdim])
    inner = xs.element_size() * s * math.prod(shp[pdim + 1:])
    out = torch.empty(pshape, dtype=x.dtype, device=x.device)
    _pack_launch([xs], out, A, n, inner, 0, perm)
    return out.permute(back)


def from_rank_major(buf: torch.Tensor, dim: int, perm=None) -> torch.Tensor:
    """[n][.., c (dim), ..] -> [.., n*c, ..]: slot ``perm[k]`` of ``buf`` becomes chunk k along
    ``dim`` (the receive buffer of an all-gather / all-to-all back in the tensor's layout).  The
    result keeps the chunks' dim order; when ``dim`` is outermost in it (and no perm) it is a
    VIEW of ``buf``."""
    n = buf.shape[0]
    if perm is not None and list(perm) == list(range(n)):
        perm = None
    chunk = buf[0]
    o = storage_order(chunk) if n > 0 else None
    dense_slots = o is not None and buf.stride(0) == chunk.numel()
    if not dense_slots:
        buf, o = buf.contiguous(), tuple(range(buf.dim() - 1))
    pbuf = buf.permute([0] + [1 + d for d in o])
    pdim = list(o).index(dim)
    cs = tuple(pbuf.shape[1:])
    out_shape = cs[:pdim] + (n * cs[pdim],) + cs[pdim + 1:]
    inv = _inv(o)
    if all(v == 1 for v in cs[:pdim]) and perm is None:
        return pbuf.reshape(out_shape).permute(inv)
    if not _pack_ok(buf) or n > 64:
        b = pbuf[list(perm)] if perm is not None else pbuf
        return b.movedim(0, pdim).reshape(out_shape).contiguous().permute(inv)
    A = math.prod(cs[:pdim])
    inner = buf.element_size() * math.prod(cs[pdim:])
    out = torch.empty(out_shape, dtype=buf.dtype, device=buf.device)
    _pack_launch([pbuf], out, A, n, inner, 1, perm)
    return out.permute(inv)


def concat_parts(parts, dim: int) -> torch.Tensor:
    """``torch.cat(parts, dim)`` of same-shape parts on one GPU in one HIP launch (a loopback
    all-gather over virtual devices); the result keeps the parts' dim order when they are dense
    in a common order."""
    p0 = parts[0]
    n = len(parts)
    if not _pack_ok(*parts) or n > 64 or any(p.shape != p0.shape or p.dtype != p0.dtype or p.device != p0.device
                                            for p in parts):
        return torch.cat(parts, dim)
    o = storage_order(p0)
    if o is None or any(storage_order(p) != o or p.stride() != p0.stride() for p in parts):
        parts, o = [p.contiguous() for p in parts], tuple(range(p0.dim()))
    pparts = [p.permute(o) for p in parts]
    pdim = list(o).index(dim)
    cs = tuple(pparts[0].shape)
    A = math.prod(cs[:pdim])
    inner = p0.element_size() * math.prod(cs[pdim:])
    out = torch.empty(cs[:pdim] + (n * cs[pdim],) + cs[pdim + 1:], dtype=p0.dtype, device=p0.device)
    _pack_launch(pparts, out, A, n, inner, 2, None)
    return out.permute(_inv(o))


def pad_box(src: torch.Tensor, full, lo) -> torch.Tensor:
    """A dense tensor of shape ``full`` holding ``src`` at offset ``lo`` and zeros elsewhere, in
    one HIP launch (the backward of a box slice; ``src`` may be strided)."""
    nd = len(full)
    assert src.dim() == nd and src.is_cuda and nd <= 6
    out = torch.empty(tuple(full), dtype=src.dtype, device=src.device)
    arr = lambda v: (c_long * nd)(*[int(x) for x in v])  # noqa: E731
    rc = lib().ljs_pad_box(_p(src), _p(out), nd, arr(full), arr(lo), arr(src.shape), arr(src.stride()),
                           src.element_size(), _stream(out))
    _ck(rc, "pad_box")
    return out


class _BoxSlice(torch.autograd.Function):
    """``t[box]`` whose backward is one :func:`pad_box` launch (torch's slice_backward is a fill
    plus a copy kernel)."""

    @staticmethod
    def forward(ctx, t, box):
        ctx.full = tuple(t.shape)
        ctx.lo = tuple(s.start for s in box)
        return t[box]

    @staticmethod
    def backward(ctx, g):
        return pad_box(g, ctx.full, ctx.lo), None


def box_slice(t: torch.Tensor, box) -> torch.Tensor:
    """``t[box]`` (a tuple of unit-step slices with explicit bounds): on a GPU tensor that needs a
    gradient, the backward runs as one HIP launch."""
    if t.is_cuda and t.requires_grad and torch.is_grad_enabled() and t.dtype.itemsize in (2, 4, 8) \
            and t.dim() <= 6 and len(box) == t.dim():
        return _BoxSlice.apply(t, tuple(box))
    return t[box]


def bcast_scalar(g: torch.Tensor, C: int, R: int, want_db: bool, db_out: Optional[torch.Tensor] = None,
                 db_bf16: Optional[torch.Tensor] = None):
    """(bf16 row [C] filled with bf16(g), f32 [C] = R * bf16(g) or None) from the 1-element
    tensor ``g`` (f32 or bf16), in one launch (``db_out``: where to write the f32 result;
    ``db_bf16``: also write it rounded to bf16)."""
    row = torch.empty((C,), dtype=torch.bfloat16, device=g.device)
    db = (db_out if db_out is not None else torch.empty((C,), dtype=torch.float32, device=g.device)) \
        if want_db else None
    rc = lib().ljs_bcast_scalar(_p(g), int(g.dtype == torch.bfloat16), C, float(R), _p(row), _p(db),
                                _p(db_bf16 if want_db else None), _stream(row))
    _ck(rc, "bcast_scalar")
    return row, db


def relu_bwd_colsum(dy: torch.Tensor, y: torch.Tensor, R: int, C: int):
    """(dy * (y > 0) as a new bf16 [R][C], its f32 column sums [C]) in one pass: the fused ReLU
    backward + bias gradient of a dense layer.  dy / y: bf16 [R][C] views with unit column
    stride (row strides may differ)."""
    masked = torch.empty((R, C), dtype=torch.bfloat16, device=dy.device)
    out = torch.empty((C,), dtype=torch.float32, device=dy.device)
    ws = _workspace(dy.device, "colsum", _COLSUM_WS_BYTES)
    rc = lib().ljs_relu_bwd_colsum(_p(dy), _p(y), R, C, dy.stride(0), y.stride(0), _p(masked), _p(out), _p(ws),
                                   _stream(dy))
    _ck(rc, "relu_bwd_colsum")
    return masked, out


def relu_bwd(dy: torch.Tensor, y: torch.Tensor, R: int, C: int) -> torch.Tensor:
    """dy * (y > 0) as a new bf16 [R][C] (the ReLU backward of a bias-free dense; same view
    requirements as :func:`relu_bwd_colsum`)."""
    masked = torch.empty((R, C), dtype=torch.bfloat16, device=dy.device)
    rc = lib().ljs_relu_bwd(_p(dy), _p(y), R, C, dy.stride(0), y.stride(0), _p(masked), _stream(dy))
    _ck(rc, "relu_bwd")
    return masked


def colsum_ld(t: torch.Tensor, R: int, C: int, ld: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Column sums of an [R][C] matrix with row stride ``ld`` (0 = one repeated row)."""
    acc = out is not None
    if out is None:
        out = torch.empty((C,), dtype=torch.float32, device=t.device)
    ws = _workspace(t.device, "colsum", _COLSUM_WS_BYTES)
    rc = lib().ljs_colsum(_p(t), int(t.dtype == torch.bfloat16), R, C, ld, _p(out), int(acc), _p(ws), _stream(t))
    _ck(rc, "colsum")
    return out


# ============================================================================ attention
def _strides3(t: torch.Tensor):
    # (batch, seq, head) strides of a (b, s, h, d) tensor with d contiguous
    return [t.stride(0), t.stride(1), t.stride(2)]


def _bs_like(shape, ref: torch.Tensor) -> torch.Tensor:
    """Empty bf16 (B, S, H, D) stored like ``ref``'s (batch, seq) dims: seq-major when ref is
    (the kernels take any batch / seq strides; the result then gathers / scatters over the
    sequence as contiguous blocks)."""
    B, S, H, D = shape
    if B > 1 and S > 1 and ref.stride(1) > ref.stride(0):
        return torch.empty((S, B, H, D), dtype=torch.bfloat16, device=ref.device).permute(1, 0, 2, 3)
    return torch.empty(shape, dtype=torch.bfloat16, device=ref.device)


# ---------------------------------------------------------------------------- fused projection
# The Q/K/V projection GEMM of a self-attention block with a 256-token sequence can run the
# attention forward of each (batch, head) in the same kernel (ljs_qkv_attn_fwd): ops/linear.py
# launches it when the model announced the attention that follows (linear.attention_next) and
# leaves (o, lse) here, keyed by the Q/K/V buffer; _Attention.forward takes them when it is called
# with exactly the q / k / v views of that buffer, and runs its own kernel otherwise.
_FUSED_ATTN: Dict[tuple, tuple] = {}


def qkv_attn_fwd(xb: torch.Tensor, wt: torch.Tensor, out: torch.Tensor, H: int, scale: float,
                 trace: Optional[torch.Tensor] = None):
    """out [T][3N] = xb [T][K] . wt[i]^T (wt: [3][N][K] bf16) AND the attention forward of every
    (batch, head) over it (sequence 256): returns (o [T][N] bf16, lse [T/256][H][256] f32).
    ``trace``: int64 [blocks][8][8][4] phase stamps (LJS_QA_TRACE builds only; scripts/qkv_attn_phases.py)."""
    T, K = xb.shape
    N = wt.shape[1]
    assert (xb.dtype == torch.bfloat16 and wt.dtype == torch.bfloat16 and out.dtype == torch.bfloat16
            and xb.stride(1) == 1 and wt.is_contiguous() and out.is_contiguous() and out.shape == (T, 3 * N)
            and wt.shape == (3, N, K) and N == 64 * H and T % 256 == 0 and K % 128 == 0)
    o = torch.empty((T, N), dtype=torch.bfloat16, device=xb.device)
    lse = torch.empty((T // 256, H, 256), dtype=torch.float32, device=xb.device)
    _ck(lib().ljs_qkv_attn_fwd(_p(xb), xb.stride(0), _p(wt), _p(out), _p(o), _p(lse), T, K, N, H, float(scale),
                               _p(trace) if trace is not None else None, _stream(xb)), "ljs_qkv_attn_fwd")
    return o, lse


def _fused_key(t: torch.Tensor, scale: float):
    return (t.data_ptr(), t._version, t.device.index, float(scale))


def clear_fused_attention() -> None:
    """Drop a fused forward nobody took (also run when a graph capture ends)."""
    _FUSED_ATTN.clear()


def register_fused_attention(out: torch.Tensor, o: torch.Tensor, lse: torch.Tensor, H: int, scale: float) -> None:
    from ..spmd import graphs as _graphs
    if clear_fused_attention not in _graphs.AFTER_CAPTURE:
        _graphs.AFTER_CAPTURE.append(clear_fused_attention)
    _FUSED_ATTN.clear()   # one pending forward at a time
    _FUSED_ATTN[_fused_key(out, scale)] = (o, lse, tuple(out.shape), H)


def _take_fused_attention(q, k, v, scale, causal, q_offset):
    if not _FUSED_ATTN or causal or q_offset:
        return None
    ent = _FUSED_ATTN.get(_fused_key(q, scale))
    if ent is None:
        return None
    o, lse, (T, N3), H = ent
    N = N3 // 3
    B, S = T // 256, 256
    es = q.element_size()
    if not (q.shape == (B, S, H, 64) and k.shape == q.shape and v.shape == q.shape
            and q.stride() == (S * N3, N3, 64, 1) and k.stride() == q.stride() and v.stride() == q.stride()
            and k.data_ptr() == q.data_ptr() + N * es and v.data_ptr() == q.data_ptr() + 2 * N * es):
        return None
    del _FUSED_ATTN[_fused_key(q, scale)]
    FUSED_ATTN_STATS["taken"] += 1
    return o.view(B, S, H, 64), lse


FUSED_ATTN_STATS = {"taken": 0}


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, q_offset):
        B, Sq, H, D = q.shape
        Sk = k.shape[1]
        pre = _take_fused_attention(q, k, v, scale, causal, q_offset)
        if pre is not None:
            o, lse = pre
        else:
            o = _bs_like((B, Sq, H, D), q)
            lse = torch.empty((B, H, Sq), dtype=torch.float32, device=q.device)
            rc = lib().ljs_attn_fwd(_p(q), _p(k), _p(v), _p(o), _p(lse), B, Sq, Sk, H, _longs(_strides3(q)),
                                    _longs(_strides3(k)), _longs(_strides3(v)), _longs(_strides3(o)), scale,
                                    int(causal), q_offset, _stream(q))
            _ck(rc, "ljs_attn_fwd")
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.args = (scale, causal, q_offset)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale, causal, q_offset = ctx.args
        B, Sq, H, D = q.shape
        Sk = k.shape[1]
        do = do.to(torch.bfloat16)
        if do.stride(3) != 1:
            do = do.contiguous()
        st = q.stride()
        fused = (Sq == Sk and k.stride() == st and v.stride() == st and st[3] == 1 and st[2] == D
                 and k.data_ptr() - q.data_ptr() == H * D * 2 and v.data_ptr() - q.data_ptr() == 2 * H * D * 2
                 and st[1] == 3 * H * D and st[0] == Sq * st[1])
        if fused:
            # q/k/v are column blocks of one fused-QKV buffer: write dq/dk/dv the same way so the
            # dense backward sees one [M, 3*H*D] gradient and runs ONE batched weight-grad GEMM
            dqkv = torch.empty((B, Sq, 3, H, D), dtype=torch.bfloat16, device=q.device)
            dq, dk, dv = dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
        else:
            dq = _bs_like((B, Sq, H, D), q)
            dk = _bs_like((B, Sk, H, D), k)
            dv = _bs_like((B, Sk, H, D), v)
        delta = torch.empty((B, H, Sq), dtype=torch.float32, device=q.device)
        rc = lib().ljs_attn_bwd(_p(q), _p(k), _p(v), _p(o), _p(do), _p(lse), _p(delta), _p(dq), _p(dk), _p(dv), B, Sq,
                                Sk, H, _longs(_strides3(q)), _longs(_strides3(k)), _longs(_strides3(v)),
                                _longs(_strides3(o)), _longs(_strides3(do)), _longs(_strides3(dq)),
                                _longs(_strides3(dk)), _longs(_strides3(dv)), scale, int(causal), q_offset,
                                _stream(q))
        _ck(rc, "ljs_attn_bwd")
        return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None, None, None


def attn_fwd_lse(q, k, v, scale: float, causal: bool = False, q_offset: int = 0):
    """Raw flash forward of one (q block, kv block) pair: (o bf16 [B,Sq,H,D], lse f32 [B,H,Sq]).
    lse is log2 of the scaled-score partition function; +inf marks rows with no unmasked key."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    o = torch.empty((B, Sq, H, D), dtype=torch.bfloat16, device=q.device)
    lse = torch.empty((B, H, Sq), dtype=torch.float32, device=q.device)
    rc = lib().ljs_attn_fwd(_p(q), _p(k), _p(v), _p(o), _p(lse), B, Sq, Sk, H, _longs(_strides3(q)),
                            _longs(_strides3(k)), _longs(_strides3(v)), _longs(_strides3(o)), scale, int(causal),
                            q_offset, _stream(q))
    _ck(rc, "ljs_attn_fwd")
    return o, lse


def attn_fwd_acc(q, k, v, scale: float, causal: bool, q_offset: int, oacc: torch.Tensor, lse: torch.Tensor, mode: int,
                 out: Optional[torch.Tensor] = None):
    """One key block of a blockwise (ring) forward merged INTO the running result in the kernel's
    epilogue: mode 1 starts (f32 ``oacc`` [B,Sq,H,D] + ``lse``), 2 merges by log-sum-exp, 3 merges
    and writes the final bf16 ``out`` (returned).  No per-hop torch merge kernels."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    assert oacc.dtype == torch.float32 and oacc.stride(3) == 1 and lse.dtype == torch.float32
    if mode == 3 and out is None:
        out = _bs_like((B, Sq, H, D), q)
    o = out if out is not None else q   # (unused unless mode 3)
    rc = lib().ljs_attn_fwd_acc(_p(q), _p(k), _p(v), _p(o), _p(lse), B, Sq, Sk, H, _longs(_strides3(q)),
                                _longs(_strides3(k)), _longs(_strides3(v)), _longs(_strides3(o)), scale, int(causal),
                                q_offset, _p(oacc), _longs(_strides3(oacc)), int(mode), _stream(q))
    _ck(rc, "ljs_attn_fwd_acc")
    return out


def attn_bwd_block(q, k, v, o, do, lse, scale: float, causal: bool = False, q_offset: int = 0):
    """Raw flash backward of one kv block given the FINAL output ``o`` and GLOBAL ``lse``
    (blockwise-separable): returns this block's (dq, dk, dv) contributions in bf16."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    do = do.to(torch.bfloat16)
    if do.stride(3) != 1:
        do = do.contiguous()
    dq = torch.empty((B, Sq, H, D), dtype=torch.bfloat16, device=q.device)
    dk = torch.empty((B, Sk, H, D), dtype=torch.bfloat16, device=q.device)
    dv = torch.empty((B, Sk, H, D), dtype=torch.bfloat16, device=q.device)
    delta = torch.empty((B, H, Sq), dtype=torch.float32, device=q.device)
    rc = lib().ljs_attn_bwd(_p(q), _p(k), _p(v), _p(o), _p(do), _p(lse), _p(delta), _p(dq), _p(dk), _p(dv), B, Sq, Sk,
                            H, _longs(_strides3(q)), _longs(_strides3(k)), _longs(_strides3(v)), _longs(_strides3(o)),
                            _longs(_strides3(do)), _longs(_strides3(dq)), _longs(_strides3(dk)), _longs(_strides3(dv)),
                            scale, int(causal), q_offset, _stream(q))
    _ck(rc, "ljs_attn_bwd")
    return dq, dk, dv


def attention(q, k, v, scale: float, causal: bool = False, q_offset: int = 0) -> torch.Tensor:
    ok = (q.shape[-1] == 64 and k.shape[-1] == 64 and v.shape[-1] == 64 and q.stride(-1) == 1
          and k.stride(-1) == 1 and v.stride(-1) == 1)
    if not ok:
        raise NotImplementedError(f"HIP attention supports head_dim 64 with contiguous head_dim; got {q.shape}")
    qb, kb, vb = (t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16) for t in (q, k, v))
    out = _Attention.apply(qb, kb, vb, float(scale), bool(causal), int(q_offset))
    return out if v.dtype == torch.bfloat16 else out.to(v.dtype)


# ============================================================================ optimizer
def adam(p, g, m, v, step, lr, b1, b2, eps, wd, inplace):
    assert p.dtype == torch.float32 and m.dtype == torch.float32 and v.dtype == torch.float32
    g = g.contiguous()
    if g.dtype not in (torch.float32, torch.bfloat16):
        g = g.float()
    pc, mc, vc = p.contiguous(), m.contiguous(), v.contiguous()
    if inplace and pc.data_ptr() == p.data_ptr():
        po, mo, vo = p, m, v
    else:
        po, mo, vo = torch.empty_like(pc), torch.empty_like(mc), torch.empty_like(vc)
    step_i = step if step.dtype == torch.int32 else step.to(torch.int32)
    rc = lib().ljs_adam_f32(_p(pc), _p(g), int(g.dtype == torch.bfloat16), _p(mc), _p(vc), _p(po), _p(mo), _p(vo),
                            _p(step_i), p.numel(), lr, b1, b2, eps, wd, _stream(p))
    _ck(rc, "ljs_adam_f32")
    return po.view(p.shape), mo.view(m.shape), vo.view(v.shape)


class SlabGrad:
    """A weight gradient not yet combined: element (r, c) is the sum over s < S of
    ``slabs.view(-1)[offset + s * slab_stride + r * ld + c]`` (the split-K slabs of its GEMM)."""
    __slots__ = ("slabs", "S", "offset", "ld", "slab_stride", "shape")

    def __init__(self, slabs, S, offset, ld, slab_stride, shape):
        self.slabs, self.S, self.offset, self.ld, self.slab_stride = slabs, S, offset, ld, slab_stride
        self.shape = tuple(shape)


class ConstGrad:
    """A gradient whose every element is ``value`` (f32)."""
    __slots__ = ("value", "shape")

    def __init__(self, value, shape):
        self.value, self.shape = float(value), tuple(shape)


# Count increments deferred inside a HIP-graph capture (a G-step graph): each Adam launch reads the
# count as it was at the last flush plus the increments still pending, and the pending increments
# become ONE launch when the capture segment ends (spmd/graphs.BEFORE_CUT) -- one count launch per
# graph instead of one per step.  Eager calls and single-controller multi-device captures
# increment at once.  LJS_ADAM_DEFER_INC=0: off.
_DEFER_INC = os.environ.get("LJS_ADAM_DEFER_INC", "1") == "1"
_PENDING_INC: Dict[int, list] = {}     # step data_ptr -> [step tensor, pending increments]


def _flush_step_incs() -> None:
    while _PENDING_INC:
        _, (st, n) = _PENDING_INC.popitem()
        if n:
            _ck(lib().ljs_step_add(_p(st), n, _stream(st)), "ljs_step_add")


def flush_step_inc(step: torch.Tensor) -> None:
    """Launch ``step``'s pending deferred increments now (in stream order), so a kernel that reads
    the count after this point -- anything but the next Adam launch, which adds the pending
    offset itself -- sees the incremented value (optim/adam.CountLocal calls this on reads)."""
    ent = _PENDING_INC.get(step.data_ptr())
    if ent is not None and ent[1]:
        _ck(lib().ljs_step_add(_p(ent[0]), ent[1], _stream(ent[0])), "ljs_step_add")
        ent[1] = 0


def _defer_step_inc(step: torch.Tensor):
    """Pending increments of ``step`` before this one (and one more recorded), or None when the
    increment must be launched now."""
    if not _DEFER_INC:
        return None
    from ..spmd import graphs as _graphs
    g = _graphs.current()
    if g is None or isinstance(g, _graphs.MultiDeviceGraph):
        return None
    if _flush_step_incs not in _graphs.BEFORE_CUT:
        _graphs.BEFORE_CUT.append(_flush_step_incs)
    ent = _PENDING_INC.setdefault(step.data_ptr(), [step, 0])
    pend = ent[1]
    ent[1] += 1
    return pend




_ADAM_ROWS = [0]


def set_adam_rows(rows: int) -> None:
    """Force the fused Adam's tile height (16 / 32 / 64; 0 = automatic: 32, or 64 when a tensor
    carries MX-fp8 shadows).  For tests of the kernel's tile paths; bit-identical results."""
    lib().ljs_adam_set_rows(int(rows))
    _ADAM_ROWS[0] = int(rows)


def adam_rows() -> int:
    return _ADAM_ROWS[0]


def adam_multi(entries, step: torch.Tensor, lr, b1, b2, eps, wd, increment_step: bool = False) -> None:
    """In-place fused Adam over many params (one launch per 32): entries = [(p, g, m, v)].

    Also rewrites each param's registered bf16 and MX-fp8 shadows (see :mod:`.shadow`).  With
    ``increment_step`` the bias corrections use ``step + 1`` and int32 ``step`` is incremented in
    place by a one-lane launch -- inside a graph capture one launch per segment for all its
    steps (``_defer_step_inc``)."""
    from . import shadow
    import numpy as np
    rows = []
    for p, g, m, v in entries:
        assert p.is_contiguous() and m.is_contiguous() and v.is_contiguous() and p.dtype == torch.float32
        R, C = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())
        if isinstance(g, SlabGrad):
            # the weight gradient is still its split-K slabs: the kernel sums them (no combine)
            assert g.shape == tuple(p.shape) and g.slabs.dtype in (torch.float32, torch.bfloat16) \
                and g.slabs.is_contiguous()
            es = g.slabs.element_size()
            gsrc = (g.slabs.data_ptr() + es * g.offset, int(es == 2), g.S, g.ld, g.slab_stride)
        elif isinstance(g, ConstGrad):
            assert g.shape == tuple(p.shape)
            bits = int(np.asarray(g.value, dtype=np.float32).view(np.int32))
            gsrc = (0, 0, -1, bits, 0)
        else:
            if g.dtype not in (torch.float32, torch.bfloat16) or not g.is_contiguous():
                g = g.float().contiguous() if g.dtype not in (torch.float32, torch.bfloat16) else g.contiguous()
            gsrc = (g.data_ptr(), int(g.dtype == torch.bfloat16), 0, C, 0)
        bufs = shadow.kinds_of(p) if p.dim() == 2 else {}
        st, sn = bufs.get("T"), bufs.get("N")
        ptr = lambda k: bufs[k].data_ptr() if k in bufs else 0  # noqa: E731
        rows.append(([p.data_ptr(), gsrc[0], m.data_ptr(), v.data_ptr(),
                      st.data_ptr() if st is not None else 0, sn.data_ptr() if sn is not None else 0,
                      R, C, gsrc[1], gsrc[2],
                      ptr("QN"), ptr("QNs"), ptr("QT"), ptr("QTs"), gsrc[3], gsrc[4]], g))
    if increment_step:
        assert step.dtype == torch.int32 and step.is_contiguous()
    step_i = step if step.dtype == torch.int32 else step.to(torch.int32)
    # inside a capture the increments are deferred (one launch per capture segment, see
    # _defer_step_inc): this launch reads the not-yet-incremented count, offset by what is pending
    pend = _defer_step_inc(step_i) if increment_step else None
    offset = int(increment_step) + (pend or 0)
    # the next step's input cast, run by the last launch's extra blocks (ops/linear.py early cast)
    cast = None
    if rows and step_i.is_cuda:
        from . import linear as _lin
        cast = _lin.take_optimizer_precast(step_i.device)
    for i in range(0, len(rows), 32):
        chunk = rows[i:i + 32]
        tab = np.asarray([r[0] for r in chunk], dtype=np.int64).reshape(-1)
        arr = (ctypes.c_long * tab.size)(*tab.tolist())
        last = i + 32 >= len(rows)
        cj = cast if last else None
        rc = lib().ljs_adam_multi(arr, len(chunk), _p(step_i), offset,
                                  None, lr, b1, b2, eps, wd,
                                  _p(cj[0]) if cj else None, _p(cj[1]) if cj else None, cj[0].numel() if cj else 0,
                                  _stream(step_i))
        _ck(rc, "ljs_adam_multi")
        if cj is not None:
            _lin.commit_optimizer_precast(cj)
    if increment_step and pend is None:
        _ck(lib().ljs_step_add(_p(step_i), 1, _stream(step_i)), "ljs_step_add")
    for p, _, _, _ in entries:
        shadow.mark_fresh(p)


# ============================================================================ clock probe
_CLOCK: Dict[int, tuple] = {}   # device index -> (records [cap, 4] int64, counter int32)


def clock_probe(dev: torch.device, ticks: int = 300, cap: int = 8192) -> None:
    """Record the shader clock here in the stream (csrc/kernels/diag.hip): one lane spins for
    ``ticks`` of the 100 MHz counter (3 us) and stores delta s_memtime / delta s_memrealtime; a
    diagnostic, launched by bench.py after every step under LJS_CLOCK_PROBE (graph-capturable)."""
    dev = torch.device(dev)
    ent = _CLOCK.get(dev.index)
    if ent is None:
        ent = _CLOCK[dev.index] = (torch.zeros((cap, 4), dtype=torch.int64, device=dev),
                                   torch.zeros(1, dtype=torch.int32, device=dev))
    rec, ctr = ent
    _ck(lib().ljs_clock_probe(_p(rec), _p(ctr), rec.shape[0], int(ticks), torch.cuda.current_stream(dev).cuda_stream),
        "ljs_clock_probe")


def clock_probe_records(dev: torch.device) -> List[dict]:
    """Every record so far, in launch order: shader clock (MHz), start (us of the 100 MHz counter)."""
    ent = _CLOCK.get(torch.device(dev).index)
    if ent is None:
        return []
    torch.cuda.synchronize(dev)
    rec, ctr = ent
    n = min(int(ctr.item()), rec.shape[0])
    out = []
    for d_sclk, d_ref, ref0, xcc in rec[:n].cpu().tolist():
        out.append({"sclk_mhz": round(d_sclk / max(1, d_ref) * 100.0, 1), "t_us": ref0 / 100.0, "xcc": int(xcc)})
    return out


# ============================================================================ RNG
_DIST = {"normal": 0, "uniform": 1, "truncated_normal": 2}


def rng_fill(shape, region, k0, k1, dist, lo, hi, dtype, device) -> torch.Tensor:
    if dist not in _DIST:
        raise NotImplementedError(dist)
    local = tuple(r1 - r0 for r0, r1 in region)
    od = dtype if dtype in (torch.float32, torch.bfloat16) else torch.float32
    out = torch.empty(local, dtype=od, device=device)
    nd = len(shape)
    strides = [1] * nd
    for i in range(nd - 2, -1, -1):
        strides[i] = strides[i + 1] * shape[i + 1]
    ea = eb = 0.0
    if dist == "truncated_normal":
        ea, eb = math.erf(lo / math.sqrt(2)), math.erf(hi / math.sqrt(2))
    if out.numel():
        rc = lib().ljs_rng_fill(_p(out), int(od == torch.bfloat16), nd, _longs([r[0] for r in region] or [0]),
                                _longs(list(local) or [1]), _longs(strides or [1]), k0, k1, _DIST[dist], lo, hi, ea,
                                eb, torch.cuda.current_stream(device).cuda_stream)
        _ck(rc, "ljs_rng_fill")
    return out if od == dtype else out.to(dtype)


# ============================================================================ dropout
def _dropout_raw(x: torch.Tensor, shape, region, k0: int, k1: int, keep: float) -> torch.Tensor:
    x = x.contiguous()
    y = torch.empty_like(x)
    nd = len(shape)
    strides = [1] * nd
    for i in range(nd - 2, -1, -1):
        strides[i] = strides[i + 1] * shape[i + 1]
    rc = lib().ljs_dropout(_p(x), _p(y), int(x.dtype == torch.bfloat16), nd, _longs([r[0] for r in region]),
                           _longs([r1 - r0 for r0, r1 in region]), _longs(strides), k0, k1, keep, _stream(x))
    _ck(rc, "ljs_dropout")
    return y


class _Dropout(torch.autograd.Function):
    """Counter-based dropout of one shard (csrc/kernels/elementwise.hip dropout_kernel): the
    backward recomputes the mask from the key, nothing is stored."""

    @staticmethod
    def forward(ctx, x, meta):
        shape, region, k0, k1, keep = meta
        ctx.meta = meta
        return _dropout_raw(x, shape, region, k0, k1, keep)

    @staticmethod
    def backward(ctx, dy):
        shape, region, k0, k1, keep = ctx.meta
        return _dropout_raw(dy, shape, region, k0, k1, keep), None


def dropout(x: torch.Tensor, shape, region, k0: int, k1: int, keep: float) -> torch.Tensor:
    """Dropout of the shard ``x`` (region ``region`` of a global array of ``shape``), f32 / bf16."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise NotImplementedError(f"dropout kernel: f32 / bf16 only, got {x.dtype}")
    return _Dropout.apply(x, (tuple(shape), tuple(region), int(k0), int(k1), float(keep)))
