// Shared helpers for the gfx950 (MI355X / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define LJS_API extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef unsigned short bf16_t;  // raw bf16 bits in memory

#define LDS_PTR(T) __attribute__((address_space(3))) T*

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN-preserving via the hardware cvt when available)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&b);
}

// two f32 -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (RNE); building the pair from two scalar
// conversions costs a cvt each plus a shift and an SDWA or
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}

// Cross-row reductions with the gfx950 lane-swap instructions (no LDS round trip, no index
// math): v_permlane16_swap exchanges odd 16-lane rows of one operand with even rows of the
// other, v_permlane32_swap the upper half with the lower; with both operands = v each lane
// ends up holding its own value and its partner's, so max/sum over lanes l, l^16, l^32,
// l^48 (the four 16-lane rows) take two swaps and two ops.
__device__ __forceinline__ float row4_max(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float row4_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// Pair exchange of the swapped-operand MFMA epilogues: lanes l and l ^ 16 hold the two 16-column
// blocks (a0, a1) of one output row; afterwards every lane holds 8 consecutive columns: lo = a0 of
// itself and of lane l + 16 (even 16-lane rows), or a1 of lane l - 16 and of itself (odd rows).
// One v_permlane16_swap per element (odd rows of the first operand <-> even rows of the second):
// no ds_bpermute round trip through the LDS crossbar and no selects.
#ifndef LJS_EPI_PLSWAP
#define LJS_EPI_PLSWAP 1
#endif
__device__ __forceinline__ void pair_rows16(const f32x4& a0, const f32x4& a1, bool even, float (&v)[8]) {
#if LJS_EPI_PLSWAP
  (void)even;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a0[e]), __float_as_uint(a1[e]), false, false);
    v[e] = __uint_as_float(r[0]);
    v[4 + e] = __uint_as_float(r[1]);
  }
#else
  const f32x4 keep = even ? a0 : a1, send = even ? a1 : a0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float recv = __shfl_xor(send[e], 16, 64);
    v[e] = even ? keep[e] : recv;
    v[4 + e] = even ? recv : keep[e];
  }
#endif
}

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: per 16-lane group a 4(row) x 16(col) block of 16-bit elements is read
// transposed; lane i of the group gets column i, rows 0..3.  Lane 4q+p supplies the address of
// row q, columns 4p..4p+3.
__device__ __forceinline__ s16x4 lds_read_tr16(const bf16_t* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds_addr));
}

__device__ __forceinline__ bf16x8 join_bf16x8(s16x4 lo, s16x4 hi) {
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// XCD-aware bijective remap of a linear block id (MI355X: 8 XCDs, blocks dealt round-robin).
// Blocks that share an XCD get a contiguous range of tile ids, so neighbouring tiles (which
// share operand panels) hit the same L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx) return bid;
  int q = nwg / nx, r = nwg % nx;
  int xcd = bid % nx, idx = bid / nx;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

// raw buffer resource over [base, base + bytes): out-of-range offsets read 0 and drop stores.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long bytes) {
  // readfirstlane the inputs so the compiler can prove the descriptor wave-uniform (no waterfall)
  const unsigned long long b = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes));
  void* p = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, nb, 0x00020000);
}

// ---- LDS-DMA from inline asm.  The compiler's waitcnt pass treats a builtin LDS-DMA as a
// possible writer of EVERY LDS location and puts vmcnt waits in front of all later ds_read /
// ds_write, which serialises a prefetch behind the math it should overlap.  Issued as asm the
// DMA is invisible to that pass; the kernel waits for it explicitly (vmcnt(0) + barrier).
// Extra untracked vector-memory ops can only make the compiler's own counted waits wait longer
// (the counter retires in order), never shorter.
__device__ __forceinline__ u32x4 rsrc_u4(const void* base, long bytes) {
  const unsigned long long b = (unsigned long long)base;
  u32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((unsigned)b);
  r[1] = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) & 0xffffu;  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((unsigned)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes));
  r[3] = 0x00020000u;
  return r;
}
// 64 lanes x 16 B from rsrc + voff (per lane) to LDS [lds, lds + 1 KiB), lane-contiguous
__device__ __forceinline__ void dma_lds_x4(const u32x4& rs, int voff, const void* lds) {
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(LDS_PTR(const void))lds);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(m) : "memory", "m0");
}
// 64 lanes x 4 B to LDS [lds, lds + 256 B)
__device__ __forceinline__ void dma_lds_x1(const u32x4& rs, int voff, const void* lds) {
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(LDS_PTR(const void))lds);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(m) : "memory", "m0");
}

// ---- in-launch "last arriver" hand-off (cdna_hip_programming.md §6 Guideline 16, valid form:
// write-through (sc1) payload stores by ONE wave, that wave's vmcnt(0), one lane's agent-scope
// atomic ticket add; the block whose add returns n-1 reads every payload with sc1 loads and
// re-arms the ticket).  Tickets live in a persistent workspace zeroed once at allocation.
__device__ __forceinline__ void sc1_store(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float sc1_load(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// returns true in exactly one block (the last of `n` arrivals); call from ONE lane after the
// storing wave's `s_waitcnt vmcnt(0)`
__device__ __forceinline__ bool ticket_last(unsigned* ticket, unsigned n) {
  unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == n - 1) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}

// Two-level arrival over n blocks (block id bid): one ticket word per group of 32 blocks
// (t[1 + group]) and one top word (t[0]) drawn by each group's last arriver.  One word retires
// only ~88 arrivals/us, so a few hundred blocks on a single word serialise for microseconds.
// Returns true in exactly one block; t needs 1 + ceil(n / 32) words, zero at rest (re-armed).
__device__ __forceinline__ bool ticket_last_2lvl(unsigned* t, unsigned bid, unsigned n) {
  const unsigned grp = bid >> 5, ngrp = (n + 31) >> 5;
  const unsigned in_grp = n - (grp << 5) < 32u ? n - (grp << 5) : 32u;
  if (!ticket_last(t + 1 + grp, in_grp)) return false;
  return ticket_last(t, ngrp);
}

__device__ __forceinline__ float warp_max64(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float warp_sum64(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- MX-fp8 (OCP e4m3 elements, e8m0 block scales over 32 elements)
// shared e8m0 exponent of a block from its amax; returns the unbiased exponent X (2^X scale).
// OCP's floor(log2 amax) - 8, plus one when amax / 2^X would exceed 448 (mantissa > 1.75), so
// no element of the block saturates.
__device__ __forceinline__ int mx_exponent(float amax) {
  if (!(amax > 0.f)) return -127;
  int e;
  const float m = frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1): floor(log2 amax) = e - 1
  int x = e - 1 - 8 + (m > 0.875f ? 1 : 0);
  return x < -127 ? -127 : (x > 127 ? 127 : x);
}

// (no clamp to +-448: every caller scales a block by 2^-mx_exponent(block amax), which puts
// the whole block inside [-448, 448] - m <= 0.875 gives at most 448, a larger mantissa raises
// the exponent and gives at most 256 -- so the 8 min/max a clamp costs per 4 values would never
// change a finite result)
// 4 e4m3 bytes of two packed bf16 pairs divided by 2^x, in two gfx950 scaled conversions
// (v_cvt_scalef32_pk_fp8_bf16 with scale 2^x: bit-identical to rounding v * 2^-x with
// pack4_e4m3, measured on 2^20 pairs by scripts/cvt_scalef_probe.py).  x = -127 (an all-zero
// block) converts with scale 1 (the values are 0 either way; 2^-127 would be an f32 denormal).
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef short s16x2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float mx_scale_pow2(int x) { return x == -127 ? 1.f : ldexpf(1.f, x); }
__device__ __forceinline__ unsigned cvt4_e4m3_bf16(unsigned lo2, unsigned hi2, float sc) {
  s16x2v_t o = {0, 0};
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o, __builtin_bit_cast(bf16x2v_t, lo2), sc, false);
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o, __builtin_bit_cast(bf16x2v_t, hi2), sc, true);
  return __builtin_bit_cast(unsigned, o);
}

__device__ __forceinline__ unsigned pack4_e4m3(float a, float b, float c, float d) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);   // bytes 0,1
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, lo, true);   // bytes 2,3
  return (unsigned)hi;
}
