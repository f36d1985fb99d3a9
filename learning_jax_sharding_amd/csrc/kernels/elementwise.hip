// Memory-bound kernels: casts (optionally transposing), reductions, softmax, fused Adam,
// Philox RNG.  All vectorised to 16 bytes per lane (CDNA Guideline 13); grid-stride loops
// capped at 2048 workgroups so one launch fills the 256 CUs without oversubscription.
#include "common.h"
#include <stdlib.h>
#include <type_traits>
#include <algorithm>

namespace {

constexpr int kMaxGrid = 2048;

inline int grid_for(long n, int per_block) {
  long g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g > kMaxGrid ? kMaxGrid : g);
}

// ------------------------------------------------------------------ casts
__global__ void cast_f32_bf16(const float* __restrict__ in, bf16_t* __restrict__ out, long n) {
  long i8 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  long stride = (long)gridDim.x * blockDim.x * 8;
  for (; i8 + 8 <= n; i8 += stride) {
    f32x4 a = *reinterpret_cast<const f32x4*>(in + i8);
    f32x4 b = *reinterpret_cast<const f32x4*>(in + i8 + 4);
    u32x4 o;
    o[0] = pack_bf16x2(a[0], a[1]);
    o[1] = pack_bf16x2(a[2], a[3]);
    o[2] = pack_bf16x2(b[0], b[1]);
    o[3] = pack_bf16x2(b[2], b[3]);
    *reinterpret_cast<u32x4*>(out + i8) = o;
  }
  if (i8 < n) for (long j = i8; j < n; ++j) out[j] = f2bf(in[j]);
}

__global__ void cast_bf16_f32(const bf16_t* __restrict__ in, float* __restrict__ out, long n) {
  long i8 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  long stride = (long)gridDim.x * blockDim.x * 8;
  for (; i8 + 8 <= n; i8 += stride) {
    u32x4 v = *reinterpret_cast<const u32x4*>(in + i8);
    f32x4 a, b;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      a[2 * k] = __uint_as_float(v[k] << 16);
      a[2 * k + 1] = __uint_as_float(v[k] & 0xffff0000u);
      b[2 * k] = __uint_as_float(v[k + 2] << 16);
      b[2 * k + 1] = __uint_as_float(v[k + 2] & 0xffff0000u);
    }
    *reinterpret_cast<f32x4*>(out + i8) = a;
    *reinterpret_cast<f32x4*>(out + i8 + 4) = b;
  }
  if (i8 < n) for (long j = i8; j < n; ++j) out[j] = bf2f(in[j]);
}

// out[c][r] = bf16(in[r][c]) for an R x C f32 matrix (row stride ldi), 64x64 tiles through LDS.
// out[c][r] = bf16(in[r][c]) through a 32 x 32 LDS tile: 16-byte f32 loads (8 lanes per input
// row), 8-byte bf16 stores (8 lanes per output row), one pass each.  (The 64 x 64 form with
// scalar loads / 2-byte stores gave a [320][512] weight shard 40 workgroups and 7.6 us -- the
// 2-D layout's per-step transposed shadow, profiles/r6ag_fake4_2d_kernels.md.)
__global__ __launch_bounds__(256) void cast_transpose_f32_bf16(const float* __restrict__ in, bf16_t* __restrict__ out,
                                                               int R, int C, long ldi, long ldo, int vin, int vout) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int t = threadIdx.x;
  {
    const int lr = t >> 3, lc = (t & 7) * 4;
    const int r = r0 + lr, c = c0 + lc;
    float v[4];
    if (vin && r < R && c + 3 < C) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(in + (long)r * ldi + c);
      v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (r < R && c + e < C) ? in[(long)r * ldi + c + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[lr][lc + e] = v[e];
  }
  __syncthreads();
  const int oc = t >> 3, orr = (t & 7) * 4;   // output row (an input column), 4 output columns
  const int c = c0 + oc, r = r0 + orr;
  if (c >= C) return;
  bf16_t* o = out + (long)c * ldo + r;
  if (vout && r + 3 < R) {
    *reinterpret_cast<u32x2*>(o) = u32x2{pack_bf16x2(tile[orr][oc], tile[orr + 1][oc]),
                                         pack_bf16x2(tile[orr + 2][oc], tile[orr + 3][oc])};
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (r + e < R) o[e] = f2bf(tile[orr + e][oc]);
  }
}

// ------------------------------------------------------------------ reductions
template <typename T>
__device__ __forceinline__ float ldv(const T* p, long i);
template <>
__device__ __forceinline__ float ldv<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldv<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }

template <typename T>
__global__ void sum_all_kernel(const T* __restrict__ in, long n, float* __restrict__ out) {
  float s = 0.f;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) s += ldv<T>(in, i);
  s = warp_sum64(s);
  __shared__ float part[16];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += part[k];
    atomicAdd(out, t);
  }
}

// 16-byte vectorised sum of a bf16 / f32 array
template <typename T>
__global__ void sum_all_vec_kernel(const T* __restrict__ in, long n, float* __restrict__ out) {
  constexpr int V = 16 / sizeof(T);
  float s = 0.f;
  long nv = n / V;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < nv; i += stride) {
    u32x4 v = *reinterpret_cast<const u32x4*>(in + i * V);
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) s += __uint_as_float(v[k] << 16) + __uint_as_float(v[k] & 0xffff0000u);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) s += __uint_as_float(v[k]);
    }
  }
  if (blockIdx.x == 0)
    for (long j = nv * V + threadIdx.x; j < n; j += blockDim.x) s += ldv<T>(in, j);
  s = warp_sum64(s);
  __shared__ float part[16];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += part[k];
    atomicAdd(out, t);
  }
}

constexpr int kGroup = 32, kMaxSumBlocks = 1024;  // sum_all: ticket group size, max grid

// Whole-array sum with the in-launch last-arriver reduction: no memset, no second kernel, and
// the result is written directly in the output dtype (f32 or bf16).
template <typename T>
__global__ void sum_all_ticket_kernel(const T* __restrict__ in, long n, float* __restrict__ partials,
                                      unsigned* __restrict__ ticket, void* __restrict__ out, int out_bf16) {
  constexpr int V = 16 / sizeof(T);
  constexpr int U = 16;  // independent 16-byte loads in flight per thread (Little's law: the
                        // launcher sizes the grid so the whole array is ~one batch in flight)
  float s = 0.f;
  const long nv = n / V;
  const long stride = (long)gridDim.x * blockDim.x;
  auto acc = [&](const u32x4& v) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) s += __uint_as_float(v[k] << 16) + __uint_as_float(v[k] & 0xffff0000u);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) s += __uint_as_float(v[k]);
    }
  };
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < nv; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const u32x4*>(in + (i + u * stride) * V);
#pragma unroll
    for (int u = 0; u < U; ++u) acc(v[u]);
  }
  for (; i < nv; i += stride) acc(*reinterpret_cast<const u32x4*>(in + i * V));
  if (blockIdx.x == 0)
    for (long j = nv * V + threadIdx.x; j < n; j += blockDim.x) s += ldv<T>(in, j);
  s = warp_sum64(s);
  __shared__ float part[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = s;
  __syncthreads();
  if (w == 0) {
    // two-level last-arriver: one ticket word per group of kGroup blocks, then one top ticket
    // over the groups (a single word retires only ~88 arrivals/us, so 1024 arrivals on one
    // word would serialise for ~12 us)
    const int G = (int)gridDim.x, grp = blockIdx.x / kGroup, ngrp = (G + kGroup - 1) / kGroup;
    const int in_grp = min(kGroup, G - grp * kGroup);
    if (lane == 0) {
      float t = 0.f;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += part[k];
      sc1_store(partials + blockIdx.x, t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) last = ticket_last(ticket + 1 + grp, in_grp);
    last = __shfl(last, 0, 64);
    if (!last) return;
    float v = lane < in_grp ? sc1_load(partials + grp * kGroup + lane) : 0.f;
    v = warp_sum64(v);
    if (lane == 0) sc1_store(partials + kMaxSumBlocks + grp, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = 0;
    if (lane == 0) last = ticket_last(ticket, ngrp);
    last = __shfl(last, 0, 64);
    if (!last) return;
    v = lane < ngrp ? sc1_load(partials + kMaxSumBlocks + lane) : 0.f;
    v = warp_sum64(v);
    if (lane == 0) {
      if (out_bf16) *reinterpret_cast<bf16_t*>(out) = f2bf(v);
      else *reinterpret_cast<float*>(out) = v;
    }
  }
}

// column sums of a bf16 [R][C] matrix, partial slabs + last-arriver per column block (no memset)
// Optional fused ReLU backward (mask != null): in *= (mask > 0) element-wise -- mask is the
// ReLU's bf16 output, same [R][C] layout with row stride ld -- and the masked values are also
// written to masked_out (row stride C).  One pass then yields both the masked gradient the
// GEMMs read and its column sums (the bias gradient).
__device__ __forceinline__ u32x4 relu_mask_bf16x8(const u32x4& v, const u32x4& m) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // a bf16 is > 0 iff its sign bit is clear and it is not +0: keep each half where that holds
    const unsigned lo = (m[k] & 0x8000u) == 0 && (m[k] & 0x7fffu) != 0 ? 0x0000ffffu : 0u;
    const unsigned hi = (m[k] & 0x80000000u) == 0 && (m[k] & 0x7fff0000u) != 0 ? 0xffff0000u : 0u;
    o[k] = v[k] & (lo | hi);
  }
  return o;
}

__global__ void colsum_ticket_kernel(const bf16_t* __restrict__ in, int R, int C, long ld, int rows_per_block,
                                     float* __restrict__ partials, unsigned* __restrict__ tickets,
                                     float* __restrict__ out, int accumulate, const bf16_t* __restrict__ mask,
                                     long mld, bf16_t* __restrict__ masked_out) {
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cl * 8;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(R, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto add = [&](const u32x4& v) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += __uint_as_float(v[k] << 16);
      acc[2 * k + 1] += __uint_as_float(v[k] & 0xffff0000u);
    }
  };
  if (c0 < C && mask) {
    int r = r0 + rl;
    for (; r + 96 < r1; r += 128) {  // 4 independent row loads (+ 4 mask loads) in flight
      u32x4 v[4], m[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = *reinterpret_cast<const u32x4*>(in + (long)(r + 32 * u) * ld + c0);
        m[u] = *reinterpret_cast<const u32x4*>(mask + (long)(r + 32 * u) * mld + c0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const u32x4 o = relu_mask_bf16x8(v[u], m[u]);
        *reinterpret_cast<u32x4*>(masked_out + (long)(r + 32 * u) * C + c0) = o;
        add(o);
      }
    }
    for (; r < r1; r += 32) {
      const u32x4 o = relu_mask_bf16x8(*reinterpret_cast<const u32x4*>(in + (long)r * ld + c0),
                                       *reinterpret_cast<const u32x4*>(mask + (long)r * mld + c0));
      *reinterpret_cast<u32x4*>(masked_out + (long)r * C + c0) = o;
      add(o);
    }
  } else if (c0 < C) {
    int r = r0 + rl;
    for (; r + 96 < r1; r += 128) {  // 4 independent row loads in flight
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4*>(in + (long)(r + 32 * u) * ld + c0);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; r < r1; r += 32) add(*reinterpret_cast<const u32x4*>(in + (long)r * ld + c0));
  }
  __shared__ float red[32][65];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rl][cl * 8 + k] = acc[k];
  __syncthreads();
  __shared__ int last_s;
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int r = 0; r < 32; ++r) s += red[r][lane];
    if (c < C) sc1_store(partials + (long)blockIdx.y * C + c, s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) last_s = ticket_last(tickets + blockIdx.x, gridDim.y);
  }
  __syncthreads();
  if (!last_s) return;
  // the last block of this column block sums the gy partial rows: 4 row slices x 64 columns,
  // 8 independent loads in flight per thread (a dependent chain of gy loads took ~20 us)
  const int gy = gridDim.y;
  float v = 0.f;
  if (c < C) {
    int y = sl;
    for (; y + 28 < gy; y += 32) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = sc1_load(partials + (long)(y + 4 * u) * C + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) v += t[u];
    }
    for (; y < gy; y += 4) v += sc1_load(partials + (long)y * C + c);
  }
  red[sl][lane] = v;
  __syncthreads();
  if (threadIdx.x < 64 && c < C) {
    const float s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    out[c] = accumulate ? out[c] + s : s;
  }
}

// column sums of a matrix whose R rows are all the same row (row stride 0)
__global__ void colsum_bcast_kernel(const void* __restrict__ in, int is_bf16, int R, int C, float* __restrict__ out,
                                    int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float v = is_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(in)[c]) : reinterpret_cast<const float*>(in)[c];
  out[c] = (accumulate ? out[c] : 0.f) + v * (float)R;
}

// Split-K combine for the weight-gradient GEMMs: the GEMM writes each K-chunk's f32 partial
// [R][C] tile set to its own slab with plain 16-byte stores (no f32 atomics, which the chip
// retires at ~1.3 TB/s, and no memset of the output), and this kernel sums the S slabs once,
// reading each slab as one streaming pass.  The output's columns may be split into column
// blocks of width cb stored as separate [R][cb] matrices (out_bs apart): the fused dW[q|k|v]
// GEMM produces [640][1536] slabs whose column blocks are dWq, dWk, dWv.
// 4 consecutive slab elements as f32 from f32 or bf16 slabs (bf16 slabs: the weight-gradient
// GEMM's split-K partials rounded once each, summed here in f32)
template <typename ST>
__device__ __forceinline__ f32x4 ld_slab4(const ST* __restrict__ p, long e) {
  // global (not flat) loads: they retire in order, so a loop can wait for an older group with a
  // counted vmcnt while a younger one is in flight (a flat load forces vmcnt(0) + lgkmcnt(0))
  if constexpr (sizeof(ST) == 4) {
    return *(const __attribute__((address_space(1))) f32x4*)(reinterpret_cast<const float*>(p) + e);
  } else {
    const u32x2 r = *(const __attribute__((address_space(1))) u32x2*)(reinterpret_cast<const bf16_t*>(p) + e);
    return f32x4{__uint_as_float(r[0] << 16), __uint_as_float(r[0] & 0xffff0000u), __uint_as_float(r[1] << 16),
                 __uint_as_float(r[1] & 0xffff0000u)};
  }
}

template <typename ST>
__global__ __launch_bounds__(256) void slab_reduce_kernel(const ST* __restrict__ slabs, int S, long slab_stride,
                                                          int R, int C, float* __restrict__ out, int cb,
                                                          long out_bs, int accumulate,
                                                          bf16_t* __restrict__ out_bf16, float* __restrict__ tail,
                                                          bf16_t* __restrict__ tail_bf16, int tail_n,
                                                          float tail_val) {
  // constant tail (the bias gradient R * bf16(g) of a loss-sum cotangent, stored right after
  // dW in the joint gradient buffer): written here instead of by a launch of its own
  if (blockIdx.x == 0) {
    for (int i = threadIdx.x; i < tail_n; i += blockDim.x) {
      tail[i] = tail_val;
      if (tail_bf16) tail_bf16[i] = f2bf(tail_val);
    }
  }
  const long n4 = (long)R * C / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long e = 4 * i;
    f32x4 acc = ld_slab4(slabs, e);
    int s = 1;
    for (; s + 3 < S; s += 4) {  // 4 independent slab loads in flight
      f32x4 v0 = ld_slab4(slabs, s * slab_stride + e);
      f32x4 v1 = ld_slab4(slabs, (s + 1) * slab_stride + e);
      f32x4 v2 = ld_slab4(slabs, (s + 2) * slab_stride + e);
      f32x4 v3 = ld_slab4(slabs, (s + 3) * slab_stride + e);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; s < S; ++s) acc += ld_slab4(slabs, s * slab_stride + e);
    const int r = (int)(e / C), c = (int)(e % C);
    float* dst = out + (long)(c / cb) * out_bs + (long)r * cb + (c % cb);
    if (accumulate) acc += *reinterpret_cast<const f32x4*>(dst);
    *reinterpret_cast<f32x4*>(dst) = acc;
    if (out_bf16)  // bf16 twin (same layout): the data-parallel all-reduce's wire buffer
      *reinterpret_cast<u32x2*>(out_bf16 + (dst - out)) = u32x2{pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3])};
  }
}

// The cotangent of y.sum() reaching a dense layer is ONE scalar g broadcast over [R][C]: write
// the bf16 row the GEMMs read with ld = 0 and, in the same launch, the bias gradient (the
// column sums of that broadcast, R * bf16(g) per column) -- one kernel instead of two.
__global__ void bcast_scalar_kernel(const void* __restrict__ g, int g_bf16, int C, float R, bf16_t* __restrict__ row,
                                    float* __restrict__ db, bf16_t* __restrict__ db_bf16) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float v = g_bf16 ? bf2f(*reinterpret_cast<const bf16_t*>(g)) : *reinterpret_cast<const float*>(g);
  const bf16_t b = f2bf(v);
  row[c] = b;
  if (db) db[c] = bf2f(b) * R;
  if (db_bf16) db_bf16[c] = f2bf(bf2f(b) * R);  // the bias gradient's bf16 wire twin
}

// sum of n f32 partials (a producer's fused per-wave output sums) -> scalar, one block
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ p, int n, void* __restrict__ out,
                                                          int out_bf16) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += p[i];
  s = warp_sum64(s);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (part[0] + part[1]) + (part[2] + part[3]);
    if (out_bf16) *reinterpret_cast<bf16_t*>(out) = f2bf(v);
    else *reinterpret_cast<float*>(out) = v;
  }
}

// out[0..n) = (bf16) *g: materialises the broadcast row of a scalar cotangent (e.g. of y.sum())
__global__ void fill_row_kernel(const void* __restrict__ g, int g_bf16, bf16_t* __restrict__ out, long n) {
  const float v = g_bf16 ? bf2f(*reinterpret_cast<const bf16_t*>(g)) : *reinterpret_cast<const float*>(g);
  const bf16_t b = f2bf(v);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] = b;
}

// column sums of a bf16 [R][C] matrix (C % 8 == 0, row stride ld; ld may be 0 = broadcast row):
// block = 8 column-lanes (16 B each, 64 columns) x 32 row-lanes; LDS reduction, one atomic per column.
__global__ void colsum_vec_kernel(const bf16_t* __restrict__ in, int R, int C, long ld, int rows_per_block,
                                  float* __restrict__ out) {
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cl * 8;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(R, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < C) {
    for (int r = r0 + rl; r < r1; r += 32) {
      u32x4 v = *reinterpret_cast<const u32x4*>(in + (long)r * ld + c0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(v[k] << 16);
        acc[2 * k + 1] += __uint_as_float(v[k] & 0xffff0000u);
      }
    }
  }
  __shared__ float red[32][65];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rl][cl * 8 + k] = acc[k];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int r = 0; r < 32; ++r) s += red[r][threadIdx.x];
    int c = blockIdx.x * 64 + threadIdx.x;
    if (c < C) atomicAdd(out + c, s);
  }
}

// out[c] (+)= sum_r in[r][c]; grid.x over column blocks of 256, grid.y over row slabs.
template <typename T>
__global__ void colsum_kernel(const T* __restrict__ in, int R, int C, long ld, float* __restrict__ out) {
  int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  int rows_per = (R + gridDim.y - 1) / gridDim.y;
  int r0 = blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += ldv<T>(in, (long)r * ld + c);
  atomicAdd(out + c, s);
}

// row softmax over the last dim (f32), one wave per row
__global__ void softmax_rows_f32(const float* __restrict__ in, float* __restrict__ out, long rows, int L) {
  long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* x = in + row * L;
  float* y = out + row * L;
  float m = -INFINITY;
  for (int i = lane; i < L; i += 64) m = fmaxf(m, x[i]);
  m = warp_max64(m);
  float s = 0.f;
  for (int i = lane; i < L; i += 64) s += __expf(x[i] - m);
  s = warp_sum64(s);
  float inv = 1.f / s;
  for (int i = lane; i < L; i += 64) y[i] = __expf(x[i] - m) * inv;
}

// ------------------------------------------------------------------ fused Adam
// m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr * (m/bc1 / (sqrt(v/bc2) + eps) + wd p)
// bias corrections from the device-side step counter (graph-capture friendly).
template <typename G>
__global__ void adam_kernel(const float* __restrict__ p, const G* __restrict__ g, const float* __restrict__ m,
                            const float* __restrict__ v, float* __restrict__ po, float* __restrict__ mo,
                            float* __restrict__ vo, const int* __restrict__ step, long n, float lr, float b1,
                            float b2, float eps, float wd) {
  const float t = (float)(*step);
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float inv_bc1 = 1.f / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  long stride = (long)gridDim.x * blockDim.x * 4;
  for (; i < n; i += stride) {
    if (i + 4 <= n) {
      f32x4 pp = *reinterpret_cast<const f32x4*>(p + i);
      f32x4 mm = *reinterpret_cast<const f32x4*>(m + i);
      f32x4 vv = *reinterpret_cast<const f32x4*>(v + i);
      f32x4 gg;
#pragma unroll
      for (int k = 0; k < 4; ++k) gg[k] = ldv<G>(g, i + k);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mm[k] = b1 * mm[k] + (1.f - b1) * gg[k];
        vv[k] = b2 * vv[k] + (1.f - b2) * gg[k] * gg[k];
        float u = (mm[k] * inv_bc1) / (sqrtf(vv[k]) * inv_sqrt_bc2 + eps) + wd * pp[k];
        pp[k] -= lr * u;
      }
      *reinterpret_cast<f32x4*>(po + i) = pp;
      *reinterpret_cast<f32x4*>(mo + i) = mm;
      *reinterpret_cast<f32x4*>(vo + i) = vv;
    } else {
      for (long j = i; j < n; ++j) {
        float gg = ldv<G>(g, j);
        float mm = b1 * m[j] + (1.f - b1) * gg;
        float vv = b2 * v[j] + (1.f - b2) * gg * gg;
        float u = (mm * inv_bc1) / (sqrtf(vv) * inv_sqrt_bc2 + eps) + wd * p[j];
        po[j] = p[j] - lr * u;
        mo[j] = mm;
        vo[j] = vv;
      }
    }
  }
}

// Multi-tensor Adam over 64x64 tiles of up to 32 parameters per launch (pointers passed by value
// in the kernel arguments, so the launch is HIP-graph capturable).  Besides p/m/v (in place) it
// refreshes the parameter's bf16 "shadows" used by the next step's MFMA GEMMs: the plain [R][C]
// copy and the transposed [C][R] copy (staged through LDS so both writes are coalesced).  This
// removes every per-step f32->bf16 weight cast kernel from the training step.
struct AdamTensor {
  long p, g, m, v, st, sn, R, C, g_bf16, tiles_c, vec;  // vec: 4-wide path allowed (C % 4, alignment)
  // MX-fp8 shadows of the new weight (0 = none; R, C % 64 == 0, 64-row tiles, vec path):
  // qn[R][C] + sn8[R][C/32] (blocks along rows, quant_mx_rows' layout: a dX GEMM's B operand)
  // and qt[C][R] + st8[C][R/32] (blocks along columns, transposed: a forward GEMM's B operand)
  long qn, sn8, qt, st8;
  // gradient source: gS = 0 a plain [R][C] tensor (row stride g_ld = C); gS > 0 the gS f32
  // split-K slabs of a weight-gradient GEMM, g_ss floats apart, row stride g_ld (the gradient is
  // their sum, added in slab_reduce's order: bit-identical, and no combine launch); gS = -1 a
  // constant gradient whose f32 bits are g_ld (the bias gradient of a loss-sum cotangent)
  long gS, g_ld, g_ss;
  long trows;   // tile height: the launch's kAdamRows, or 16 / 32 (4-wide path, C % 64 == 0)
};

// the slab sum of slab_reduce_kernel, in its order (bit-identical results)
template <typename ST>
__device__ __forceinline__ float slab_sum1(const ST* __restrict__ g, long gS, long ss, long i) {
  auto ld = [&](long j) {
    if constexpr (sizeof(ST) == 4) return reinterpret_cast<const float*>(g)[j];
    else return bf2f(reinterpret_cast<const bf16_t*>(g)[j]);
  };
  float acc = ld(i);
  long s = 1;
  for (; s + 3 < gS; s += 4) acc += (ld(s * ss + i) + ld((s + 1) * ss + i)) + (ld((s + 2) * ss + i) + ld((s + 3) * ss + i));
  for (; s < gS; ++s) acc += ld(s * ss + i);
  return acc;
}
#ifndef LJS_ADAM_SLAB_DB
#define LJS_ADAM_SLAB_DB 1
#endif
constexpr int kAdamMax = 32;
// rows per Adam tile (x 64 columns): a template parameter (LJS_ADAM_ROWS = 16 / 32 / 64); smaller
// tiles give more, shorter workgroups (a ragged last round of 64-row tiles idles most CUs)
struct AdamBatch {
  AdamTensor t[kAdamMax];
  int tile_start[kAdamMax + 1];
  int n;
};

// `step_offset`: the kernel uses t = *step + step_offset (the optimizer's count as of the last
// increment plus the increments still pending, ops/hip.py adam_multi).  kThreads: 256 (16 rows x 64
// columns per pass).  512 / 1024 (more waves per tile, fewer loads per thread) measured the same,
// 20.9 / 21.7 / 21.5 us in the B=64 step (gpurun_out/r5m).  The count increment is its own one-lane
// launch, one per graph segment: an in-kernel two-level arrival ticket (the last-arriving block
// stores the new count) measured no better in the step and cost 13.2 vs 10.8 us in the probe
// (scripts/adam_probe.py, profiles/r5n_adam_probe_*.txt), so it was removed.

// Blocks past the Adam tiles (cast_n > 0): the next training step's f32 -> bf16 input cast
// (ops/linear.py, the early input cast), run by the same launch so its streaming blocks fill the
// CUs as the Adam blocks drain (both are bandwidth-bound) instead of starting a kernel after them.
struct CastJob {
  const float* src;
  bf16_t* dst;
  long n;
};

template <int kAdamRows, int kThreads>
__global__ __launch_bounds__(kThreads) void adam_multi_kernel(AdamBatch batch, int* __restrict__ step, int step_offset,
                                                         float lr, float b1, float b2, float eps, float wd,
                                                         CastJob cast) {
  __shared__ float tr[kAdamRows][65];
  const int id = blockIdx.x;
  if (cast.n > 0 && id >= batch.tile_start[batch.n]) {
    // cast_f32_bf16's loop over the cast blocks (same rounding)
    const int cb = id - batch.tile_start[batch.n], ncb = (int)gridDim.x - batch.tile_start[batch.n];
    long i8 = ((long)cb * kThreads + threadIdx.x) * 8;
    const long stride = (long)ncb * kThreads * 8;
    for (; i8 + 8 <= cast.n; i8 += stride) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(cast.src + i8);
      const f32x4 c = *reinterpret_cast<const f32x4*>(cast.src + i8 + 4);
      u32x4 o;
      o[0] = pack_bf16x2(a[0], a[1]);
      o[1] = pack_bf16x2(a[2], a[3]);
      o[2] = pack_bf16x2(c[0], c[1]);
      o[3] = pack_bf16x2(c[2], c[3]);
      *reinterpret_cast<u32x4*>(cast.dst + i8) = o;
    }
    if (i8 < cast.n)
      for (long j = i8; j < cast.n; ++j) cast.dst[j] = f2bf(cast.src[j]);
    return;
  }
  // tensor of this tile: every tile_start compared at once (the loop form chained one kernel-
  // argument load per tensor before the tile's first data load could issue)
  int ti = 0;
#pragma unroll
  for (int i = 1; i < kAdamMax; ++i) ti += (i < batch.n && id >= batch.tile_start[i]) ? 1 : 0;
  const AdamTensor T = batch.t[ti];
  const int local = id - batch.tile_start[ti];
  const int tr_i = local / (int)T.tiles_c, tc_i = local % (int)T.tiles_c;
  const int s0 = *step;
  const float t = (float)(s0 + step_offset);
  const float inv_bc1 = 1.f / (1.f - powf(b1, t)), inv_sqrt_bc2 = rsqrtf(1.f - powf(b2, t));
  float* P = reinterpret_cast<float*>(T.p);
  float* Mm = reinterpret_cast<float*>(T.m);
  float* Vv = reinterpret_cast<float*>(T.v);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int col = tc_i * 64 + tx;
  constexpr int RPP = kThreads / 16;   // rows per pass of the 4-wide path
  // the 4-wide path of one tile of TR = RPP x NQ rows (the tensor's tile height T.trows)
  auto vec_tile = [&](auto nq_tag) {
    constexpr int NQ = decltype(nq_tag)::value;
    constexpr int TR = RPP * NQ;
    static_assert(NQ >= 1 && TR <= kAdamRows, "tile height");
    // full-width column block, 16-byte aligned rows: each thread owns 4 consecutive columns of
    // NQ rows (all loads issued up front), vector p/m/v/g loads and stores, 8-byte bf16
    // shadow stores; the transposed shadow leaves as 8-byte stores from the LDS transpose
    const int c4 = (threadIdx.x & 15) * 4, r0 = threadIdx.x >> 4;
    const long cbase = (long)tc_i * 64 + c4;
    f32x4 gv[NQ], mv[NQ], vv[NQ], pv[NQ];
    bool ok[NQ];
    long gix[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int row = tr_i * TR + r0 + RPP * q;
      ok[q] = row < T.R;
      gix[q] = ok[q] ? (long)row * T.g_ld + cbase : cbase;
      const long i = ok[q] ? (long)row * T.C + cbase : cbase;
      // (global, not flat, loads: see ld_slab4)
      mv[q] = *(const __attribute__((address_space(1))) f32x4*)(Mm + i);
      vv[q] = *(const __attribute__((address_space(1))) f32x4*)(Vv + i);
      pv[q] = *(const __attribute__((address_space(1))) f32x4*)(P + i);
    }
    if (T.gS > 0) {
      // the slab sum of slab_reduce_kernel (same order, bit-identical) with the loads of all NQ
      // rows of a 4-slab group in flight together; f32 or bf16 slabs (T.g_bf16)
      auto slab_sum = [&](auto tag) {
        using ST = decltype(tag);
        const ST* G = reinterpret_cast<const ST*>(T.g);
#pragma unroll
        for (int q = 0; q < NQ; ++q) gv[q] = ld_slab4(G, gix[q]);
        long s = 1;
#if LJS_ADAM_SLAB_DB
        // groups of 4 slabs double-buffered: group g + 1's loads are issued before group g is
        // added, so a tile with S slabs pays ~S / 8 exposed round trips instead of S / 4 (dWo at
        // B=64: 24 slabs).  Same additions in the same order as slab_reduce (bit-identical).
        // (tiles of <= 32 rows: two 64-row buffers would spill)
        const long full = NQ <= 2 ? 1 + ((T.gS - 1) / 4) * 4 : 1;   // slabs [1, full) in groups of 4
        if (s < full) {
          f32x4 va[NQ][4], vb[NQ][4];
          auto load = [&](f32x4 (&v)[NQ][4], long s0) {
#pragma unroll
            for (int q = 0; q < NQ; ++q)
#pragma unroll
              for (int j = 0; j < 4; ++j) v[q][j] = ld_slab4(G, (s0 + j) * T.g_ss + gix[q]);
          };
          auto add = [&](f32x4 (&v)[NQ][4]) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) gv[q] += (v[q][0] + v[q][1]) + (v[q][2] + v[q][3]);
          };
          load(va, s);
          for (;;) {
            if (s + 4 < full) load(vb, s + 4);
            add(va);
            s += 4;
            if (s >= full) break;
            if (s + 4 < full) load(va, s + 4);
            add(vb);
            s += 4;
            if (s >= full) break;
          }
        }
#endif
        for (; s + 3 < T.gS; s += 4) {
          f32x4 v[NQ][4];
#pragma unroll
          for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[q][j] = ld_slab4(G, (s + j) * T.g_ss + gix[q]);
#pragma unroll
          for (int q = 0; q < NQ; ++q) gv[q] += (v[q][0] + v[q][1]) + (v[q][2] + v[q][3]);
        }
        // the 1-3 remaining slabs: their loads issued together (one round trip, not one each),
        // added one by one in slab_reduce's order
        if (NQ <= 2 && s < T.gS) {   // (64-row tiles: registers would halve the occupancy)
          f32x4 r[NQ][3];
#pragma unroll
          for (int j = 0; j < 3; ++j)
            if (s + j < T.gS) {
#pragma unroll
              for (int q = 0; q < NQ; ++q) r[q][j] = ld_slab4(G, (s + j) * T.g_ss + gix[q]);
            }
#pragma unroll
          for (int j = 0; j < 3; ++j)
            if (s + j < T.gS) {
#pragma unroll
              for (int q = 0; q < NQ; ++q) gv[q] += r[q][j];
            }
          s = T.gS;
        }
        for (; s < T.gS; ++s) {
#pragma unroll
          for (int q = 0; q < NQ; ++q) gv[q] += ld_slab4(G, s * T.g_ss + gix[q]);
        }
      };
      if (T.g_bf16) slab_sum(bf16_t{});
      else slab_sum(float{});
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const long gi = gix[q];
      if (T.gS > 0) {
      } else if (T.gS < 0) {
        const float c = __int_as_float((int)T.g_ld);
        gv[q] = f32x4{c, c, c, c};
      } else if (T.g_bf16) {
        const u32x2 raw = *reinterpret_cast<const u32x2*>(reinterpret_cast<const bf16_t*>(T.g) + gi);
        gv[q] = f32x4{__uint_as_float(raw[0] << 16), __uint_as_float(raw[0] & 0xffff0000u),
                      __uint_as_float(raw[1] << 16), __uint_as_float(raw[1] & 0xffff0000u)};
      } else {
        gv[q] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(T.g) + gi);
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int rl = r0 + RPP * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = gv[q][e];
        const float m = b1 * mv[q][e] + (1.f - b1) * g;
        const float v = b2 * vv[q][e] + (1.f - b2) * g * g;
        const float p = pv[q][e];
        mv[q][e] = m;
        vv[q][e] = v;
        pv[q][e] = p - lr * ((m * inv_bc1) / (sqrtf(v) * inv_sqrt_bc2 + eps) + wd * p);
        tr[rl][c4 + e] = pv[q][e];
      }
      if (ok[q]) {
        const long i = (long)(tr_i * TR + rl) * T.C + cbase;
        *reinterpret_cast<f32x4*>(P + i) = pv[q];
        *reinterpret_cast<f32x4*>(Mm + i) = mv[q];
        *reinterpret_cast<f32x4*>(Vv + i) = vv[q];
        if (T.sn)
          *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(T.sn) + i) =
              u32x2{pack_bf16x2(pv[q][0], pv[q][1]), pack_bf16x2(pv[q][2], pv[q][3])};
      }
      if (T.qn) {
        // MX block = 32 columns of this row = the 8 lanes (tid & 15) / 8 of a 16-lane row group
        float amax = fmaxf(fmaxf(fabsf(pv[q][0]), fabsf(pv[q][1])), fmaxf(fabsf(pv[q][2]), fabsf(pv[q][3])));
        amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
        const int x = mx_exponent(amax);
        const float inv = ldexpf(1.f, -x);
        if (ok[q]) {
          const long i = (long)(tr_i * TR + rl) * T.C + cbase;
          *reinterpret_cast<unsigned*>(reinterpret_cast<unsigned char*>(T.qn) + i) =
              pack4_e4m3(pv[q][0] * inv, pv[q][1] * inv, pv[q][2] * inv, pv[q][3] * inv);
          if ((threadIdx.x & 7) == 0) reinterpret_cast<unsigned char*>(T.sn8)[i / 32] = (unsigned char)(x + 127);
        }
      }
    }
    if (T.st || T.qt) {
      __syncthreads();
      // shadow_t[c][r]: thread -> 4 consecutive rows r4..r4+3 of output row c (bank-conflict
      // free: tr's row stride is 65 words)
      constexpr int RL = TR / 4;            // lanes across the tile's rows
      const int r4 = (threadIdx.x % RL) * 4, cl0 = threadIdx.x / RL;
      const int orow0 = tc_i * 64, ocol = tr_i * TR + r4;
      const bool rows_vec = (T.R & 3) == 0 && ocol + 4 <= T.R;
      static_assert(kThreads / RL <= 64, "transpose pass wider than the tile");
#pragma unroll
      for (int q = 0; q < 64 / (kThreads / RL); ++q) {
        const int cl = cl0 + (kThreads / RL) * q, c = orow0 + cl;
        if (T.st) {
          bf16_t* dst = reinterpret_cast<bf16_t*>(T.st) + (long)c * T.R + ocol;
          if (rows_vec) {
            *reinterpret_cast<u32x2*>(dst) = u32x2{pack_bf16x2(tr[r4][cl], tr[r4 + 1][cl]),
                                                   pack_bf16x2(tr[r4 + 2][cl], tr[r4 + 3][cl])};
          } else {
            for (int k = 0; k < 4 && ocol + k < T.R; ++k) dst[k] = f2bf(tr[r4 + k][cl]);
          }
        }
        if (T.qt) {
          // MX block = 32 consecutive rows of column c = 8 lanes of RL (= 16 at 64-row tiles)
          const float a0 = tr[r4][cl], a1 = tr[r4 + 1][cl], a2 = tr[r4 + 2][cl], a3 = tr[r4 + 3][cl];
          float amax = fmaxf(fmaxf(fabsf(a0), fabsf(a1)), fmaxf(fabsf(a2), fabsf(a3)));
          amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
          amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
          amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
          const int x = mx_exponent(amax);
          const float inv = ldexpf(1.f, -x);
          const long o = (long)c * T.R + ocol;
          *reinterpret_cast<unsigned*>(reinterpret_cast<unsigned char*>(T.qt) + o) =
              pack4_e4m3(a0 * inv, a1 * inv, a2 * inv, a3 * inv);
          if ((threadIdx.x & 7) == 0) reinterpret_cast<unsigned char*>(T.st8)[o / 32] = (unsigned char)(x + 127);
        }
      }
    }
  };
  if (T.vec && (tc_i + 1) * 64 <= T.C) {
    // per-tensor tile height (the launch's choice): shorter tiles for tensors with many gradient
    // slabs, so their blocks' slab streams are no longer the kernel's tail
    if constexpr (RPP == 16) {
      if (T.trows == 16) vec_tile(std::integral_constant<int, 1>{});
      else if (kAdamRows >= 32 && T.trows == 32) vec_tile(std::integral_constant<int, (kAdamRows >= 32 ? 2 : 1)>{});
      else vec_tile(std::integral_constant<int, kAdamRows / RPP>{});
    } else {
      vec_tile(std::integral_constant<int, kAdamRows / RPP>{});
    }
    return;
  }
#pragma unroll 4
  for (int rr = 0; rr < kAdamRows / (kThreads / 64); ++rr) {
    const int rl = ty + (kThreads / 64) * rr, row = tr_i * kAdamRows + rl;
    float newp = 0.f;
    if (row < T.R && col < T.C) {
      const long i = (long)row * T.C + col;
      const long gi = (long)row * T.g_ld + col;
      float g = T.gS > 0   ? (T.g_bf16 ? slab_sum1(reinterpret_cast<const bf16_t*>(T.g), T.gS, T.g_ss, gi)
                                        : slab_sum1(reinterpret_cast<const float*>(T.g), T.gS, T.g_ss, gi))
                : T.gS < 0 ? __int_as_float((int)T.g_ld)
                : T.g_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(T.g)[gi])
                           : reinterpret_cast<const float*>(T.g)[gi];
      float m = b1 * Mm[i] + (1.f - b1) * g;
      float v = b2 * Vv[i] + (1.f - b2) * g * g;
      float p = P[i];
      newp = p - lr * ((m * inv_bc1) / (sqrtf(v) * inv_sqrt_bc2 + eps) + wd * p);
      P[i] = newp;
      Mm[i] = m;
      Vv[i] = v;
      if (T.sn) reinterpret_cast<bf16_t*>(T.sn)[i] = f2bf(newp);
    }
    tr[rl][tx] = newp;
  }
  if (T.st) {
    __syncthreads();
    const int orow0 = tc_i * 64;  // shadow_t[c][r]
    for (int idx = threadIdx.x; idx < kAdamRows * 64; idx += kThreads) {
      const int r = idx % kAdamRows, cl = idx / kAdamRows, c = orow0 + cl, ocol = tr_i * kAdamRows + r;
      if (c < T.C && ocol < T.R) reinterpret_cast<bf16_t*>(T.st)[(long)c * T.R + ocol] = f2bf(tr[r][cl]);
    }
  }
}

// ------------------------------------------------------------------ Philox RNG
struct RngRegion {
  long start[8];
  long size[8];
  long gstride[8];
  int ndim;
};

__device__ __forceinline__ void philox10(unsigned& c0, unsigned& c1, unsigned& c2, unsigned& c3, unsigned k0,
                                         unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
    unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    unsigned n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ double u01(unsigned x) { return ((double)(x >> 8) + 0.5) * (1.0 / 16777216.0); }

template <typename T>
__global__ void rng_kernel(T* __restrict__ out, RngRegion reg, long n, unsigned k0, unsigned k1, int dist, float lo,
                           float hi, float erf_a, float erf_b) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    // local row-major index -> global linear index
    long rem = i, gidx = 0;
    for (int d = reg.ndim - 1; d >= 0; --d) {
      long li = rem % reg.size[d];
      rem /= reg.size[d];
      gidx += (reg.start[d] + li) * reg.gstride[d];
    }
    unsigned c0 = (unsigned)gidx, c1 = (unsigned)(gidx >> 32), c2 = 0, c3 = 0;
    philox10(c0, c1, c2, c3, k0, k1);
    float val;
    if (dist == 0) {  // normal (Box-Muller)
      double u1 = u01(c0), u2 = u01(c1);
      val = (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
    } else if (dist == 1) {  // uniform
      val = (float)(lo + (hi - lo) * u01(c0));
    } else {  // truncated normal (inverse CDF)
      double u = erf_a + (erf_b - erf_a) * u01(c0);
      double z = 1.4142135623730951 * erfinv(u);
      val = (float)fmin(fmax(z, (double)lo), (double)hi);
    }
    if constexpr (sizeof(T) == 4) out[i] = val;
    else out[i] = f2bf(val);
  }
}

// Dropout with a counter-based mask (no mask stored): element i of the shard is kept iff the
// Philox uniform of its GLOBAL index is < keep (the draw of random.uniform for that index, so the
// mask is mesh-invariant and equal to the host path's), kept values divided by keep.  The
// backward is the same kernel on dY (the mask is recomputed from the key).
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, RngRegion reg, long n, unsigned k0,
                               unsigned k1, float keep) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    long rem = i, gidx = 0;
    for (int d = reg.ndim - 1; d >= 0; --d) {
      const long li = rem % reg.size[d];
      rem /= reg.size[d];
      gidx += (reg.start[d] + li) * reg.gstride[d];
    }
    unsigned c0 = (unsigned)gidx, c1 = (unsigned)(gidx >> 32), c2 = 0, c3 = 0;
    philox10(c0, c1, c2, c3, k0, k1);
    const float u = (float)u01(c0);
    if constexpr (sizeof(T) == 4) {
      y[i] = u < keep ? x[i] / keep : 0.f;
    } else {
      y[i] = u < keep ? f2bf(bf2f(x[i]) / keep) : (bf16_t)0;
    }
  }
}

// out[s][b][k] = bf16(in[b][s][k]) for a [B][S][K] f32 or bf16 array (K % 8 == 0): the activations'
// (batch, seq) storage order swapped to seq-major while they are rounded to bf16, so a sequence-
// sharded layer gathers / scatters whole contiguous blocks (ops/linear.py, ops/hip.py storage_order)
template <typename T>
__global__ void swap01_bf16_kernel(const T* __restrict__ in, bf16_t* __restrict__ out, int B, int S, int K8) {
  // blockIdx.y = output row s (no 64-bit divisions per element); x covers its B * K8 chunks
  const int s = blockIdx.y;
  const int nbk = B * K8;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nbk; j += gridDim.x * blockDim.x) {
    const int b = j / K8, k8 = j - b * K8;
    const long o = (long)s * nbk + j;
    const long i = ((long)b * S + s) * K8 + k8;
    u32x4 w;
    if constexpr (sizeof(T) == 4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(in + i * 8);
      const f32x4 c = *reinterpret_cast<const f32x4*>(in + i * 8 + 4);
      w[0] = pack_bf16x2(a[0], a[1]);
      w[1] = pack_bf16x2(a[2], a[3]);
      w[2] = pack_bf16x2(c[0], c[1]);
      w[3] = pack_bf16x2(c[2], c[3]);
    } else {
      w = *reinterpret_cast<const u32x4*>(in + i * 8);
    }
    *reinterpret_cast<u32x4*>(out + o * 8) = w;
  }
}


// out[c][r] = in[r][c] for an R x C bf16 matrix (row strides ldi / ldo), 64x64 tiles through LDS:
// the plain [in][out] shadow of a weight derived from its gathered transposed shadow.  16-byte
// loads (8 columns of one row per lane) and 16-byte stores (8 rows of one output row per lane);
// the LDS tile rows are padded so the transposed reads spread over the banks.
__global__ void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out, int R, int C, long ldi,
                                      long ldo) {
  __shared__ unsigned short tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;                 // 256 threads
  const bool vec = (C % 8 == 0) && (R % 8 == 0) && (ldi % 8 == 0) && (ldo % 8 == 0) &&
                   ((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0;
  if (vec) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {            // 64 rows x 8 chunks of 8 columns
      const int idx = t + 256 * p, row = idx >> 3, ch = idx & 7;
      const int r = r0 + row, c = c0 + ch * 8;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (r < R && c < C) v = *reinterpret_cast<const u32x4*>(in + (long)r * ldi + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tile[row][ch * 8 + 2 * k] = (unsigned short)(v[k] & 0xffffu);
        tile[row][ch * 8 + 2 * k + 1] = (unsigned short)(v[k] >> 16);
      }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; ++p) {            // 64 output rows (= input columns) x 8 chunks of 8 rows
      const int idx = t + 256 * p, oc = idx >> 3, ch = idx & 7;
      const int c = c0 + oc, r = r0 + ch * 8;
      if (c < C && r < R) {
        u32x4 v;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = (unsigned)tile[ch * 8 + 2 * k][oc] | ((unsigned)tile[ch * 8 + 2 * k + 1][oc] << 16);
        *reinterpret_cast<u32x4*>(out + (long)c * ldo + r) = v;
      }
    }
    return;
  }
  const int tx = t & 63, ty = t >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? in[(long)r * ldi + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) out[(long)c * ldo + r] = tile[tx][i];
  }
}

// out = sum of n same-shape f32 / bf16 arrays (f32 accumulation, output in the inputs' dtype): the
// loopback reduce-scatter / all-reduce over virtual devices that share one GPU, in ONE launch
struct SumPtrs {
  const void* p[128];
};

template <typename T>
__global__ void sum_n_kernel(SumPtrs sp, int n, long count, T* __restrict__ out) {
  const T* const* ins = reinterpret_cast<const T* const*>(sp.p);
  constexpr int V = 16 / sizeof(T);
  const long nv = count / V;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    // inputs in groups of 4: four independent 16-byte loads in flight per thread (in order:
    // the sum is the same left-to-right f32 sum for every group size)
    for (int j0 = 0; j0 < n; j0 += 4) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j0 + u < n) v[u] = *reinterpret_cast<const u32x4*>(ins[j0 + u] + i * V);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j0 + u >= n) break;
        if constexpr (sizeof(T) == 4) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] += __uint_as_float(v[u][e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[2 * e] += __uint_as_float(v[u][e] << 16);
            acc[2 * e + 1] += __uint_as_float(v[u][e] & 0xffff0000u);
          }
        }
      }
    }
    u32x4 o;
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = __float_as_uint(acc[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack_bf16x2(acc[2 * e], acc[2 * e + 1]);
    }
    *reinterpret_cast<u32x4*>(out + i * V) = o;
  }
  if (blockIdx.x == 0) {
    for (long j = nv * V + threadIdx.x; j < count; j += blockDim.x) {
      float a = 0.f;
      for (int k = 0; k < n; ++k) {
        if constexpr (sizeof(T) == 4) a += ins[k][j];
        else a += bf2f(ins[k][j]);
      }
      if constexpr (sizeof(T) == 4) out[j] = a;
      else out[j] = f2bf(a);
    }
  }
}

}  // namespace

// ============================================================================ C ABI
LJS_API int ljs_cast_f32_bf16(const void* in, void* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16, dim3(grid_for(n, 256 * 8)), dim3(256), 0, s, (const float*)in, (bf16_t*)out, n);
  return (int)hipGetLastError();
}

LJS_API int ljs_swap01_bf16(const void* in, int in_bf16, void* out, int B, int S, int K, hipStream_t s) {
  if (K % 8 || (((uintptr_t)in) & 15) || (((uintptr_t)out) & 15)) return (int)hipErrorInvalidValue;
  const long nbk = (long)B * (K / 8);
  if (S > 65535 || nbk >= (1L << 31)) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)((nbk + 255) / 256 < 64 ? (nbk + 255) / 256 : 64), (unsigned)S);
  if (in_bf16)
    hipLaunchKernelGGL(swap01_bf16_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, B, S,
                       K / 8);
  else
    hipLaunchKernelGGL(swap01_bf16_kernel<float>, g, dim3(256), 0, s, (const float*)in, (bf16_t*)out, B, S,
                       K / 8);
  return (int)hipGetLastError();
}

LJS_API int ljs_transpose_bf16(const void* in, void* out, int R, int C, long ldi, long ldo, hipStream_t s) {
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, R, C, ldi, ldo);
  return (int)hipGetLastError();
}

LJS_API int ljs_sum_n(const void* const* ins, int n, int is_bf16, long count, void* out, hipStream_t s) {
  // the n input pointers travel BY VALUE in the kernel arguments (graph-capturable, no copy)
  if (n < 1 || n > 128 || (((uintptr_t)out) & 15)) return (int)hipErrorInvalidValue;
  SumPtrs sp = {};
  for (int j = 0; j < n; ++j) {
    if (((uintptr_t)ins[j]) & 15) return (int)hipErrorInvalidValue;
    sp.p[j] = ins[j];
  }
  const int g = grid_for(count / (is_bf16 ? 8 : 4) + 1, 256);
  if (is_bf16)
    hipLaunchKernelGGL(sum_n_kernel<bf16_t>, dim3(g), dim3(256), 0, s, sp, n, count, (bf16_t*)out);
  else
    hipLaunchKernelGGL(sum_n_kernel<float>, dim3(g), dim3(256), 0, s, sp, n, count, (float*)out);
  return (int)hipGetLastError();
}

// out[c] = sum_r in[r][c] for a SHORT f32 matrix (the per-row-tile partials a GEMM epilogue wrote):
// one workgroup per 64 columns, its 4 waves take every 4th row with all of a lane's loads issued
// before the first add, then one LDS combine -- one memory round trip instead of the column-sum
// kernels' long-R loop (3 workgroups, ~21 us for 64 x 640) or slab_reduce's one workgroup
__global__ __launch_bounds__(256) void rows_sum_f32_kernel(const float* __restrict__ in, int R, int C, long ld,
                                                          float* __restrict__ out) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  float acc = 0.f;
  if (c < C) {
    int r = w;
    for (; r + 28 < R; r += 32) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = in[(long)(r + 4 * i) * ld + c];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += v[i];
    }
    for (; r < R; r += 4) acc += in[(long)r * ld + c];
  }
  part[w][threadIdx.x & 63] = acc;
  __syncthreads();
  if (w == 0 && c < C) out[c] = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
}

LJS_API int ljs_rows_sum_f32(const void* in, int R, int C, long ld, void* out, hipStream_t s) {
  if (R < 1 || C < 1 || ld < C) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_sum_f32_kernel, dim3((C + 63) / 64), dim3(256), 0, s, (const float*)in, R, C, ld,
                     (float*)out);
  return (int)hipGetLastError();
}

LJS_API int ljs_cast_bf16_f32(const void* in, void* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32, dim3(grid_for(n, 256 * 8)), dim3(256), 0, s, (const bf16_t*)in, (float*)out, n);
  return (int)hipGetLastError();
}

LJS_API int ljs_cast_transpose_f32_bf16(const void* in, void* out, int R, int C, long ldi, long ldo, hipStream_t s) {
  if ((R + 31) / 32 > 65535) return (int)hipErrorInvalidValue;
  dim3 grid((C + 31) / 32, (R + 31) / 32);
  const int vin = ldi % 4 == 0 && (((uintptr_t)in) & 15) == 0;
  const int vout = ldo % 4 == 0 && (((uintptr_t)out) & 7) == 0;
  hipLaunchKernelGGL(cast_transpose_f32_bf16, grid, dim3(256), 0, s, (const float*)in, (bf16_t*)out, R, C, ldi, ldo,
                     vin, vout);
  return (int)hipGetLastError();
}

// out (scalar, f32 or bf16 per out_bf16) = sum(in); in is f32 (is_bf16=0) or bf16.
// ws: persistent workspace of >= 1089 floats whose ticket words are zero at rest.
LJS_API int ljs_sum_all(const void* in, int is_bf16, long n, void* out, int out_bf16, void* ws, hipStream_t s) {
  // ws layout: [partials: kMaxSumBlocks][group partials: 32][top ticket][group tickets: 32]
  float* partials = (float*)ws;
  unsigned* ticket = (unsigned*)ws + kMaxSumBlocks + 32;
  const bool aligned = (((uintptr_t)in) & 15) == 0;
  if (aligned) {
    // one batch of U = 16 independent 16-byte loads per thread covers the array (21 MB of the
    // bench's bf16 output in flight at once: an HBM-latency-bound read otherwise)
    long per = 256L * (is_bf16 ? 8 : 4) * 16;
    int g = grid_for(n, (int)per);
    if (g > kMaxSumBlocks) g = kMaxSumBlocks;
    if (is_bf16)
      hipLaunchKernelGGL(sum_all_ticket_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)in, n, partials,
                         ticket, out, out_bf16);
    else
      hipLaunchKernelGGL(sum_all_ticket_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)in, n, partials,
                         ticket, out, out_bf16);
    return (int)hipGetLastError();
  }
  if (out_bf16) return (int)hipErrorInvalidValue;
  (void)hipMemsetAsync(out, 0, sizeof(float), s);
  int g = grid_for(n, 256 * 16);
  if (is_bf16)
    hipLaunchKernelGGL(sum_all_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)in, n, (float*)out);
  else
    hipLaunchKernelGGL(sum_all_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)in, n, (float*)out);
  return (int)hipGetLastError();
}

// out[C] f32 = column sums of in[R][C]; accumulate=1 adds into out
// ws (may be null): persistent workspace, >= kColsumWsFloats floats, tickets zero at rest; with it
// the bf16 vector path needs no memset (per-column-block last-arriver combine).
constexpr long kColsumWsFloats = 1L << 20;
LJS_API long ljs_colsum_ws_floats() { return kColsumWsFloats; }
LJS_API int ljs_colsum(const void* in, int is_bf16, int R, int C, long ld, void* out, int accumulate, void* ws,
                       hipStream_t s) {
  if (ld == 0) {  // one repeated row: out = R * row
    hipLaunchKernelGGL(colsum_bcast_kernel, dim3((C + 255) / 256), dim3(256), 0, s, in, is_bf16, R, C, (float*)out,
                       accumulate);
    return (int)hipGetLastError();
  }
  if (is_bf16 && C % 8 == 0 && ld % 8 == 0 && (((uintptr_t)in) & 15) == 0) {
    int cb = (C + 63) / 64;
    int want = 512 / cb;
    int gy = want < 1 ? 1 : want;
    int rpb = (R + gy - 1) / gy;
    if (rpb < 32) rpb = 32;
    gy = (R + rpb - 1) / rpb;
    // workspace layout: [tickets: 4096 words][partials: gy * C floats]
    if (ws && cb <= 4096 && (long)gy * C + 4096 <= kColsumWsFloats) {
      hipLaunchKernelGGL(colsum_ticket_kernel, dim3(cb, gy), dim3(256), 0, s, (const bf16_t*)in, R, C, ld, rpb,
                         (float*)ws + 4096, (unsigned*)ws, (float*)out, accumulate, (const bf16_t*)nullptr, 0L,
                         (bf16_t*)nullptr);
      return (int)hipGetLastError();
    }
    if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * C, s);
    hipLaunchKernelGGL(colsum_vec_kernel, dim3(cb, gy), dim3(256), 0, s, (const bf16_t*)in, R, C, ld, rpb,
                       (float*)out);
    return (int)hipGetLastError();
  }
  if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * C, s);
  int gy = R / 256;
  if (gy < 1) gy = 1;
  if (gy > 64) gy = 64;
  dim3 grid((C + 255) / 256, gy);
  if (is_bf16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)in, R, C, ld, (float*)out);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)in, R, C, ld, (float*)out);
  return (int)hipGetLastError();
}

// out (column blocks of width cb, out_bs floats apart) = sum of S f32 [R][C] slabs (slab_stride
// floats apart).  Requires C % 4 == 0, cb % 4 == 0, C % cb == 0 and 16-byte aligned buffers.
LJS_API int ljs_slab_reduce(const void* slabs, int S, long slab_stride, int R, int C, void* out, int cb, long out_bs,
                            int accumulate, void* out_bf16, void* tail, void* tail_bf16, int tail_n, float tail_val,
                            int slabs_bf16, hipStream_t s) {
  if (tail_n < 0 || (tail_n > 0 && !tail)) return (int)hipErrorInvalidValue;
  if (C % 4 || cb % 4 || C % cb || slab_stride % 4 || out_bs % 4 || S < 1 || (((uintptr_t)slabs) & 15) ||
      (((uintptr_t)out) & 15))
    return (int)hipErrorInvalidValue;
  const long n4 = (long)R * C / 4;
  int grid = (int)((n4 + 255) / 256);
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  if (out_bf16 && (((uintptr_t)out_bf16) & 7)) return (int)hipErrorInvalidValue;
  if (slabs_bf16)
    hipLaunchKernelGGL(slab_reduce_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)slabs, S, slab_stride,
                       R, C, (float*)out, cb, out_bs, accumulate, (bf16_t*)out_bf16, (float*)tail,
                       (bf16_t*)tail_bf16, tail_n, tail_val);
  else
    hipLaunchKernelGGL(slab_reduce_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)slabs, S, slab_stride, R,
                       C, (float*)out, cb, out_bs, accumulate, (bf16_t*)out_bf16, (float*)tail, (bf16_t*)tail_bf16,
                       tail_n, tail_val);
  return (int)hipGetLastError();
}

LJS_API int ljs_bcast_scalar(const void* g, int g_bf16, int C, float R, void* row, void* db, void* db_bf16,
                             hipStream_t s) {
  hipLaunchKernelGGL(bcast_scalar_kernel, dim3((C + 255) / 256), dim3(256), 0, s, g, g_bf16, C, R, (bf16_t*)row,
                     (float*)db, (bf16_t*)db_bf16);
  return (int)hipGetLastError();
}

// out (dense, row-major `full`) = src inside the box [lo, lo + size), zeros elsewhere: the
// backward of a box slice (a sharded view of a replicated array) in one launch instead of a fill
// plus a strided copy.  src element (c - lo) at sum_d (c_d - lo_d) * sstride_d.
struct PadBox {
  long full[6], lo[6], size[6], sstride[6];
  int nd;
};
template <typename T>
__global__ __launch_bounds__(256) void pad_box_kernel(const T* __restrict__ src, T* __restrict__ out, PadBox b,
                                                      long total) {
  if (b.nd == 1 && total < (1L << 31)) {   // (a vector: 32-bit index math)
    const int lo = (int)b.lo[0], n = (int)b.size[0], ss = (int)b.sstride[0];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)total; i += gridDim.x * 256) {
      const int rel = i - lo;
      out[i] = (rel >= 0 && rel < n) ? src[rel * ss] : T(0);
    }
    return;
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    long r = i, so = 0;
    bool in = true;
    for (int d = b.nd - 1; d >= 0; --d) {
      const long c = r % b.full[d];
      r /= b.full[d];
      const long rel = c - b.lo[d];
      in = in && rel >= 0 && rel < b.size[d];
      so += rel * b.sstride[d];
    }
    out[i] = in ? src[so] : T(0);
  }
}

LJS_API int ljs_pad_box(const void* src, void* out, int nd, const long* full, const long* lo, const long* size,
                        const long* sstride, int esize, hipStream_t s) {
  if (nd < 1 || nd > 6) return (int)hipErrorInvalidValue;
  PadBox b;
  long total = 1;
  for (int d = 0; d < nd; ++d) {
    b.full[d] = full[d];
    b.lo[d] = lo[d];
    b.size[d] = size[d];
    b.sstride[d] = sstride[d];
    total *= full[d];
  }
  b.nd = nd;
  if (total == 0) return 0;
  long grid = (total + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (esize == 2)
    hipLaunchKernelGGL(pad_box_kernel<unsigned short>, dim3(grid), dim3(256), 0, s, (const unsigned short*)src,
                       (unsigned short*)out, b, total);
  else if (esize == 4)
    hipLaunchKernelGGL(pad_box_kernel<unsigned>, dim3(grid), dim3(256), 0, s, (const unsigned*)src, (unsigned*)out, b,
                       total);
  else if (esize == 8)
    hipLaunchKernelGGL(pad_box_kernel<unsigned long long>, dim3(grid), dim3(256), 0, s,
                       (const unsigned long long*)src, (unsigned long long*)out, b, total);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

LJS_API int ljs_sum_partials(const void* p, int n, void* out, int out_bf16, hipStream_t s) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, (const float*)p, n, out, out_bf16);
  return (int)hipGetLastError();
}

// masked_out[R][C] = in * (mask > 0) and out[C] (f32) = its column sums, in one pass (fused ReLU
// backward + bias gradient).  bf16 in / mask with row stride ld, C % 8 == 0, 16-byte aligned.
LJS_API int ljs_relu_bwd_colsum(const void* in, const void* mask, int R, int C, long ld, long mld, void* masked_out,
                                void* out, void* ws, hipStream_t s) {
  if (C % 8 || ld % 8 || mld % 8 || (((uintptr_t)in) & 15) || (((uintptr_t)mask) & 15) || (((uintptr_t)masked_out) & 15) || !ws)
    return (int)hipErrorInvalidValue;
  int cb = (C + 63) / 64;
  int want = 512 / cb;
  int gy = want < 1 ? 1 : want;
  int rpb = (R + gy - 1) / gy;
  if (rpb < 32) rpb = 32;
  gy = (R + rpb - 1) / rpb;
  if (cb > 4096 || (long)gy * C + 4096 > kColsumWsFloats) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(colsum_ticket_kernel, dim3(cb, gy), dim3(256), 0, s, (const bf16_t*)in, R, C, ld, rpb,
                     (float*)ws + 4096, (unsigned*)ws, (float*)out, 0, (const bf16_t*)mask, mld,
                     (bf16_t*)masked_out);
  return (int)hipGetLastError();
}

// masked_out[R][C] = in * (mask > 0) without column sums (the ReLU backward of a bias-free dense):
// a flat grid over 8-element vectors fills the chip, where the column-sum kernel is limited to
// ~512 workgroups by its per-column-block reduction.  Same layout requirements as above.
__global__ void __launch_bounds__(256) relu_bwd_kernel(const bf16_t* __restrict__ in, const bf16_t* __restrict__ mask,
                                                       int C8, long n8, long ld, long mld,
                                                       bf16_t* __restrict__ masked_out) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const long r = i / C8;
    const int c = (int)(i - r * C8) * 8;
    const u32x4 v = *reinterpret_cast<const u32x4*>(in + r * ld + c);
    const u32x4 m = *reinterpret_cast<const u32x4*>(mask + r * mld + c);
    *reinterpret_cast<u32x4*>(masked_out + i * 8) = relu_mask_bf16x8(v, m);
  }
}

LJS_API int ljs_relu_bwd(const void* in, const void* mask, int R, int C, long ld, long mld, void* masked_out,
                         hipStream_t s) {
  if (C % 8 || ld % 8 || mld % 8 || (((uintptr_t)in) & 15) || (((uintptr_t)mask) & 15) || (((uintptr_t)masked_out) & 15))
    return (int)hipErrorInvalidValue;
  const long n8 = (long)R * (C / 8);
  long grid = (n8 + 255) / 256;
  if (grid > 8192) grid = 8192;  // 32 workgroups per CU, then grid-stride
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)grid), dim3(256), 0, s, (const bf16_t*)in, (const bf16_t*)mask,
                     C / 8, n8, ld, mld, (bf16_t*)masked_out);
  return (int)hipGetLastError();
}

LJS_API int ljs_fill_row_bf16(const void* g, int g_bf16, void* out, long n, hipStream_t s) {
  int grid = grid_for(n, 256);
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(fill_row_kernel, dim3(grid), dim3(256), 0, s, g, g_bf16, (bf16_t*)out, n);
  return (int)hipGetLastError();
}

LJS_API int ljs_softmax_rows_f32(const void* in, void* out, long rows, int L, hipStream_t s) {
  hipLaunchKernelGGL(softmax_rows_f32, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, (const float*)in,
                     (float*)out, rows, L);
  return (int)hipGetLastError();
}

LJS_API int ljs_adam_f32(const void* p, const void* g, int g_bf16, const void* m, const void* v, void* po, void* mo,
                         void* vo, const void* step, long n, float lr, float b1, float b2, float eps, float wd,
                         hipStream_t s) {
  int grid = grid_for(n, 256 * 4);
  if (g_bf16)
    hipLaunchKernelGGL(adam_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const float*)p, (const bf16_t*)g,
                       (const float*)m, (const float*)v, (float*)po, (float*)mo, (float*)vo, (const int*)step, n, lr,
                       b1, b2, eps, wd);
  else
    hipLaunchKernelGGL(adam_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)p, (const float*)g,
                       (const float*)m, (const float*)v, (float*)po, (float*)mo, (float*)vo, (const int*)step, n, lr,
                       b1, b2, eps, wd);
  return (int)hipGetLastError();
}

// dist: 0 normal, 1 uniform[lo,hi), 2 truncated normal on [lo,hi]; out f32 (is_bf16=0) or bf16
LJS_API int ljs_rng_fill(void* out, int is_bf16, int ndim, const long* start, const long* size, const long* gstride,
                         unsigned k0, unsigned k1, int dist, float lo, float hi, float erf_a, float erf_b,
                         hipStream_t s) {
  RngRegion reg;
  long n = 1;
  reg.ndim = ndim;
  for (int d = 0; d < ndim && d < 8; ++d) {
    reg.start[d] = start[d];
    reg.size[d] = size[d];
    reg.gstride[d] = gstride[d];
    n *= size[d];
  }
  if (ndim == 0) {
    reg.ndim = 1; reg.start[0] = 0; reg.size[0] = 1; reg.gstride[0] = 1;
  }
  int g = grid_for(n, 256 * 4);
  if (is_bf16)
    hipLaunchKernelGGL(rng_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (bf16_t*)out, reg, n, k0, k1, dist, lo, hi,
                       erf_a, erf_b);
  else
    hipLaunchKernelGGL(rng_kernel<float>, dim3(g), dim3(256), 0, s, (float*)out, reg, n, k0, k1, dist, lo, hi, erf_a,
                       erf_b);
  return (int)hipGetLastError();
}

// y = dropout(x) of one shard (see dropout_kernel); x, y contiguous f32 (is_bf16 = 0) or bf16
LJS_API int ljs_dropout(const void* x, void* y, int is_bf16, int ndim, const long* start, const long* size,
                        const long* gstride, unsigned k0, unsigned k1, float keep, hipStream_t s) {
  if (ndim < 1 || ndim > 8 || !(keep > 0.f)) return (int)hipErrorInvalidValue;
  RngRegion reg;
  long n = 1;
  reg.ndim = ndim;
  for (int d = 0; d < ndim; ++d) {
    reg.start[d] = start[d];
    reg.size[d] = size[d];
    reg.gstride[d] = gstride[d];
    n *= size[d];
  }
  if (n == 0) return 0;
  const int g = grid_for(n, 256 * 4);
  if (is_bf16)
    hipLaunchKernelGGL(dropout_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, reg, n, k0,
                       k1, keep);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, (float*)y, reg, n, k0, k1,
                       keep);
  return (int)hipGetLastError();
}

// the optimizer count's increment as its own one-lane launch (ops/hip.py adam_multi: the ticket
// form's cost in the Adam kernel exceeds a launch, scripts/adam_probe.py)
__global__ void step_add_kernel(int* step, int n) {
  if (threadIdx.x == 0) *step += n;
}
LJS_API int ljs_step_add(void* step, int n, hipStream_t s) {
  hipLaunchKernelGGL(step_add_kernel, dim3(1), dim3(64), 0, s, (int*)step, n);
  return (int)hipGetLastError();
}

// table: n x 16 int64 {p, g, m, v, shadow_t, shadow_n, R, C, g_bf16, gS, qn, sn8, qt, st8, g_ld, g_ss}
// (see AdamTensor); up to 32 per call
static int g_adam_rows = 0;
LJS_API void ljs_adam_set_rows(int rows) { g_adam_rows = rows; }
LJS_API int ljs_adam_multi(const long* table, int n, void* step, int step_offset, void* ticket, float lr, float b1,
                           float b2, float eps, float wd, const void* cast_src, void* cast_dst, long cast_n,
                           hipStream_t s) {
  if (n < 1 || n > kAdamMax) return (int)hipErrorInvalidValue;
  if (ticket) return (int)hipErrorInvalidValue;   // (the in-kernel count ticket was removed)
  CastJob cast{(const float*)cast_src, (bf16_t*)cast_dst, cast_src && cast_dst ? cast_n : 0};
  if (cast.n > 0 && ((((uintptr_t)cast.src) & 15) || (((uintptr_t)cast.dst) & 15))) return (int)hipErrorInvalidValue;
  AdamBatch b;
  // Tile height (x 64 columns): 32 rows by default -- 660 workgroups for the step's 1.3 M
  // parameters instead of 330 of 64 rows, which left a ragged second round on 256 CUs (B=8 step
  // 0.0752-0.0753 vs 0.0775-0.0778 ms, B=64 0.1987-0.2007 vs 0.2005-0.2036, x3 interleaved,
  // profiles/r5aj_adam_rows_lines.txt); 64 when a tensor carries MX-fp8 shadows (written by 64-row
  // tiles only).  ljs_adam_set_rows (16 / 32 / 64; 0 = automatic) forces the launch's height (tests).
  const int rows = g_adam_rows;
  bool any_mx = false;
  for (int i = 0; i < n; ++i) any_mx = any_mx || table[16 * i + 10] || table[16 * i + 12];
  const int kAdamRows = rows == 16 || rows == 32 || rows == 64 ? rows : (any_mx ? 64 : 32);
  // Tile heights balance the blocks' slab streams: a tensor whose gradient has r x the slabs of
  // the launch's lightest slab gradient gets half-height tiles at r >= 2 (16-row at r >= 4), so
  // its blocks are not the kernel's tail -- W_o's 24 slabs against the QKV weights' 8 at B=64, 12
  // against 4 at B=8 before the weight-gradient pair's joint split counts (B=8 step 0.0805-0.0813
  // vs 0.0824-0.0827 ms, profiles/r5x_b8_lines.txt).
  constexpr int balance = 1;
  long gs_min = 0;
  for (int i = 0; i < n; ++i) {
    const long g = table[16 * i + 9];
    if (g > 0 && (gs_min == 0 || g < gs_min)) gs_min = g;
  }
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const long* r = table + 16 * i;
    AdamTensor& t = b.t[i];
    t.p = r[0]; t.g = r[1]; t.m = r[2]; t.v = r[3]; t.st = r[4]; t.sn = r[5]; t.R = r[6]; t.C = r[7];
    t.g_bf16 = r[8];
    t.qn = r[10]; t.sn8 = r[11]; t.qt = r[12]; t.st8 = r[13];
    t.gS = r[9]; t.g_ld = r[14]; t.g_ss = r[15];
    if (t.gS == 0) t.g_ld = t.C;
    if (t.gS > 0 && (t.g_ld < t.C || t.g_ss < 1)) return (int)hipErrorInvalidValue;   // (g_bf16: bf16 slabs)
    t.tiles_c = (t.C + 63) / 64;
    auto al = [](long ptr, long a) { return ptr % a == 0; };
    t.vec = t.C % 4 == 0 && al(t.p, 16) && al(t.m, 16) && al(t.v, 16) && al(t.sn, 8) && al(t.st, 8) &&
            (t.gS < 0 || (al(t.g, t.g_bf16 ? 8 : 16) && t.g_ld % 4 == 0 && (t.gS == 0 || t.g_ss % 4 == 0)));
    // MX shadows are written by the 4-wide path of full 64 x 64 tiles only: refuse anything else
    // (a shadow left stale would silently feed old weights to the fp8 GEMMs)
    if ((t.qn || t.qt) && (!t.vec || kAdamRows != 64 || t.R % 64 || t.C % 64 || !al(t.qn, 4) || !al(t.qt, 4) ||
                           (t.qn && !t.sn8) || (t.qt && !t.st8)))
      return (int)hipErrorInvalidValue;
    t.trows = kAdamRows;
    const bool short_ok = t.vec && t.C % 64 == 0 && !t.qn && !t.qt;
    // a 64-row launch chosen for another tensor's MX shadows: the rest keep the 32-row default
    if (short_ok && rows == 0 && kAdamRows == 64) t.trows = 32;
    if (t.trows >= 32 && balance && gs_min > 0 && short_ok && t.gS >= 2 * gs_min)
      t.trows = t.gS >= 4 * gs_min || t.trows == 32 ? 16 : 32;
    b.tile_start[i] = tiles;
    tiles += (int)(((t.R + t.trows - 1) / t.trows) * t.tiles_c);
  }
  b.tile_start[n] = tiles;
  b.n = n;
  // cast blocks: one 8-element chunk per thread per pass, at most 2048 blocks (grid-stride)
  const long cast_blocks = cast.n > 0 ? std::min<long>(2048, (cast.n + 256 * 8 - 1) / (256 * 8)) : 0;
  const unsigned grid = (unsigned)(tiles + cast_blocks);
  if (kAdamRows == 16)
    hipLaunchKernelGGL((adam_multi_kernel<16, 256>), dim3(grid), dim3(256), 0, s, b, (int*)step, step_offset,
                       lr, b1, b2, eps, wd, cast);
  else if (kAdamRows == 32)
    hipLaunchKernelGGL((adam_multi_kernel<32, 256>), dim3(grid), dim3(256), 0, s, b, (int*)step, step_offset,
                       lr, b1, b2, eps, wd, cast);
  else
    hipLaunchKernelGGL((adam_multi_kernel<64, 256>), dim3(grid), dim3(256), 0, s, b, (int*)step, step_offset,
                       lr, b1, b2, eps, wd, cast);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ collective pack / unpack
// The layout changes around a collective (comm/backend.py): a tensor [A][n x s][rest] viewed
// as rows of `inner` bytes, moved to / from the rank-major buffer a collective sends and
// receives, with an optional rank permutation (tile order vs sorted process ranks), or the
// per-member parts of a loopback all-gather concatenated along the gather dim.
//   mode 0 (pack)  : dst[b][a] = src0[a][perm[b]]       (A x B rows in, B x A rows out)
//   mode 1 (unpack): dst[a][b] = src0[perm[b]][a]
//   mode 2 (concat): dst[a][b] = src_b[a]                (B separate sources of A rows each)
// One thread per 16 / 4 / 1-byte unit (the widest that divides `inner` and every address).
namespace {
constexpr int kPackMax = 64;
struct PackArgs {
  const unsigned char* src[kPackMax];
  unsigned char* dst;
  long A, B, inner;
  int mode, unit;
  int perm[kPackMax];
};

template <typename U>
__global__ void pack_rows_kernel(PackArgs p) {
  const long upr = p.inner / (long)sizeof(U);  // units per row
  const long total = p.A * p.B * upr;
  for (long u = (long)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (long)gridDim.x * blockDim.x) {
    const long row = u / upr, off = u - row * upr;
    const unsigned char* src;
    long drow;
    if (p.mode == 0) {          // out row (b, a)
      const long b = row / p.A, a = row - b * p.A;
      src = p.src[0] + (a * p.B + p.perm[b]) * p.inner;
      drow = row;
    } else {                    // out row (a, b)
      const long a = row / p.B, b = row - a * p.B;
      src = p.mode == 1 ? p.src[0] + ((long)p.perm[b] * p.A + a) * p.inner : p.src[b] + a * p.inner;
      drow = row;
    }
    reinterpret_cast<U*>(p.dst + drow * p.inner)[off] = reinterpret_cast<const U*>(src)[off];
  }
}
}  // namespace

LJS_API int ljs_pack_rows(const void* const* srcs, int nsrc, void* dst, long A, long B, long inner, int mode,
                          const int* perm, hipStream_t s) {
  if (B < 1 || B > kPackMax || A < 0 || inner < 0 || nsrc < 1 || nsrc > kPackMax || (mode == 2 && nsrc != B) ||
      mode < 0 || mode > 2)
    return (int)hipErrorInvalidValue;
  PackArgs p;
  uintptr_t al = (uintptr_t)dst | (uintptr_t)inner;
  for (int i = 0; i < nsrc; ++i) {
    p.src[i] = (const unsigned char*)srcs[i];
    al |= (uintptr_t)srcs[i];
  }
  for (int i = nsrc; i < kPackMax; ++i) p.src[i] = nullptr;
  for (int b = 0; b < kPackMax; ++b) p.perm[b] = b < B ? (perm ? perm[b] : b) : 0;
  for (int b = 0; b < B; ++b)
    if (p.perm[b] < 0 || p.perm[b] >= B) return (int)hipErrorInvalidValue;
  p.dst = (unsigned char*)dst;
  p.A = A;
  p.B = B;
  p.inner = inner;
  p.mode = mode;
  const long bytes = A * B * inner;
  if (bytes == 0) return 0;
  const int unit = (al & 15) == 0 ? 16 : ((al & 3) == 0 ? 4 : 1);
  p.unit = unit;
  const long units = bytes / unit;
  const int threads = 256;
  long blocks = (units + threads - 1) / threads;
  if (blocks > 8192) blocks = 8192;
  if (unit == 16) hipLaunchKernelGGL(pack_rows_kernel<u32x4>, dim3((unsigned)blocks), dim3(threads), 0, s, p);
  else if (unit == 4) hipLaunchKernelGGL(pack_rows_kernel<unsigned>, dim3((unsigned)blocks), dim3(threads), 0, s, p);
  else hipLaunchKernelGGL(pack_rows_kernel<unsigned char>, dim3((unsigned)blocks), dim3(threads), 0, s, p);
  return (int)hipGetLastError();
}
