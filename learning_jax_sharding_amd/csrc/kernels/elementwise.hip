// Memory-bound kernels: casts (optionally transposing), reductions, softmax, fused Adam,
// Philox RNG.  All vectorised to 16 bytes per lane (CDNA Guideline 13); grid-stride loops
// capped at 2048 workgroups so one launch fills the 256 CUs without oversubscription.
#include "common.h"

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
__global__ void cast_transpose_f32_bf16(const float* __restrict__ in, bf16_t* __restrict__ out, int R, int C,
                                        long ldi, long ldo) {
  __shared__ float tile[64][65];
  int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 64 x 4
  for (int i = ty; i < 64; i += 4) {
    int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? in[(long)r * ldi + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) out[(long)c * ldo + r] = f2bf(tile[tx][i]);
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

}  // namespace

// ============================================================================ C ABI
LJS_API int ljs_cast_f32_bf16(const void* in, void* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16, dim3(grid_for(n, 256 * 8)), dim3(256), 0, s, (const float*)in, (bf16_t*)out, n);
  return (int)hipGetLastError();
}

LJS_API int ljs_cast_bf16_f32(const void* in, void* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32, dim3(grid_for(n, 256 * 8)), dim3(256), 0, s, (const bf16_t*)in, (float*)out, n);
  return (int)hipGetLastError();
}

LJS_API int ljs_cast_transpose_f32_bf16(const void* in, void* out, int R, int C, long ldi, long ldo, hipStream_t s) {
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(cast_transpose_f32_bf16, grid, dim3(256), 0, s, (const float*)in, (bf16_t*)out, R, C, ldi, ldo);
  return (int)hipGetLastError();
}

// out (f32 scalar) = sum(in); in is f32 (is_bf16=0) or bf16
LJS_API int ljs_sum_all(const void* in, int is_bf16, long n, void* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(float), s);
  int g = grid_for(n, 256 * 16);
  if (is_bf16)
    hipLaunchKernelGGL(sum_all_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)in, n, (float*)out);
  else
    hipLaunchKernelGGL(sum_all_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)in, n, (float*)out);
  return (int)hipGetLastError();
}

// out[C] f32 = column sums of in[R][C]; accumulate=1 adds into out
LJS_API int ljs_colsum(const void* in, int is_bf16, int R, int C, long ld, void* out, int accumulate, hipStream_t s) {
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
