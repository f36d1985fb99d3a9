// Fused mean-squared-error loss for a bf16 prediction against an f32 or bf16 target.
//
// A general (non-constant) training cotangent: loss = scale * sum((y - t)^2) over this shard,
// and, when a gradient is wanted, dY = bf16(2 * scale * (y - t)) written in the SAME pass - so
// the backward of the loss costs no kernel of its own and y / t are read once.  The scalar is
// reduced in-launch by the last-arriving workgroup (two-level ticket, no memset, no second
// kernel).  16-byte loads, 8 elements per lane per iteration, several iterations in flight.
#include "common.h"

namespace {

constexpr int kMseMaxBlocks = 1024;

template <bool kTgtBf16, bool kWantDy>
__global__ void __launch_bounds__(256) mse_kernel(const bf16_t* __restrict__ y, const void* __restrict__ tgt,
                                                  long n, float scale, bf16_t* __restrict__ dy,
                                                  float* __restrict__ partials, unsigned* __restrict__ ticket,
                                                  float* __restrict__ out) {
  const long nv = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  const float g2 = 2.f * scale;
  float s = 0.f;
  auto step = [&](long i) {
    const u32x4 yv = *reinterpret_cast<const u32x4*>(y + i * 8);
    float tv[8];
    if constexpr (kTgtBf16) {
      const u32x4 t = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(tgt) + i * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tv[2 * k] = __uint_as_float(t[k] << 16);
        tv[2 * k + 1] = __uint_as_float(t[k] & 0xffff0000u);
      }
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(tgt) + i * 8);
      const f32x4 b = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(tgt) + i * 8 + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tv[k] = a[k];
        tv[4 + k] = b[k];
      }
    }
    float d[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[2 * k] = __uint_as_float(yv[k] << 16) - tv[2 * k];
      d[2 * k + 1] = __uint_as_float(yv[k] & 0xffff0000u) - tv[2 * k + 1];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) s = fmaf(d[k], d[k], s);
    if constexpr (kWantDy) {
      u32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = pack_bf16x2(g2 * d[2 * k], g2 * d[2 * k + 1]);
      *reinterpret_cast<u32x4*>(dy + i * 8) = o;
    }
  };
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < nv; i += 4 * stride) {
    step(i);
    step(i + stride);
    step(i + 2 * stride);
    step(i + 3 * stride);
  }
  for (; i < nv; i += stride) step(i);
  if (blockIdx.x == 0) {
    for (long j = nv * 8 + threadIdx.x; j < n; j += blockDim.x) {
      const float t = kTgtBf16 ? bf2f(reinterpret_cast<const bf16_t*>(tgt)[j]) : reinterpret_cast<const float*>(tgt)[j];
      const float d = bf2f(y[j]) - t;
      s = fmaf(d, d, s);
      if constexpr (kWantDy) dy[j] = f2bf(g2 * d);
    }
  }
  s = warp_sum64(s);
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = s;
  __syncthreads();
  if (w != 0) return;
  if (lane == 0) sc1_store(partials + blockIdx.x, part[0] + part[1] + part[2] + part[3]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int last = 0;
  if (lane == 0) last = ticket_last_2lvl(ticket, blockIdx.x, gridDim.x);
  last = __shfl(last, 0, 64);
  if (!last) return;
  // the last arriver sums the partials with 4 independent loads in flight per lane
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  const int G = (int)gridDim.x;
  int k = lane;
  for (; k + 192 < G; k += 256) {
    v0 += sc1_load(partials + k);
    v1 += sc1_load(partials + k + 64);
    v2 += sc1_load(partials + k + 128);
    v3 += sc1_load(partials + k + 192);
  }
  for (; k < G; k += 64) v0 += sc1_load(partials + k);
  float v = warp_sum64((v0 + v1) + (v2 + v3));
  if (lane == 0) *out = v * scale;
}


// The same loss with its gradient AND the gradient's column sums (the bias gradient of the dense
// layer that produced y) in one pass over [R][C] rows: grid (C / 64 column blocks, row blocks),
// 256 threads = 8 column lanes (8 columns each) x 32 row lanes.  Column partials per row block go
// to a slab; the last-arriving row block of a column block sums its slab column (ticket per
// column block); the loss partials are summed by the overall last arriver (two-level ticket).
template <bool kTgtBf16>
__global__ void __launch_bounds__(256) mse_colsum_kernel(const bf16_t* __restrict__ y, const void* __restrict__ tgt,
                                                         int R, int C, int rows_per_block, float scale,
                                                         bf16_t* __restrict__ dy, float* __restrict__ col_part,
                                                         float* __restrict__ loss_part, unsigned* __restrict__ tickets,
                                                         float* __restrict__ colsum, float* __restrict__ out) {
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cl * 8;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(R, r0 + rows_per_block);
  const float g2 = 2.f * scale;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float s = 0.f;
  auto one = [&](long r, const u32x4& yv, const float (&tv)[8]) {
    float d[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[2 * k] = __uint_as_float(yv[k] << 16) - tv[2 * k];
      d[2 * k + 1] = __uint_as_float(yv[k] & 0xffff0000u) - tv[2 * k + 1];
    }
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s = fmaf(d[2 * k], d[2 * k], s);
      s = fmaf(d[2 * k + 1], d[2 * k + 1], s);
      o[k] = pack_bf16x2(g2 * d[2 * k], g2 * d[2 * k + 1]);
      // the bias gradient sums the bf16 values the GEMMs read
      acc[2 * k] += __uint_as_float(o[k] << 16);
      acc[2 * k + 1] += __uint_as_float(o[k] & 0xffff0000u);
    }
    *reinterpret_cast<u32x4*>(dy + r * C + c0) = o;
  };
  auto load_t = [&](long r, float (&tv)[8]) {
    if constexpr (kTgtBf16) {
      const u32x4 t = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(tgt) + r * C + c0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tv[2 * k] = __uint_as_float(t[k] << 16);
        tv[2 * k + 1] = __uint_as_float(t[k] & 0xffff0000u);
      }
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(tgt) + r * C + c0);
      const f32x4 b = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(tgt) + r * C + c0 + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tv[k] = a[k];
        tv[4 + k] = b[k];
      }
    }
  };
  if (c0 < C) {
    int r = r0 + rl;
    for (; r + 64 < r1; r += 96) {  // 3 rows in flight per thread
      u32x4 yv[3];
      float tv[3][8];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        yv[u] = *reinterpret_cast<const u32x4*>(y + (long)(r + 32 * u) * C + c0);
        load_t(r + 32 * u, tv[u]);
      }
#pragma unroll
      for (int u = 0; u < 3; ++u) one(r + 32 * u, yv[u], tv[u]);
    }
    for (; r < r1; r += 32) {
      float tv[8];
      load_t(r, tv);
      one(r, *reinterpret_cast<const u32x4*>(y + (long)r * C + c0), tv);
    }
  }
  __shared__ float red[32][65];
  __shared__ float lred[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rl][cl * 8 + k] = acc[k];
  s = warp_sum64(s);
  if ((threadIdx.x & 63) == 0) lred[threadIdx.x >> 6] = s;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nblk = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
  unsigned* col_tickets = tickets;                 // one per column block
  unsigned* loss_tickets = tickets + gridDim.x;    // two-level over all blocks
  __shared__ int last_col, last_all;
  __shared__ float fin[4][64];
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + lane;
    float cs = 0.f;
    for (int r = 0; r < 32; ++r) cs += red[r][lane];
    if (c < C) sc1_store(col_part + (long)blockIdx.y * C + c, cs);
    if (lane == 0) sc1_store(loss_part + bid, lred[0] + lred[1] + lred[2] + lred[3]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      last_col = ticket_last(col_tickets + blockIdx.x, gridDim.y);
      last_all = ticket_last_2lvl(loss_tickets, bid, nblk);
    }
  }
  __syncthreads();
  // the last row block of this column block sums its column partials: 4 waves x row slices,
  // 2 independent loads in flight per lane, then across the waves through LDS
  if (last_col) {
    const int c = blockIdx.x * 64 + lane;
    float t0 = 0.f, t1 = 0.f;
    if (c < C) {
      int yb = w;
      for (; yb + 4 < (int)gridDim.y; yb += 8) {
        t0 += sc1_load(col_part + (long)yb * C + c);
        t1 += sc1_load(col_part + (long)(yb + 4) * C + c);
      }
      for (; yb < (int)gridDim.y; yb += 4) t0 += sc1_load(col_part + (long)yb * C + c);
    }
    fin[w][lane] = t0 + t1;
    __syncthreads();
    if (w == 0 && c < C) colsum[c] = (fin[0][lane] + fin[1][lane]) + (fin[2][lane] + fin[3][lane]);
    __syncthreads();
  }
  if (last_all) {
    float v0 = 0.f, v1 = 0.f;
    int k = threadIdx.x;
    for (; k + 256 < nblk; k += 512) {
      v0 += sc1_load(loss_part + k);
      v1 += sc1_load(loss_part + k + 256);
    }
    for (; k < nblk; k += 256) v0 += sc1_load(loss_part + k);
    const float v = warp_sum64(v0 + v1);
    if (lane == 0) fin[w][0] = v;
    __syncthreads();
    if (threadIdx.x == 0) *out = ((fin[0][0] + fin[1][0]) + (fin[2][0] + fin[3][0])) * scale;
  }
}

}  // namespace

// y: bf16 [n]; tgt: f32 or bf16 [n] (16-byte aligned, contiguous); dy: bf16 [n] or null (no
// gradient pass); out: f32 scalar.  ws: kMseMaxBlocks floats of partials followed by 33 zeroed
// ticket words (re-armed by the kernel).
LJS_API int ljs_mse_loss(const void* y, const void* tgt, int tgt_bf16, long n, float scale, void* dy, void* out,
                         void* ws, hipStream_t s) {
  if ((((uintptr_t)y) | ((uintptr_t)tgt) | ((uintptr_t)dy)) & 15) return (int)hipErrorInvalidValue;
  float* partials = (float*)ws;
  unsigned* ticket = (unsigned*)((float*)ws + kMseMaxBlocks);
  long blocks = (n / 8 + 256 * 4 - 1) / (256 * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > kMseMaxBlocks) blocks = kMseMaxBlocks;
  const dim3 g((unsigned)blocks), b(256);
#define LJS_MSE(TB, WD)                                                                                        \
  hipLaunchKernelGGL((mse_kernel<TB, WD>), g, b, 0, s, (const bf16_t*)y, tgt, n, scale, (bf16_t*)dy, partials, \
                     ticket, (float*)out)
  if (tgt_bf16) {
    if (dy) LJS_MSE(true, true); else LJS_MSE(true, false);
  } else {
    if (dy) LJS_MSE(false, true); else LJS_MSE(false, false);
  }
#undef LJS_MSE
  return (int)hipGetLastError();
}

LJS_API int ljs_mse_ws_bytes() { return (kMseMaxBlocks + 33) * 4; }

// Fused loss + dY + dY's column sums over [R][C] (C % 64 == 0, 16-byte aligned rows).  ws: at
// least ljs_mse_colsum_ws_bytes(R, C) zeroed bytes (tickets re-armed by the kernel).
static void mse_colsum_geom(int R, int C, int* cb, int* gy, int* rpb) {
  *cb = C / 64;
  int want = 1024 / (*cb > 0 ? *cb : 1);         // ~1024 blocks over the whole array
  if (want < 1) want = 1;
  int r = (R + want - 1) / want;
  r = ((r + 95) / 96) * 96;                       // whole 3-row groups per row lane
  if (r < 96) r = 96;
  *rpb = r;
  *gy = (R + r - 1) / r;
}

LJS_API long ljs_mse_colsum_ws_bytes(int R, int C) {
  int cb, gy, rpb;
  mse_colsum_geom(R, C, &cb, &gy, &rpb);
  const long nblk = (long)cb * gy;
  return 4L * (cb + 1 + (nblk + 31) / 32 + 64) + 4L * ((long)gy * C + nblk + 64);
}

LJS_API int ljs_mse_colsum(const void* y, const void* tgt, int tgt_bf16, int R, int C, float scale, void* dy,
                           void* colsum, void* out, void* ws, hipStream_t s) {
  if (C % 64 || (((uintptr_t)y) | ((uintptr_t)tgt) | ((uintptr_t)dy)) & 15) return (int)hipErrorInvalidValue;
  int cb, gy, rpb;
  mse_colsum_geom(R, C, &cb, &gy, &rpb);
  const long nblk = (long)cb * gy;
  unsigned* tickets = (unsigned*)ws;
  const long nt = cb + 1 + (nblk + 31) / 32 + 64;
  float* col_part = (float*)ws + nt;
  float* loss_part = col_part + (long)gy * C;
  if (tgt_bf16)
    hipLaunchKernelGGL(mse_colsum_kernel<true>, dim3(cb, gy), dim3(256), 0, s, (const bf16_t*)y, tgt, R, C, rpb,
                       scale, (bf16_t*)dy, col_part, loss_part, tickets, (float*)colsum, (float*)out);
  else
    hipLaunchKernelGGL(mse_colsum_kernel<false>, dim3(cb, gy), dim3(256), 0, s, (const bf16_t*)y, tgt, R, C, rpb,
                       scale, (bf16_t*)dy, col_part, loss_part, tickets, (float*)colsum, (float*)out);
  return (int)hipGetLastError();
}
