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
  float v = 0.f;
  for (int k = lane; k < (int)gridDim.x; k += 64) v += sc1_load(partials + k);
  v = warp_sum64(v);
  if (lane == 0) *out = v * scale;
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
