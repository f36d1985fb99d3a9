// MFMA issue-rate probe for gfx950: how fast can v_mfma_f32_16x16x32_bf16 chains run per SIMD,
// alone and with LDS fragment reads interleaved the way the GEMM K-loops do?
//
//   hipcc -O3 --offload-arch=gfx950 scripts/mfma_rate.hip -o scripts/mfma_rate && ./scripts/mfma_rate
//
// Each wave keeps NACC independent 16x16 f32 accumulators and issues NACC MFMAs per iteration
// (optionally RD ds_read_b128 fragment reads per iteration, consumed as the next iteration's
// operands).  Grid: 256 CUs x BPC blocks of 4 waves (one wave per SIMD per block), so BPC is the
// number of waves per SIMD.  Prints TFLOPS (dense bf16 flops) per configuration.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int NACC, int RD>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[256 * 64];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 256 * 64; i += 256) lds[i] = (unsigned short)(i * 7 + 3);
  __syncthreads();
  f32x4 acc[NACC];
#pragma unroll
  for (int a = 0; a < NACC; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 ua = u32x4{0x3f803f80u + lane, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
  u32x4 ub = u32x4{0x3f803f80u, 0x3f803f80u + lane, 0x3f803f80u, 0x3f803f80u};
  bf16x8 fa = __builtin_bit_cast(bf16x8, ua), fb = __builtin_bit_cast(bf16x8, ub);
  const int wave = threadIdx.x >> 6;
  for (int it = 0; it < iters; ++it) {
    bf16x8 ra[RD > 0 ? RD : 1];
#pragma unroll
    for (int r = 0; r < RD; ++r)
      ra[r] = __builtin_bit_cast(bf16x8,
                                 *reinterpret_cast<const u32x4*>(lds + ((wave * 16 + r * 4 + it) & 255) * 64 + lane * 8 % 64));
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[a], 0, 0, 0);
    if constexpr (RD > 0) {
      fa = ra[0];
      if constexpr (RD > 1) fb = ra[1];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < NACC; ++a) s += acc[a][0] + acc[a][1] + acc[a][2] + acc[a][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NACC, int RD>
void run(int bpc, int cus, float* out) {
  const int iters = 4096;
  const int grid = cus * bpc;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((mfma_loop<NACC, RD>), dim3(grid), dim3(256), 0, 0, out, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((mfma_loop<NACC, RD>), dim3(grid), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)reps * grid * 4 /*waves*/ * iters * NACC * 16.0 * 16 * 32 * 2;
  const double tf = flops / (ms * 1e-3) / 1e12;
  // cycles per MFMA per SIMD at the measured clock is not known here: report the rate and the
  // implied ns per MFMA per SIMD
  const double mfma_per_simd = (double)reps * bpc * iters * NACC;
  printf("NACC %2d  LDS reads/iter %d  waves/SIMD %d : %8.1f TFLOPS  (%.2f ns per MFMA per SIMD)\n", NACC, RD, bpc,
         tf, ms * 1e6 / mfma_per_simd);
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  float* out;
  (void)hipMalloc(&out, sizeof(float) * 256 * 256 * 8);
  printf("CUs %d\n", cus);
  for (int bpc : {1, 2, 4}) {
    run<1, 0>(bpc, cus, out);
    run<4, 0>(bpc, cus, out);
    run<16, 0>(bpc, cus, out);
    run<16, 2>(bpc, cus, out);
    run<8, 2>(bpc, cus, out);
  }
  (void)hipFree(out);
  return 0;
}
