// Does an LDS-DMA issue (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction) hold up the
// ISSUING wave's MFMAs, and does it hold up its SIMD partner's?  (gfx950; verdict r4 item 1: the
// GEMM K-loop spends ~1960 cycles per K-tile per wave for 512 MFMA cycles.)
// One 512-thread block per CU (8 waves, 2 per SIMD), L2-resident 2 MiB source, per loop
// iteration and wave: D DMA pieces and/or M v_mfma_f32_16x16x32_bf16 on independent
// accumulators, no LDS reads.  Variants:
//   mfma   : every wave M MFMAs, no DMA                   (MFMA floor)
//   dma    : every wave D DMA pieces, no MFMA             (fill floor)
//   both   : every wave D DMA then M MFMAs                (same wave does both)
//   split  : waves 0-3 only DMA (2 D), waves 4-7 only MFMA (2 M)  (role split across SIMD partners)
//   +lds   : both, plus R ds_read_b128 per iteration whose data feed the NEXT iteration's MFMAs
//            (double-buffered operands, as a software-pipelined K-loop)
//   +bar   : +lds with one s_barrier per iteration (after an lgkmcnt(0)), as the GEMM's K-tile
//   +bar8  : +bar with the reads split 8 / 8 around the two halves of the MFMAs (k-step pipelining)
//   +salu  : +bar plus ~90 scalar ALU instructions and 6 taken/not-taken branches per iteration (the
//            real K-loop's per-K-tile bookkeeping: stage index mod NST, wait selection, cursors)
//   +stag  : +bar with waves 4-7 shifted by half an iteration (their barrier falls in the middle of
//            their MFMAs, so at every barrier release one wave per SIMD issues DMA + reads while
//            its partner issues MFMAs: MI355X_MICROARCH.md "Two waves per SIMD" item 9)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_dma_mfma.hip -o scripts/probe_dma_mfma.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define LDS_PTR(T) __attribute__((address_space(3))) T*
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long bytes) {
  const unsigned long long b = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  void* p = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
}

constexpr int D = 6, M = 32, R = 16, ITERS = 2048;
constexpr long SPAN = 2L << 20;

template <int MODE>
__global__ __launch_bounds__(512) void k(const char* __restrict__ src, float* out, float seed) {
  __shared__ __attribute__((aligned(16))) char lds[128 * 1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, SPAN);
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{seed, 0.f, 0.f, (float)i};
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(seed * (lane + i));
    b[i] = (__bf16)(seed - i);
  }
  const bool do_dma = MODE == 1 || MODE == 2 || (MODE == 3 && wave < 4) || MODE >= 4;
  const bool do_mfma = MODE == 0 || MODE == 2 || (MODE == 3 && wave >= 4) || MODE >= 4;
  // conflict-free 16-byte reads: lane-linear within each wave's own 16 KiB window
  const char* rbase = lds + (wave & 7) * 16384 + lane * 16;
  const int nd = MODE == 3 ? 2 * D : D, nm = MODE == 3 ? 2 * M : M;
  int off = (blockIdx.x * 65536) % (int)SPAN;
  for (int it = 0; it < ITERS; ++it) {
    if (do_dma) {
      for (int i = 0; i < nd; ++i) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_PTR(void))(lds + ((wave * 16 + i) & 127) * 1024), 16,
                                                 lane * 16, off, 0, 0);
        off += 1024;
        if (off >= SPAN) off = 0;
      }
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    }
    if (MODE >= 4) {
      // R reads per iteration; their data is sunk (kept live) right before the barrier point, so
      // the MFMAs (fixed operands) never wait on them -- what a k-step-pipelined loop achieves
      const bool late = MODE == 7 && wave >= 4;
      auto mf = [&](int n) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < n)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
      };
      if (late) mf(2);          // the second half of the previous iteration's MFMAs
      bf16x8 na[8], nb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) na[i] = *reinterpret_cast<const bf16x8*>(rbase + i * 1024);
      if (MODE == 6) mf(2);
#pragma unroll
      for (int i = 0; i < 8; ++i) nb[i] = *reinterpret_cast<const bf16x8*>(rbase + 8192 + i * 1024);
      mf(late ? 2 : (MODE == 6 ? 2 : 4));
      if (MODE >= 5) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(na[i]), "v"(nb[i]));
      if (MODE == 8) {
        // scalar bookkeeping: a chain of wave-uniform integer ops and data-dependent branches
        int sv = __builtin_amdgcn_readfirstlane(it);
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          asm volatile(
              "s_mul_hi_i32 s90, %0, 0x55555556\n s_lshr_b32 s91, s90, 31\n s_add_i32 s90, s90, s91\n"
              "s_mul_i32 s90, s90, 3\n s_sub_i32 s91, %0, s90\n s_mul_i32 s91, s91, 0xc000\n"
              "s_add_i32 s92, s91, %0\n s_or_b32 s92, s92, s91\n s_cmp_lt_i32 s92, 7\n"
              "s_cselect_b64 s[94:95], -1, 0\n s_and_b64 vcc, exec, s[94:95]\n s_cbranch_vccnz 1f\n"
              "s_add_i32 s92, s92, 1\n1:\n s_add_i32 %0, %0, s92\n s_lshr_b32 %0, %0, 1\n"
              : "+s"(sv) : : "s90", "s91", "s92", "s94", "s95", "vcc", "scc");
        }
        asm volatile("" ::"s"(sv));
      }
      if (MODE >= 5) __builtin_amdgcn_s_barrier();
    } else if (do_mfma) {
      for (int j = 0; j < nm; j += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5f) out[blockIdx.x * 512 + tid] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  char* src;
  float* out;
  hipMalloc(&src, SPAN);
  hipMemset(src, 1, SPAN);
  hipMalloc(&out, (long)cus * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"mfma", "dma", "both", "split", "+lds", "+bar", "+bar8", "+stag", "+salu"};
  for (int mode = 0; mode < 9; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 5) hipLaunchKernelGGL(k<5>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 6) hipLaunchKernelGGL(k<6>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 7) hipLaunchKernelGGL(k<7>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      if (mode == 8) hipLaunchKernelGGL(k<8>, dim3(cus), dim3(512), 0, 0, src, out, 0.001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    // per wave-pair (SIMD) per iteration: 2 waves x M MFMAs (16 cycles each at full rate)
    const double us = best * 1e3;
    const double cyc_per_iter = best * 1e-3 * 2.2e9 / ITERS;   // at an assumed 2.2 GHz
    const double mfma_floor = 2.0 * M * 16;
    const double dma_bytes = 8.0 * D * 1024 * ITERS * cus;
    printf("%-6s %8.1f us  %7.0f cyc/iter (@2.2GHz; MFMA floor %4.0f)  fill %6.1f GB/s/CU\n", names[mode], us,
           cyc_per_iter, mfma_floor, mode == 0 ? 0.0 : dma_bytes / (best * 1e-3) / 1e9 / cus);
  }
  return 0;
}
