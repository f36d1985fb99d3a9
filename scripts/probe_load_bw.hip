// Per-CU load bandwidth probe (gfx950): LDS-DMA (buffer_load ... lds) vs global_load_dwordx4
// into VGPRs vs global_load + ds_write_b128, from an L2-resident and an HBM-sized source.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_load_bw.hip -o /tmp/probe_load_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
#define LDS_PTR(T) __attribute__((address_space(3))) T*

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long bytes) {
  const unsigned long long b = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes));
  void* p = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, nb, 0x00020000);
}

// each block streams `per_block` bytes starting at a block-dependent offset (wrapping in `span`)
// MODE 0: LDS-DMA 1 KiB per wave-instruction into a 4-deep 32 KiB ring, counted vmcnt
// MODE 1: global_load_dwordx4 into VGPRs (8 in flight per lane), xor-accumulated
// MODE 2: global_load_dwordx4 + ds_write_b128 into a ring (the register-staged GEMM path)
template <int MODE>
__global__ __launch_bounds__(256) void probe(const char* __restrict__ src, long span, long per_block, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 32768];  // 64 KiB: two blocks per CU fit
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long base = ((long)blockIdx.x * per_block) % span;
  unsigned acc = 0;
  if constexpr (MODE == 0) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, span);
    // one step = 32 KiB per block = 8 DMA instructions per wave
    const long steps = per_block / 32768;
    for (long st = 0; st < steps; ++st) {
      const int slot = st & 1;
      long off = (base + st * 32768) % span;
      if (off + 32768 > span) off = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int piece = wave * 8 + i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_PTR(void))(lds + slot * 32768 + piece * 1024), 16,
                                                 lane * 16, (int)(off + piece * 1024), 0, 0);
      }
      if (st >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // 3 steps in flight
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc = *reinterpret_cast<unsigned*>(lds + tid * 4);
  } else {
    const long steps = per_block / 32768;
    for (long st = 0; st < steps; ++st) {
      long off = (base + st * 32768) % span;
      if (off + 32768 > span) off = 0;
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const u32x4*>(src + off + (i * 256 + tid) * 16);
      if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc ^= v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
      } else {
        const int slot = st & 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<u32x4*>(lds + slot * 32768 + (i * 256 + tid) * 16) = v[i];
      }
    }
    if constexpr (MODE == 2) {
      __syncthreads();
      acc = *reinterpret_cast<unsigned*>(lds + tid * 4);
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x * 256 + tid] = acc;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const long big = 1L << 30;
  char* src;
  unsigned* out;
  hipMalloc(&src, big);
  hipMemset(src, 1, big);
  hipMalloc(&out, 64L << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (long span : {2L << 20, 32L << 20, big}) {
    for (int bpc : {1, 2}) {
      const int grid = cus * bpc;
      const long per_block = (8L << 20) / bpc;  // 8 MiB per CU
      for (int mode = 0; mode < 3; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
          hipEventRecord(e0);
          if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, src, span, per_block, out);
          if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, src, span, per_block, out);
          if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, src, span, per_block, out);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms = 0;
          hipEventElapsedTime(&ms, e0, e1);
          if (rep > 0 && ms < best) best = ms;
        }
        const double bytes = (double)grid * per_block;
        printf("span %5ld MiB  blocks/CU %d  %-18s %8.1f GB/s chip  %6.1f GB/s per CU  (%.3f ms)\n", span >> 20, bpc,
               mode == 0 ? "lds-dma" : mode == 1 ? "global->vgpr" : "global->vgpr->lds", bytes / best / 1e6,
               bytes / best / 1e6 / cus, best);
      }
    }
  }
  return 0;
}
