// LDS-DMA fill rate per CU vs bytes in flight (gfx950): does the L2 -> LDS stream of a GEMM's
// operand panels saturate at a per-CU rate, or is it latency-bound (Little's law) so that a deeper
// ring would raise it?  Every wave issues P 1-KiB buffer_load...lds pieces per step and keeps
// DEPTH steps in flight (counted vmcnt); NW waves per block, one block per CU.  Sources: a 2 MiB
// span (L2-resident, as the GEMMs' weight panels), 24 MiB (activations: L2 + Infinity Cache) and
// 1 GiB (HBM).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_fill.hip -o /tmp/probe_fill
#include <hip/hip_runtime.h>
#include <cstdio>

#define LDS_PTR(T) __attribute__((address_space(3))) T*

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long bytes) {
  const unsigned long long b = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes));
  void* p = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, nb, 0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int P = 4;  // pieces (1 KiB) per wave per step

template <int NW, int DEPTH>
__global__ __launch_bounds__(NW * 64) void fill(const char* __restrict__ src, long span, int steps, unsigned* out) {
  constexpr int SLOT = NW * P * 1024;
  // (nothing reads the ring: slots may be reused while pieces are in flight)
  constexpr int SLOTS = (DEPTH + 1) * SLOT <= 160 * 1024 ? DEPTH + 1 : (160 * 1024) / SLOT;
  __shared__ __attribute__((aligned(16))) char lds[SLOTS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, span);
  // blocks start at different offsets (like GEMM blocks on different panels)
  long off = ((long)blockIdx.x * 65536) % span;
  for (int st = 0; st < steps; ++st) {
    const int slot = st % SLOTS;
    if (off + SLOT > span) off = 0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int piece = wave * P + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_PTR(void))(lds + slot * SLOT + piece * 1024), 16, lane * 16,
                                               (int)(off + piece * 1024), 0, 0);
    }
    off += SLOT;
    if (st >= DEPTH) wait_vm<P * DEPTH>();
  }
  wait_vm<0>();
  __syncthreads();
  const unsigned v = *reinterpret_cast<unsigned*>(lds + tid * 4);
  if (v == 0x12345678u) out[blockIdx.x * 1024 + tid] = v;
}

template <int NW, int DEPTH>
void run(const char* src, long span, unsigned* out, int cus, hipEvent_t e0, hipEvent_t e1) {
  constexpr int SLOT = NW * P * 1024;
  const int steps = (int)((16L << 20) / SLOT);  // 16 MiB per CU
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((fill<NW, DEPTH>), dim3(cus), dim3(NW * 64), 0, 0, src, span, steps, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  const double bytes = (double)cus * steps * SLOT;
  printf("span %5ld MiB  waves %2d  depth %d  in-flight %4d KiB/CU  %7.1f GB/s chip  %6.1f GB/s/CU\n", span >> 20, NW,
         DEPTH, NW * P * DEPTH, bytes / best / 1e6, bytes / best / 1e6 / cus);
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
  for (long span : {2L << 20, 24L << 20, big}) {
    run<4, 1>(src, span, out, cus, e0, e1);
    run<4, 2>(src, span, out, cus, e0, e1);
    run<4, 4>(src, span, out, cus, e0, e1);
    run<4, 8>(src, span, out, cus, e0, e1);
    run<8, 1>(src, span, out, cus, e0, e1);
    run<8, 2>(src, span, out, cus, e0, e1);
    run<8, 3>(src, span, out, cus, e0, e1);
    run<8, 4>(src, span, out, cus, e0, e1);
    run<16, 1>(src, span, out, cus, e0, e1);
    run<16, 2>(src, span, out, cus, e0, e1);
  }
  return 0;
}
