// Direct peer-memory collectives for small messages: on an MI355X
// node every GPU pair has its own xGMI link, so a ONE-SHOT kernel that reads all k-1 peers'
// buffers at once uses all k-1 links in parallel and pays one synchronisation, where a ring
// pays 2(k-1) latency-bound steps over 2 links.  RCCL stays the bulk path.
//
// Buffers: every member owns one staging allocation in fine-grained UNCACHED device memory
// (hipExtMallocWithFlags(hipDeviceMallocUncached), exported by IPC handle to the other
// processes, or peer-mapped in single-process runs), so peer reads over xGMI never see a stale
// cache line.  Layout per member: [flags: 64 x u32 | counter | pad to 4 KiB][in: cap][res: cap].
//
// Barrier: member r stores the new sequence number into slot r of EVERY member's flag array
// (system-scope release stores over xGMI) and polls its own slots until every member has
// arrived.  The sequence number comes from a device-side counter so a HIP-graph replay of the
// same launch keeps advancing it.  A poll that exceeds the timeout sets *err and exits: a lost
// peer can never hang the GPU.
#include "common.h"

namespace {

constexpr int P2P_MAX = 8;
struct PeerPtrs { const char* p[P2P_MAX]; };
struct PeerFlags { unsigned* p[P2P_MAX]; };

__global__ __launch_bounds__(64) void p2p_barrier_kernel(PeerFlags peers, unsigned* my_flags, unsigned* ctr, int n,
                                                         int rank, long timeout_ticks, int* err) {
  __shared__ unsigned seq_s;
  const int t = threadIdx.x;
  if (t == 0) {
    unsigned s = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_store(ctr, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    seq_s = s;
  }
  __syncthreads();
  const unsigned seq = seq_s;
  if (t < n) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: prior writes reach memory
    __hip_atomic_store(peers.p[t] + rank, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const long t0 = (long)__builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(my_flags + t, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__device__ __forceinline__ u32x4 ld_sys16(const char* p) {
  // one 16-byte load of fine-grained peer memory, bypassing every non-coherent cache level
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// out[i] = sum over members r (in member order: bitwise identical on every member) of
// peer_r[src_off + i]; 16-byte vectors, f32 accumulation for bf16
template <bool BF16>
__global__ __launch_bounds__(256) void p2p_reduce_kernel(PeerPtrs peers, int n, long src_off_bytes, char* out,
                                                         long nvec) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const long off = src_off_bytes + v * 16;
    float acc[8];
    if constexpr (BF16) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = 0.f;
    }
    u32x4 x[P2P_MAX];
#pragma unroll
    for (int r = 0; r < P2P_MAX; ++r)
      if (r < n) x[r] = ld_sys16(peers.p[r] + off);
#pragma unroll
    for (int r = 0; r < P2P_MAX; ++r) {
      if (r < n) {
        if constexpr (BF16) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[2 * k] += __uint_as_float(x[r][k] << 16);
            acc[2 * k + 1] += __uint_as_float(x[r][k] & 0xffff0000u);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] += __uint_as_float(x[r][k]);
        }
      }
    }
    u32x4 o;
    if constexpr (BF16) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = pack_bf16x2(acc[2 * k], acc[2 * k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(acc[k]);
    }
    *reinterpret_cast<u32x4*>(out + v * 16) = o;
  }
}

// out[r * chunk + i] = peer_r[src_off + i]  (all-gather: src_off = 0; all-to-all: src_off =
// this member's chunk)
__global__ __launch_bounds__(256) void p2p_gather_kernel(PeerPtrs peers, int n, long src_off_bytes, char* out,
                                                         long chunk_vec) {
  const long total = chunk_vec * n;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int r = (int)(v / chunk_vec);
    const long i = v - (long)r * chunk_vec;
    const char* src = r == 0 ? peers.p[0] : r == 1 ? peers.p[1] : r == 2 ? peers.p[2] : r == 3 ? peers.p[3]
                    : r == 4 ? peers.p[4] : r == 5 ? peers.p[5] : r == 6 ? peers.p[6] : peers.p[7];
    *reinterpret_cast<u32x4*>(out + v * 16) = ld_sys16(src + src_off_bytes + i * 16);
  }
}

int grid_for(long nvec) {
  long g = (nvec + 255) / 256;
  return (int)(g < 1 ? 1 : g > 1024 ? 1024 : g);
}

PeerPtrs to_peers(const void* const* ptrs, int n) {
  PeerPtrs pp = {};
  for (int r = 0; r < n && r < P2P_MAX; ++r) pp.p[r] = static_cast<const char*>(ptrs[r]);
  return pp;
}

}  // namespace

// flags[r] = member r's flag array (64 u32 slots); my_flags / ctr / err are this member's.
LJS_API int ljs_p2p_barrier(void* const* flags, int n, int rank, void* my_flags, void* ctr, long timeout_ms, void* err,
                            hipStream_t s) {
  if (n < 1 || n > P2P_MAX || rank < 0 || rank >= n) return (int)hipErrorInvalidValue;
  PeerFlags pf = {};
  for (int r = 0; r < n; ++r) pf.p[r] = static_cast<unsigned*>(flags[r]);
  const long ticks = timeout_ms * 100000L;  // s_memrealtime runs at 100 MHz
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, s, pf, (unsigned*)my_flags, (unsigned*)ctr, n, rank,
                     ticks, (int*)err);
  return (int)hipGetLastError();
}

// dtype: 0 f32, 1 bf16.  Byte counts must be multiples of 16 and buffers 16-byte aligned.
LJS_API int ljs_p2p_reduce(const void* const* srcs, int n, long src_off_bytes, void* out, long nbytes, int dtype,
                           hipStream_t s) {
  if (n < 1 || n > P2P_MAX || nbytes % 16 || src_off_bytes % 16) return (int)hipErrorInvalidValue;
  const long nvec = nbytes / 16;
  if (nvec == 0) return 0;
  PeerPtrs pp = to_peers(srcs, n);
  if (dtype == 1)
    hipLaunchKernelGGL(p2p_reduce_kernel<true>, dim3(grid_for(nvec)), dim3(256), 0, s, pp, n, src_off_bytes,
                       (char*)out, nvec);
  else
    hipLaunchKernelGGL(p2p_reduce_kernel<false>, dim3(grid_for(nvec)), dim3(256), 0, s, pp, n, src_off_bytes,
                       (char*)out, nvec);
  return (int)hipGetLastError();
}

LJS_API int ljs_p2p_copy(void* dst, const void* src, long nbytes, hipStream_t s) {
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDevice, s);
}

LJS_API int ljs_p2p_gather(const void* const* srcs, int n, long src_off_bytes, void* out, long chunk_bytes,
                           hipStream_t s) {
  if (n < 1 || n > P2P_MAX || chunk_bytes % 16 || src_off_bytes % 16) return (int)hipErrorInvalidValue;
  const long cv = chunk_bytes / 16;
  if (cv == 0) return 0;
  hipLaunchKernelGGL(p2p_gather_kernel, dim3(grid_for(cv * n)), dim3(256), 0, s, to_peers(srcs, n), n, src_off_bytes,
                     (char*)out, cv);
  return (int)hipGetLastError();
}
