// MX-fp8 (OCP e4m3 elements + e8m0 block scales, 32 elements per block along K) quantization
// and the block-scaled MFMA GEMM for gfx950 (v_mfma_scale_f32_16x16x128_f8f6f4: twice the
// bf16 MFMA rate per clock).
//
//   quant   : x[R][K] (f32 or bf16)          -> q[R][K] e4m3, s[R][K/32] e8m0   (blocks along rows)
//   quant_t : w[K][N] (f32 or bf16, row-major) -> q[N][K] e4m3, s[N][K/32] e8m0 (transposed)
//   gemm    : C[M][N] = sum_k (qa[m][k] 2^sa[m][k/32]) (qb[n][k] 2^sb[n][k/32])  (+bias)(relu)
//
// Scale rule: OCP MX v1.0's shared exponent floor(log2(amax)) - 8 (8 = emax of e4m3), raised by
// one when the block max would exceed 448; elements RNE-rounded to e4m3 after division by 2^exp.
//
// MFMA operand layout (measured with scripts/mfma_f8_layout.py): lane l (g = l >> 4) holds row
// l & 15, bytes 0-15 = k 16g..16g+15 and bytes 16-31 = k 64+16g..64+16g+15; the scale of
// 32-element k-block kb of row r is byte 0 of lane r + 16 kb's scale operand.
//
// GEMM structure: 128x128 output tile, 4 waves (2x2, 64x64 each), BK = 128 (one MFMA K step),
// buffer LDS-DMA staging of the fp8 tiles (128-byte rows, the same XOR-swizzled image as the
// bf16 kernels) AND of the per-row scale words, two-stage ring, counted vmcnt, one raw
// barrier per K-tile.  The MFMA operands are swapped (C^T blocks) so each lane ends with 4
// consecutive output columns: packed 16-byte row stores after a lane-pair exchange.
#include "common.h"

namespace {

constexpr int F8_BK = 128;  // K elements (bytes) per K-tile and per MFMA
typedef __attribute__((ext_vector_type(8))) int i32x8;

__device__ __forceinline__ float ldf(const void* p, long i, int is_bf16) {
  return is_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(p)[i]) : reinterpret_cast<const float*>(p)[i];
}

// (mx_exponent / pack4_e4m3: common.h, shared with the optimizer's MX weight shadows)

// one thread per 32-element block of a row.  xb (f32 input only, may be null): the same rows
// rounded to bf16, [R][K] contiguous -- the MX layer's backward operand, written from the values
// already in registers instead of by a second pass over x (verdict r5 item 5: no standalone
// cast_f32_bf16 in the MX-fp8 layer)
__global__ void quant_mx_rows_kernel(const void* __restrict__ in, int is_bf16, long ld, int R, int K,
                                     unsigned char* __restrict__ q, unsigned char* __restrict__ s,
                                     bf16_t* __restrict__ xb) {
  const long nb = (long)R * (K / 32);
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb) return;
  const int r = (int)(t / (K / 32)), kb = (int)(t % (K / 32));
  const long base = (long)r * ld + (long)kb * 32;
  float v[32];
  if (is_bf16) {
    const u32x4* p = reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(in) + base);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      u32x4 w = p[c];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[8 * c + 2 * k] = __uint_as_float(w[k] << 16);
        v[8 * c + 2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
      }
    }
  } else {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(in) + base);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      f32x4 w = p[c];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 * c + k] = w[k];
    }
    if (xb) {
      u32x4* bo = reinterpret_cast<u32x4*>(xb + (long)r * K + (long)kb * 32);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        bo[c] = u32x4{pack_bf16x2(v[8 * c], v[8 * c + 1]), pack_bf16x2(v[8 * c + 2], v[8 * c + 3]),
                      pack_bf16x2(v[8 * c + 4], v[8 * c + 5]), pack_bf16x2(v[8 * c + 6], v[8 * c + 7])};
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(v[i]));
  const int x = mx_exponent(amax);
  const float inv = ldexpf(1.f, -x);
  u32x4 o[2];
#pragma unroll
  for (int c = 0; c < 8; ++c)
    o[c >> 2][c & 3] = pack4_e4m3(v[4 * c] * inv, v[4 * c + 1] * inv, v[4 * c + 2] * inv, v[4 * c + 3] * inv);
  u32x4* qo = reinterpret_cast<u32x4*>(q + (long)r * K + (long)kb * 32);
  qo[0] = o[0];
  qo[1] = o[1];
  s[t] = (unsigned char)(x + 127);
}

// w[K][N] row-major -> q[N][K], s[N][K/32]: thread (n, kb); consecutive threads take
// consecutive n so every k-row read is coalesced
__global__ void quant_mx_cols_kernel(const void* __restrict__ in, int is_bf16, long ld, int K, int N,
                                     unsigned char* __restrict__ q, unsigned char* __restrict__ s) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int kb = blockIdx.y;
  if (n >= N) return;
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    v[i] = ldf(in, (long)(kb * 32 + i) * ld + n, is_bf16);
    amax = fmaxf(amax, fabsf(v[i]));
  }
  const int x = mx_exponent(amax);
  const float inv = ldexpf(1.f, -x);
  u32x4 o[2];
#pragma unroll
  for (int c = 0; c < 8; ++c)
    o[c >> 2][c & 3] = pack4_e4m3(v[4 * c] * inv, v[4 * c + 1] * inv, v[4 * c + 2] * inv, v[4 * c + 3] * inv);
  u32x4* qo = reinterpret_cast<u32x4*>(q + (long)n * K + (long)kb * 32);
  qo[0] = o[0];
  qo[1] = o[1];
  s[(long)n * (K / 32) + kb] = (unsigned char)(x + 127);
}

// bf16 x[K][N] -> q[N][K], s[N][K/32] through an LDS tile of 128 (K) x 64 (N): rows are read
// coalesced (128 B per row), and the 4 blocks of a column go to 4 consecutive lanes, so every
// wave writes 16 rows of q as 128-byte runs (the one-thread-per-block kernel above wrote 32-byte
// pieces of 64 different rows per wave-instruction: ~1 TB/s on a [16384][640] input)
// (qr / sr non-null: the same pass also writes the row-blocked quantization qr[K][N], sr[K][N/32]
// -- one read of x for both MX operands it feeds.  F32: x is f32; it is rounded to bf16 on load,
// the bf16 copy written to xb[K][N] (the block's residual operand) and quantized from those bf16
// values -- bit-identical to a cast pass followed by the bf16 kernel, without the second pass)
template <bool F32>
__global__ __launch_bounds__(256) void quant_mx_cols_tiled_kernel(const void* __restrict__ in, long ld, int K, int N,
                                                                  unsigned char* __restrict__ q,
                                                                  unsigned char* __restrict__ s,
                                                                  unsigned char* __restrict__ qr,
                                                                  unsigned char* __restrict__ sr,
                                                                  bf16_t* __restrict__ xb) {
  __shared__ __attribute__((aligned(16))) unsigned char tile[128 * 128];  // [k][n] bf16, 16 B chunk ^ (k >> 5)
  const int tid = threadIdx.x;
  const int n0 = blockIdx.x * 64, k0 = blockIdx.y * 128;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = tid + 256 * j, r = c >> 3, ch = c & 7;
    u32x4 v;
    if constexpr (F32) {
      const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(in) + (long)(k0 + r) * ld + n0 + ch * 8);
      const f32x4 a = p[0], b = p[1];
      v = u32x4{pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(b[0], b[1]), pack_bf16x2(b[2], b[3])};
      *reinterpret_cast<u32x4*>(xb + (long)(k0 + r) * N + n0 + ch * 8) = v;
    } else {
      v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(in) + (long)(k0 + r) * ld + n0 + ch * 8);
    }
    *reinterpret_cast<u32x4*>(tile + r * 128 + ((ch ^ ((r >> 5) & 3)) << 4)) = v;
  }
  __syncthreads();
  const int n = tid >> 2, kb = tid & 3;
  // the column's 32 bf16 re-paired along k, amax as an integer max of the magnitude bits, then
  // the gfx950 scaled conversions (cvt4_e4m3_bf16; bit-identical to the multiply + pack4 path)
  unsigned pr[16];
  unsigned mx = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = kb * 32 + 2 * i;
    const unsigned lo =
        *reinterpret_cast<const unsigned short*>(tile + r * 128 + (((n >> 3) ^ kb) << 4) + ((n & 7) << 1));
    const unsigned hi =
        *reinterpret_cast<const unsigned short*>(tile + (r + 1) * 128 + (((n >> 3) ^ kb) << 4) + ((n & 7) << 1));
    pr[i] = lo | (hi << 16);
    mx = max(mx, max(lo & 0x7fffu, hi & 0x7fffu));
  }
  const int x = mx_exponent(__uint_as_float(mx << 16));
  const float sc = mx_scale_pow2(x);
  u32x4 o[2];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c >> 2][c & 3] = cvt4_e4m3_bf16(pr[2 * c], pr[2 * c + 1], sc);
  u32x4* qo = reinterpret_cast<u32x4*>(q + (long)(n0 + n) * K + k0 + kb * 32);
  qo[0] = o[0];
  qo[1] = o[1];
  s[(long)(n0 + n) * (K / 32) + k0 / 32 + kb] = (unsigned char)(x + 127);
  if (qr) {
    // row blocks: thread (tile row r, 32-column half hb) -- 4 x 16 B LDS chunks
    const int r = tid >> 1, hb = tid & 1;
    u32x4 raw[4];
    unsigned mr = 0u;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int ch = hb * 4 + c4;
      raw[c4] = *reinterpret_cast<const u32x4*>(tile + r * 128 + ((ch ^ ((r >> 5) & 3)) << 4));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned a = raw[c4][e] & 0x7fff7fffu;
        mr = max(mr, max(a & 0xffffu, a >> 16));
      }
    }
    const int xr = mx_exponent(__uint_as_float(mr << 16));
    const float scr = mx_scale_pow2(xr);
    u32x4 orr[2];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      orr[c >> 2][c & 3] = cvt4_e4m3_bf16(raw[c >> 1][2 * (c & 1)], raw[c >> 1][2 * (c & 1) + 1], scr);
    u32x4* qd = reinterpret_cast<u32x4*>(qr + (long)(k0 + r) * N + n0 + hb * 32);
    qd[0] = orr[0];
    qd[1] = orr[1];
    sr[(long)(k0 + r) * (N / 32) + n0 / 32 + hb] = (unsigned char)(xr + 127);
  }
}

// x[K][N] (bf16, or f32 with xb != null: xb[K][N] receives x rounded to bf16) -> BOTH its
// row-blocked (qr [K][N]) and transposed column-blocked (q [N][K]) MX quantizations in one pass;
// K % 128, N % 64
LJS_API int ljs_quant_mx_both(const void* in, long ld, int K, int N, void* q, void* s, void* qr, void* sr, void* xb,
                              hipStream_t stream) {
  if (K % 128 || N % 64 || ld % 8 || ((uintptr_t)in & 15) || ((uintptr_t)q & 15) || ((uintptr_t)qr & 15) ||
      ((uintptr_t)xb & 15))
    return (int)hipErrorInvalidValue;
  if (xb)
    hipLaunchKernelGGL(quant_mx_cols_tiled_kernel<true>, dim3(N / 64, K / 128), dim3(256), 0, stream, in, ld, K, N,
                       (unsigned char*)q, (unsigned char*)s, (unsigned char*)qr, (unsigned char*)sr, (bf16_t*)xb);
  else
    hipLaunchKernelGGL(quant_mx_cols_tiled_kernel<false>, dim3(N / 64, K / 128), dim3(256), 0, stream, in, ld, K, N,
                       (unsigned char*)q, (unsigned char*)s, (unsigned char*)qr, (unsigned char*)sr, nullptr);
  return (int)hipGetLastError();
}

// one scalar cotangent broadcast as TWO rows (lengths C1, C2): bf16 row 1 and the MX bytes of
// both (the dY rows of y.sum() that the FF block's dA GEMM and dW_out GEMM read), one launch
__global__ void bcast_scalar_mx2_kernel(const void* __restrict__ g, int g_bf16, int C1, bf16_t* __restrict__ row,
                                        unsigned char* __restrict__ q1, unsigned char* __restrict__ s1, int C2,
                                        unsigned char* __restrict__ q2, unsigned char* __restrict__ s2) {
  const int c4 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  const float v = bf2f(f2bf(g_bf16 ? bf2f(*reinterpret_cast<const bf16_t*>(g)) : *reinterpret_cast<const float*>(g)));
  const int x = mx_exponent(fabsf(v));
  const float sv = v * ldexpf(1.f, -x);
  const unsigned qq = pack4_e4m3(sv, sv, sv, sv);
  if (c4 < C1) {
    *reinterpret_cast<u32x2*>(row + c4) = u32x2{pack_bf16x2(v, v), pack_bf16x2(v, v)};
    *reinterpret_cast<unsigned*>(q1 + c4) = qq;
    if ((c4 & 31) == 0) s1[c4 / 32] = (unsigned char)(x + 127);
  }
  if (c4 < C2) {
    *reinterpret_cast<unsigned*>(q2 + c4) = qq;
    if ((c4 & 31) == 0) s2[c4 / 32] = (unsigned char)(x + 127);
  }
}

LJS_API int ljs_bcast_scalar_mx2(const void* g, int g_bf16, int C1, void* row, void* q1, void* s1, int C2, void* q2,
                                 void* s2, hipStream_t stream) {
  if (C1 % 32 || C2 % 32) return (int)hipErrorInvalidValue;
  const int c = C1 > C2 ? C1 : C2;
  hipLaunchKernelGGL(bcast_scalar_mx2_kernel, dim3((c / 4 + 255) / 256), dim3(256), 0, stream, g, g_bf16, C1,
                     (bf16_t*)row, (unsigned char*)q1, (unsigned char*)s1, C2, (unsigned char*)q2, (unsigned char*)s2);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------- GEMM
struct F8Args {
  const unsigned char *A, *B, *SA, *SB;  // A[M][K], B[N][K] e4m3; SA[M][K/32], SB[N][K/32] e8m0
  void* C;
  const void* bias;
  long ldc;
  int M, N, K;
  int flags;  // 1 relu, 2 bias, 4 bias f32, 32 f32 output, 64 residual add, 128 ReLU mask (R > 0),
              // 256 quantized output copy (QC / SC), 512 transposed quantized copy (QT / ST),
              // 1024 R is e4m3 bytes (mask mode: keep where the e4m3 value is > 0)
  const bf16_t* R;      // epilogue operand [M][N] bf16 (or e4m3), row stride ldr elements (0: one row)
  long ldr;
  unsigned char* QC;    // MX-fp8 copy of the (bf16-rounded) output: QC[M][N] e4m3, SC[M][N/32] e8m0
  unsigned char* SC;
  unsigned char* QT;    // TRANSPOSED MX-fp8 copy: QT[N][M] (row stride ldqt), blocks of 32 along M,
  unsigned char* ST;    //   ST[N][M/32] -- the output as the K-major operand of a GEMM over M
  long ldqt;
  int lda, ldsa;        // A / SA row strides in bytes (K, K / 32; both 0: one broadcast row)
  int ldb, ldsb;        // B / SB row strides in bytes (K, K / 32; both 0: one broadcast row)
  int kps, nsplit;      // split-K: K-tiles per split, splits (split s -> f32 slab C + s * sC)
  long sC;
  float* csum;          // flags & 2048 (8-wave kernel, bf16 output): per-row-tile column sums of the
                        // bf16 output, csum[tile row][N] (summed over tile rows by the caller)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t f8_rsrc(const void* base, long bytes) {
  const unsigned long long b = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, nb, 0x00020000);
}

// 16-byte chunk c of a 128-byte LDS row, XOR-swizzled (conflict-free row reads)
__device__ __forceinline__ int f8_swz(int row, int c) { return c ^ ((row >> 1) & 7); }

// device-only wrappers of the gfx950 builtins (called from a kernel TEMPLATE, whose body the host
// pass also instantiates)
__device__ __forceinline__ void f8_dma(__amdgpu_buffer_rsrc_t rs, void* lds, int bytes, int voff, int soff) {
  if (bytes == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_PTR(void))lds, 16, voff, soff, 0, 0);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_PTR(void))lds, 4, voff, soff, 0, 0);
}
__device__ __forceinline__ f32x4 f8_mfma(const i32x8& a, const i32x8& b, const f32x4& c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// BM x 128 output tile, BM / 64 x 2 waves of 64 x 64 (BM = 128: 4 waves; 256: 8 waves, two per
// SIMD), BK = 128 (one MFMA K step per K-tile), an NST-deep ring of LDS-DMA stages (A and B
// tiles + the per-row scale words), counted vmcnt, one raw barrier per K-tile.
// FIX: the epilogue's flags as compile-time constants for the FF block's two epilogue-heavy
// GEMMs (1: up projection = ReLU + both MX copies, no bf16 output; 2: dA = e4m3 ReLU mask +
// both MX copies, no bf16 output; 3: plain f32 output, the weight gradients' split-K slabs); 0 reads
// p.flags at run time
template <int FIX>
__device__ __forceinline__ int f8_flags(const F8Args& p) {
  return FIX == 1 ? (1 | 256 | 512) : FIX == 2 ? (128 | 1024 | 256 | 512) : FIX == 3 ? 32 : p.flags;
}

template <int BM, int NST, int FIX = 0>
__global__ __launch_bounds__(BM * 2) void gemm_mx_fp8_kernel(F8Args p) {
  constexpr int NW = BM / 32;                      // waves (BM / 64 rows x 2 cols)
  constexpr int A_TILE = BM * F8_BK, B_TILE = 128 * F8_BK;
  constexpr int STAGE = A_TILE + B_TILE + BM * 4 + 128 * 4;
  constexpr int PA = BM / 8 / NW, PB = 16 / NW;    // 1 KiB data pieces per wave (A, B)
  constexpr int L = PA + PB + 1;                   // DMA instructions per wave per K-tile (+1 scale)
  static_assert(PA >= 1 && PB >= 1 && L * (NST - 1) <= 63, "piece split");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntn = (p.N + 127) / 128;
  const int ntiles = ((p.M + BM - 1) / BM) * ntn;
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = item % ntiles, split = item / ntiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * 128;
  if (m0 >= p.M) return;
  const int KB = p.K / 32;  // scale bytes per row
  // this split's K-tiles [kt0, kt0 + nk)
  const int kt0 = split * p.kps;
  const int nk = min(p.K / F8_BK - kt0, p.kps);

  const __amdgpu_buffer_rsrc_t ra = f8_rsrc(p.A, (long)(p.M - 1) * p.lda + p.K);
  const __amdgpu_buffer_rsrc_t rb = f8_rsrc(p.B, (long)(p.N - 1) * p.ldb + p.K);
  const __amdgpu_buffer_rsrc_t rsa = f8_rsrc(p.SA, (long)(p.M - 1) * p.ldsa + KB);
  const __amdgpu_buffer_rsrc_t rsb = f8_rsrc(p.SB, (long)(p.N - 1) * p.ldsb + KB);

  int voa[PA], vob[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int q = wave + NW * i;
    const int row = 8 * q + (lane >> 3), slot = lane & 7;
    voa[i] = (m0 + row) * p.lda + 16 * f8_swz(row, slot);
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int q = wave + NW * i;
    const int row = 8 * q + (lane >> 3), slot = lane & 7;
    vob[i] = (n0 + row) * p.ldb + 16 * f8_swz(row, slot);
  }
  // scale words (4 B per lane = one row's 4 scale bytes of a K-tile, 64 rows per instruction):
  // the first BM / 64 waves load A's, the next two B's, any further waves repeat B's (same
  // bytes to the same place) so every wave issues exactly one and vmcnt counts stay uniform
  const int sw = wave < BM / 64 ? wave : (BM / 64 + ((wave - BM / 64) & 1));
  const bool s_is_a = sw < BM / 64;
  const int s_row = 64 * (s_is_a ? sw : sw - BM / 64) + lane;
  const int vos = s_is_a ? (m0 + s_row) * p.ldsa : (n0 + s_row) * p.ldsb;
  const __amdgpu_buffer_rsrc_t rs = s_is_a ? rsa : rsb;
  const int s_dst = s_is_a ? 64 * 4 * sw : BM * 4 + 64 * 4 * (sw - BM / 64);

  // (a macro, not a lambda: a lambda in a kernel template is also instantiated for the host,
  // where the LDS-DMA builtin does not exist)
#define F8_ISSUE(KT, ST)                                                                           \
  do {                                                                                             \
    unsigned char* base_ = smem + (ST) * STAGE;                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < PA; ++i_)                                              \
        f8_dma(ra, base_ + (wave + NW * i_) * 1024, 16, voa[i_], (kt0 + (KT)) * F8_BK);            \
    _Pragma("unroll") for (int i_ = 0; i_ < PB; ++i_)                                              \
        f8_dma(rb, base_ + A_TILE + (wave + NW * i_) * 1024, 16, vob[i_], (kt0 + (KT)) * F8_BK);   \
    f8_dma(rs, base_ + A_TILE + B_TILE + s_dst, 4, vos, (kt0 + (KT)) * 4);                         \
  } while (0)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) F8_ISSUE(s, s);
  const int g = lane >> 4, r16 = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    // K-tile kt landed (this wave's pieces); the younger stages may stay in flight
    if constexpr (NST >= 3) {
      if (kt + NST - 2 >= nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned char* As_ = smem + (kt % NST) * STAGE;
    const unsigned char* Bs_ = As_ + A_TILE;
    const unsigned* Sa = reinterpret_cast<const unsigned*>(As_ + A_TILE + B_TILE);
    const unsigned* Sb = reinterpret_cast<const unsigned*>(As_ + A_TILE + B_TILE + BM * 4);
    i32x8 af[4], bfr[4];
    int sa[4], sb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + 16 * i + r16;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(As_ + row * 128 + 16 * f8_swz(row, g));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(As_ + row * 128 + 16 * f8_swz(row, g + 4));
      af[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      sa[i] = (int)((Sa[row] >> (8 * g)) & 0xff);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wc * 64 + 16 * j + r16;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Bs_ + row * 128 + 16 * f8_swz(row, g));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Bs_ + row * 128 + 16 * f8_swz(row, g + 4));
      bfr[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      sb[j] = (int)((Sb[row] >> (8 * g)) & 0xff);
    }
    // next stage's DMA after this K-tile's fragment reads: its issue time overlaps their LDS
    // latency and the MFMAs (as in the bf16 LDS-DMA GEMM)
    if (kt + NST - 1 < nk) F8_ISSUE(kt + NST - 1, (kt + NST - 1) % NST);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)  // C^T block: B rows as the MFMA A operand
        acc[i][j] = f8_mfma(bfr[j], af[i], acc[i][j], sb[j], sa[i]);
  }

  // epilogue: lane holds C[row 16 i + r16][cols 16 j + 4 g .. +3]; lane pairs (g, g^1) trade
  // halves -> 8 consecutive columns per lane -> one 16-byte (bf16) / 2 x 16-byte (f32) store.
  // A 32-column MX block of a row sits in the 4 lanes r16, r16 + 16, + 32, + 48 (g = 0..3).
  const int flags = f8_flags<FIX>(p);
  const bool relu = flags & 1, has_bias = flags & 2, bias_f32 = flags & 4, out_f32 = flags & 32;
  const bool res_add = flags & 64, res_mask = flags & 128, qout = flags & 256;
  const bool qtout = flags & 512, r_fp8 = flags & 1024;
  void* const Cp = (FIX == 1 || FIX == 2) ? nullptr : p.C;   // (those fixed epilogues write no bf16 output)
  const bool even = (g & 1) == 0;
  // the epilogue operand's 8 chunks per lane are all requested before the first is used (one
  // exposed latency per item instead of one per 16-row block); rows / columns outside the
  // output read 0 through the buffer range check
  // bf16 outputs (and their MX copy) are staged through LDS (the idle ring) and leave as whole
  // tile rows -- 256 B of bf16 / 128 B of e4m3 per row, 16 B per lane -- instead of 64 B / 32 B
  // row pieces per 16-lane group and single scale bytes
  const bool staged = !out_f32;
  unsigned char* const Cs = smem;                 // [BM][256 B], 16 B chunks ^ (row & 15)
  unsigned char* const Qs = smem + BM * 256;      // [BM][128 B], 16 B chunks ^ (row & 7)
  unsigned char* const Ss = smem + BM * 384;      // [BM][4] scale bytes
  static_assert(BM * 388 <= NST * STAGE, "staging fits the ring");
  if (staged) __syncthreads();  // every wave's last fragment reads are done with the ring
  u32x4 rv[2][4];
  if (res_add || res_mask) {
    const int esz = r_fp8 ? 1 : 2;
    const __amdgpu_buffer_rsrc_t rr = f8_rsrc(p.R, esz * ((long)(p.M - 1) * p.ldr + p.N));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int col = n0 + wc * 64 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * 64 + 16 * i + r16;
        const bool ok = row < p.M && col < p.N;
        const int off = ok ? (int)(((long)row * p.ldr + col) * esz) : 0x7ffffff0;
        if (r_fp8) {  // 8 e4m3 bytes
          const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(rr, off, 0, 0);
          rv[q][i] = u32x4{b[0], b[1], 0u, 0u};
        } else {
          rv[q][i] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int col = n0 + wc * 64 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
    float bv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bv[e] = 0.f;
      if (has_bias && col + e < p.N) bv[e] = bias_f32 ? reinterpret_cast<const float*>(p.bias)[col + e]
                                                      : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[col + e]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 a0 = acc[i][2 * q], a1 = acc[i][2 * q + 1];
      float v[8];
      pair_rows16(a0, a1, even, v);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += bv[e];
        v[4 + e] += bv[4 + e];
        if (relu) {
          v[e] = fmaxf(v[e], 0.f);
          v[4 + e] = fmaxf(v[4 + e], 0.f);
        }
      }
      const int row = m0 + wr * 64 + 16 * i + r16;
      const bool ok = row < p.M && col < p.N;  // N % 8 == 0 (launcher)
      if (res_mask && r_fp8) {
        // the mask of a ReLU whose output is kept only as e4m3: keep where that value is > 0
        // (sign clear, not zero)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const unsigned byte = (rv[q][i][e >> 2] >> (8 * (e & 3))) & 0xffu;
          v[e] = (byte & 0x80u) == 0u && byte != 0u ? v[e] : 0.f;
        }
      } else if (res_add || res_mask) {
        const u32x4 rw = rv[q][i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float r0 = __uint_as_float(rw[e] << 16), r1 = __uint_as_float(rw[e] & 0xffff0000u);
          if (res_add) {  // bf16(bf16(y) + R): the unfused bf16 add
            v[2 * e] = bf2f(f2bf(v[2 * e])) + r0;
            v[2 * e + 1] = bf2f(f2bf(v[2 * e + 1])) + r1;
          } else {
            v[2 * e] = r0 > 0.f ? v[2 * e] : 0.f;
            v[2 * e + 1] = r1 > 0.f ? v[2 * e + 1] : 0.f;
          }
        }
      }
      if (qout && staged) {
        // MX-fp8 copy of the bf16-rounded outputs from their packed bf16 pairs: block amax over
        // the 4 lanes of the block (rounding is monotonic: max of the rounded values = the
        // rounded max), then the scaled conversions; lane g = 0 stores the e8m0 scale
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
        amax = bf2f(f2bf(amax));
        amax = row4_max(amax);   // lanes l, l ^ 16, l ^ 32, l ^ 48: two lane swaps, no ds_bpermute
        const int x = mx_exponent(amax);
        const float sc = mx_scale_pow2(x);
        u32x4 pb;
#pragma unroll
        for (int e = 0; e < 4; ++e) pb[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
        const u32x2 qq = u32x2{cvt4_e4m3_bf16(pb[0], pb[1], sc), cvt4_e4m3_bf16(pb[2], pb[3], sc)};
        const int lr = row - m0, lc = col - n0;
        *reinterpret_cast<u32x2*>(Qs + lr * 128 + (((lc >> 4) ^ (lr & 7)) << 4) + (((lc >> 3) & 1) << 3)) = qq;
        if (g == 0) Ss[lr * 4 + (lc >> 5)] = (unsigned char)(x + 127);
        if (Cp || qtout) *reinterpret_cast<u32x4*>(Cs + lr * 256 + (((lc >> 3) ^ (lr & 15)) << 4)) = pb;
        continue;
      }
      if (qout) {
        // MX-fp8 copy of the bf16-rounded outputs: block amax over the 4 lanes of the block,
        // then each lane stores its 8 e4m3 bytes and lane g = 0 the block's e8m0 scale
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = bf2f(f2bf(v[e]));
          amax = fmaxf(amax, fabsf(v[e]));
        }
        amax = row4_max(amax);   // lanes l, l ^ 16, l ^ 32, l ^ 48: two lane swaps, no ds_bpermute
        const int x = mx_exponent(amax);
        const float inv = ldexpf(1.f, -x);
        const u32x2 qq = u32x2{pack4_e4m3(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv),
                               pack4_e4m3(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv)};
        if (staged) {
          const int lr = row - m0, lc = col - n0;
          *reinterpret_cast<u32x2*>(Qs + lr * 128 + (((lc >> 4) ^ (lr & 7)) << 4) + (((lc >> 3) & 1) << 3)) = qq;
          if (g == 0) Ss[lr * 4 + (lc >> 5)] = (unsigned char)(x + 127);
        } else if (ok) {
          *reinterpret_cast<u32x2*>(p.QC + (long)row * p.N + col) = qq;
          if (g == 0) p.SC[(long)row * (p.N / 32) + col / 32] = (unsigned char)(x + 127);
        }
      }
      if (staged) {
        if (Cp || qtout) {  // (the transposed MX copy is formed from this bf16 image)
          u32x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
          const int lr = row - m0, lc = col - n0;
          *reinterpret_cast<u32x4*>(Cs + lr * 256 + (((lc >> 3) ^ (lr & 15)) << 4)) = pk;
        }
        continue;
      }
      if (!ok) continue;
      if (out_f32) {
        float* C = reinterpret_cast<float*>(Cp) + split * p.sC + (long)row * p.ldc + col;
        *reinterpret_cast<f32x4*>(C) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(C + 4) = f32x4{v[4], v[5], v[6], v[7]};
      } else if (Cp) {
        u32x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
        *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(Cp) + (long)row * p.ldc + col) = pk;
      }
    }
  }
  if (!staged) return;
  __syncthreads();
  constexpr int NT = BM * 2;  // threads
  if (Cp) {
#pragma unroll
    for (int r = 0; r < BM * 16 / NT; ++r) {
      const int c = tid + NT * r, lr = c >> 4, ch = c & 15;
      const int grow = m0 + lr, gcol = n0 + ch * 8;
      const u32x4 val = *reinterpret_cast<const u32x4*>(Cs + lr * 256 + ((ch ^ (lr & 15)) << 4));
      if (grow < p.M && gcol < p.N)
        *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(Cp) + (long)grow * p.ldc + gcol) = val;
    }
  }
  if (qout) {
#pragma unroll
    for (int r = 0; r < BM * 8 / NT; ++r) {
      const int c = tid + NT * r, lr = c >> 3, ch = c & 7;
      const int grow = m0 + lr, gcol = n0 + ch * 16;
      const u32x4 val = *reinterpret_cast<const u32x4*>(Qs + lr * 128 + ((ch ^ (lr & 7)) << 4));
      if (grow < p.M && gcol < p.N) *reinterpret_cast<u32x4*>(p.QC + (long)grow * p.N + gcol) = val;
    }
    if (tid < BM) {
      const int grow = m0 + tid;
      const int nsb = p.N / 32;  // scale bytes per row
      if (grow < p.M) {
        const unsigned val = *reinterpret_cast<const unsigned*>(Ss + tid * 4);
        unsigned char* dst = p.SC + (long)grow * nsb + n0 / 32;
        if (n0 + 128 <= p.N && (nsb & 3) == 0) {
          *reinterpret_cast<unsigned*>(dst) = val;
        } else {
          for (int b = 0; b < 4 && n0 + 32 * b < p.N; ++b) dst[b] = (unsigned char)(val >> (8 * b));
        }
      }
    }
  }
  if (qtout) {
    // transposed MX copy from the bf16 image: work item (column pair c, c + 1; 32-row block tb),
    // one 4-byte LDS read per row for both columns; the row blocks of a pair sit in consecutive
    // lanes, so each store instruction writes 16 rows of QT as 128-byte runs
    constexpr int NB = BM / 32;
#pragma unroll
    for (int r = 0; r < 64 * NB / NT; ++r) {
      const int w = tid + NT * r, c = 2 * (w / NB), tb = w % NB;
      // 32 rows of the column pair (c, c + 1) as packed bf16 words; the block amax of each column
      // as an integer max of the magnitude bits (both columns at once), then the rows re-paired
      // along the column for the scaled conversions
      unsigned h[32];
      unsigned mx = 0u;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const int lr = tb * 32 + k;
        h[k] = *reinterpret_cast<const unsigned*>(Cs + lr * 256 + (((c >> 3) ^ (lr & 15)) << 4) + ((c & 7) << 1));
        const unsigned a = h[k] & 0x7fff7fffu;
        mx = max(mx & 0xffffu, a & 0xffffu) | max(mx & 0xffff0000u, a & 0xffff0000u);
      }
      const float a0 = __uint_as_float(mx << 16), a1 = __uint_as_float(mx & 0xffff0000u);
      const int x0 = mx_exponent(a0), x1 = mx_exponent(a1);
      const float s0 = mx_scale_pow2(x0), s1 = mx_scale_pow2(x1);
      u32x4 o0[2], o1[2];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const unsigned p00 = (h[4 * k] & 0xffffu) | (h[4 * k + 1] << 16);
        const unsigned p01 = (h[4 * k + 2] & 0xffffu) | (h[4 * k + 3] << 16);
        const unsigned p10 = (h[4 * k] >> 16) | (h[4 * k + 1] & 0xffff0000u);
        const unsigned p11 = (h[4 * k + 2] >> 16) | (h[4 * k + 3] & 0xffff0000u);
        o0[k >> 2][k & 3] = cvt4_e4m3_bf16(p00, p01, s0);
        o1[k >> 2][k & 3] = cvt4_e4m3_bf16(p10, p11, s1);
      }
      const int gcol = n0 + c, grow = m0 + tb * 32;
      if (grow < p.M) {  // M % 32 == 0 (launcher): blocks are whole; N % 8: pairs are whole
        if (gcol < p.N) {
          u32x4* dst = reinterpret_cast<u32x4*>(p.QT + (long)gcol * p.ldqt + grow);
          dst[0] = o0[0];
          dst[1] = o0[1];
          p.ST[(long)gcol * (p.ldqt / 32) + grow / 32] = (unsigned char)(x0 + 127);
        }
        if (gcol + 1 < p.N) {
          u32x4* dst = reinterpret_cast<u32x4*>(p.QT + (long)(gcol + 1) * p.ldqt + grow);
          dst[0] = o1[0];
          dst[1] = o1[1];
          p.ST[(long)(gcol + 1) * (p.ldqt / 32) + grow / 32] = (unsigned char)(x1 + 127);
        }
      }
    }
  }
}

#undef F8_ISSUE
template __global__ void gemm_mx_fp8_kernel<128, 2, 0>(F8Args);
template __global__ void gemm_mx_fp8_kernel<128, 3, 0>(F8Args);
template __global__ void gemm_mx_fp8_kernel<256, 2, 0>(F8Args);
template __global__ void gemm_mx_fp8_kernel<256, 3, 0>(F8Args);
template __global__ void gemm_mx_fp8_kernel<128, 2, 1>(F8Args);
template __global__ void gemm_mx_fp8_kernel<128, 2, 2>(F8Args);
template __global__ void gemm_mx_fp8_kernel<128, 2, 3>(F8Args);

// ---------------------------------------------------------------------------- GEMM, 8 waves
// Large-tile MX-fp8 GEMM: BM x BN output tile, 8 waves (WM x WN, each (BM/WM) x (BN/WN)), BK =
// 128, a two-stage LDS-DMA ring.  Why not the 4-wave 128x128 kernel above: at T=16384 its
// 128x128 tiles pull 32 KiB per 512 MFMA cycles per CU from L2 / the Infinity Cache (about the
// L2's whole bandwidth at the fp8 MFMA rate), the 16-MFMA K-tile is too short to cover the
// next tile's load latency, and its runtime-flag epilogue costs ~1900 VALU per wave (PMC:
// 24 VALU per MFMA, MFMA busy 20 %).  Here a 256x256 tile halves the bytes per FLOP, two
// waves per SIMD interleave, and the epilogue is one pass that writes the finished bf16 tile
// into an LDS image (the idle ring), followed by cooperative passes for each requested output:
// the bf16 rows, the row-blocked MX copy and the transposed (token-blocked) MX copy, each read
// from the image with conflict-free lane mappings and stored as whole 16 / 32-byte pieces.
// F32: plain (split-K slab) f32 output straight from the accumulators.
template <int BM, int BN, int WM, bool F32, int NST>
__global__ __launch_bounds__(512) void gemm_mx8_kernel(F8Args p) {
  constexpr int NW = 8, WN = NW / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  constexpr int A_T = BM * F8_BK, B_T = BN * F8_BK;
  constexpr int NSA = (BM + 63) / 64, NSB = (BN + 63) / 64;  // 64-row scale-word instructions
  constexpr int STAGE = A_T + B_T + 256 * (NSA + NSB);
  constexpr int PA = (BM / 8 + NW - 1) / NW, PB = (BN / 8 + NW - 1) / NW, PS = (NSA + NSB + NW - 1) / NW;
  constexpr int L = PA + PB + PS;  // DMA instructions per wave per K-tile (uniform: extras repeat)
  constexpr int RS = BN * 2 + 16;  // image row stride (bytes): padded so 16 rows spread over banks
  constexpr int CSP = 512 / BN;    // column-sum partials per column (threads per column)
  constexpr int IMG = BM * RS + 4 * CSP * BN;
  constexpr int SMEM = NST * STAGE > IMG ? NST * STAGE : IMG;
  static_assert(SMEM <= 163840 && L * (NST - 1) <= 63, "LDS / vmcnt budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int ntn = (p.N + BN - 1) / BN;
  const int ntiles = ((p.M + BM - 1) / BM) * ntn;
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = item % ntiles, split = item / ntiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int KB = p.K / 32;
  const int kt0 = split * p.kps;
  const int nk = min(p.K / F8_BK - kt0, p.kps);

  const __amdgpu_buffer_rsrc_t ra = f8_rsrc(p.A, (long)(p.M - 1) * p.lda + p.K);
  const __amdgpu_buffer_rsrc_t rb = f8_rsrc(p.B, (long)(p.N - 1) * p.ldb + p.K);
  const __amdgpu_buffer_rsrc_t rsa = f8_rsrc(p.SA, (long)(p.M - 1) * p.ldsa + KB);
  const __amdgpu_buffer_rsrc_t rsb = f8_rsrc(p.SB, (long)(p.N - 1) * p.ldsb + KB);

  // 1 KiB pieces (8 rows x 128 B): piece q of A / B; waves past the last piece repeat it
  int voa[PA], vob[PB], vos[PS], dsa[PA], dsb[PB], dss[PS];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int q = min(wave + NW * i, BM / 8 - 1);
    const int row = 8 * q + (lane >> 3), slot = lane & 7;
    voa[i] = (m0 + row) * p.lda + 16 * f8_swz(row, slot);
    dsa[i] = q * 1024;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int q = min(wave + NW * i, BN / 8 - 1);
    const int row = 8 * q + (lane >> 3), slot = lane & 7;
    vob[i] = (n0 + row) * p.ldb + 16 * f8_swz(row, slot);
    dsb[i] = A_T + q * 1024;
  }
  // scale words (4 B per lane: one row's 4 scale bytes of a K-tile, 64 rows per instruction);
  // rows past the tile read whatever the buffer holds (or 0 past its end) into unused words
  bool sis_a[PS];
#pragma unroll
  for (int i = 0; i < PS; ++i) {
    const int si = min(wave + NW * i, NSA + NSB - 1);
    sis_a[i] = si < NSA;
    const int r = 64 * (sis_a[i] ? si : si - NSA) + lane;
    vos[i] = sis_a[i] ? (m0 + r) * p.ldsa : (n0 + r) * p.ldsb;
    dss[i] = A_T + B_T + 256 * si;
  }

#define MX8_ISSUE(KT, ST)                                                                         \
  do {                                                                                            \
    unsigned char* base_ = smem + (ST) * STAGE;                                                   \
    _Pragma("unroll") for (int i_ = 0; i_ < PA; ++i_)                                             \
        f8_dma(ra, base_ + dsa[i_], 16, voa[i_], (kt0 + (KT)) * F8_BK);                           \
    _Pragma("unroll") for (int i_ = 0; i_ < PB; ++i_)                                             \
        f8_dma(rb, base_ + dsb[i_], 16, vob[i_], (kt0 + (KT)) * F8_BK);                           \
    _Pragma("unroll") for (int i_ = 0; i_ < PS; ++i_)                                             \
        f8_dma(sis_a[i_] ? rsa : rsb, base_ + dss[i_], 4, vos[i_], (kt0 + (KT)) * 4);             \
  } while (0)

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) MX8_ISSUE(s, s);
  const int g = lane >> 4, r16 = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    // K-tile kt landed (this wave's pieces); younger stages may stay in flight
    if constexpr (NST >= 3) {
      if (kt + NST - 2 >= nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned char* As_ = smem + (kt % NST) * STAGE;
    const unsigned char* Bs_ = As_ + A_T;
    const unsigned* Sa = reinterpret_cast<const unsigned*>(As_ + A_T + B_T);
    const unsigned* Sb = reinterpret_cast<const unsigned*>(As_ + A_T + B_T + 256 * NSA);
    i32x8 bfr[TN];
    int sb[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wc * WTN + 16 * j + r16;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Bs_ + row * 128 + 16 * f8_swz(row, g));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Bs_ + row * 128 + 16 * f8_swz(row, g + 4));
      bfr[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      sb[j] = (int)((Sb[row] >> (8 * g)) & 0xff);
    }
    // the DMA NST-1 K-tiles ahead once this wave's fragment reads are issued (its stage was
    // released by every wave at the barrier above)
    if (kt + NST - 1 < nk) MX8_ISSUE(kt + NST - 1, (kt + NST - 1) % NST);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * WTM + 16 * i + r16;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(As_ + row * 128 + 16 * f8_swz(row, g));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(As_ + row * 128 + 16 * f8_swz(row, g + 4));
      const i32x8 af = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      const int sa = (int)((Sa[row] >> (8 * g)) & 0xff);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f8_mfma(bfr[j], af, acc[i][j], sb[j], sa);
    }
  }
#undef MX8_ISSUE

  // lane (g, r16) holds C[m0 + wr WTM + 16 i + r16][n0 + wc WTN + 16 j + 4 g + e], e = 0..3
  const bool relu = p.flags & 1, has_bias = p.flags & 2, bias_f32 = p.flags & 4;
  const int rowb = wr * WTM + r16, colb = wc * WTN + 4 * g;
  float bv[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = n0 + colb + 16 * j + e;
      bv[j][e] = (has_bias && col < p.N) ? (bias_f32 ? reinterpret_cast<const float*>(p.bias)[col]
                                                     : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[col]))
                                         : 0.f;
    }
  if constexpr (F32) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + rowb + 16 * i;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + colb + 16 * j;
        if (row < p.M && col < p.N) {
          f32x4 v = acc[i][j];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] += bv[j][e];
            if (relu) v[e] = fmaxf(v[e], 0.f);
          }
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.C) + split * p.sC + (long)row * p.ldc + col) = v;
        }
      }
    }
    return;
  } else {
    const bool res_add = p.flags & 64, res_mask = p.flags & 128, qout = p.flags & 256;
    const bool qtout = p.flags & 512, r_fp8 = p.flags & 1024;
    __syncthreads();  // every wave is done reading the ring: it becomes the bf16 image
    const __amdgpu_buffer_rsrc_t rr =
        f8_rsrc(p.R, (r_fp8 ? 1 : 2) * ((long)(p.M - 1) * p.ldr + p.N) * ((res_add || res_mask) ? 1 : 0));
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int lr = rowb + 16 * i, row = m0 + lr;
      u32x2 rv[TN];
      if (res_add || res_mask) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + colb + 16 * j;
          const bool ok = row < p.M && col < p.N;
          if (r_fp8) {
            const unsigned b = __builtin_amdgcn_raw_buffer_load_b32(rr, ok ? (int)((long)row * p.ldr + col) : 0x7ffffff0, 0, 0);
            rv[j] = u32x2{b, 0u};
          } else {
            rv[j] = __builtin_amdgcn_raw_buffer_load_b64(rr, ok ? (int)(((long)row * p.ldr + col) * 2) : 0x7ffffff0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] + bv[j][e];
          if (relu) v[e] = fmaxf(v[e], 0.f);
        }
        if (res_mask && r_fp8) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const unsigned byte = (rv[j][0] >> (8 * e)) & 0xffu;
            v[e] = ((byte & 0x80u) == 0u && byte != 0u) ? v[e] : 0.f;
          }
        } else if (res_add || res_mask) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const unsigned w = rv[j][e >> 1];
            const float r = (e & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
            if (res_add) v[e] = bf2f(f2bf(v[e])) + r;
            else v[e] = r > 0.f ? v[e] : 0.f;
          }
        }
        *reinterpret_cast<u32x2*>(smem + lr * RS + (colb + 16 * j) * 2) =
            u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
      }
    }
    __syncthreads();
    if (p.flags & 2048) {
      // column sums of the bf16 output tile (a bias gradient downstream): CSP threads per column
      // over row ranges, partials through LDS, one f32 per column and tile row to csum
      float* part = reinterpret_cast<float*>(smem + BM * RS);
      if (tid < CSP * BN) {
        const int c = tid % BN, pr = tid / BN;
        const int r0 = pr * BM / CSP, r1 = min((pr + 1) * BM / CSP, p.M - m0);
        float acc = 0.f;
        for (int r = r0; r < r1; ++r) acc += bf2f(*reinterpret_cast<const bf16_t*>(smem + r * RS + c * 2));
        part[pr * BN + c] = acc;
      }
      __syncthreads();
      if (tid < BN && n0 + tid < p.N) {
        float a = 0.f;
#pragma unroll
        for (int pr = 0; pr < CSP; ++pr) a += part[pr * BN + tid];
        p.csum[(long)(m0 / BM) * p.N + n0 + tid] = a;
      }
    }
    if (p.C) {  // bf16 rows: 16 B per lane, consecutive lanes along a row
      for (int c = tid; c < BM * (BN / 8); c += 512) {
        const int lr = c / (BN / 8), ch = c % (BN / 8);
        const int grow = m0 + lr, gcol = n0 + ch * 8;
        const u32x4 val = *reinterpret_cast<const u32x4*>(smem + lr * RS + ch * 16);
        if (grow < p.M && gcol < p.N)
          *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(p.C) + (long)grow * p.ldc + gcol) = val;
      }
    }
    if (qout) {  // row-blocked MX copy: lane = (row, 32-column block), rows consecutive across lanes
      for (int it = tid; it < BM * (BN / 32); it += 512) {
        const int lr = it % BM, b = it / BM;
        const int grow = m0 + lr, gcol = n0 + 32 * b;
        // 32 bf16 of the row as 16 packed words: amax as an integer max of the magnitude bits,
        // then the scaled conversions straight from the pairs
        u32x4 w[4];
        unsigned mx = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          w[k] = *reinterpret_cast<const u32x4*>(smem + lr * RS + b * 64 + k * 16);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const unsigned a = w[k][e] & 0x7fff7fffu;
            mx = max(mx, max(a & 0xffffu, a >> 16));
          }
        }
        const int x = mx_exponent(__uint_as_float(mx << 16));
        const float sc = mx_scale_pow2(x);
        u32x4 o[2];
#pragma unroll
        for (int c = 0; c < 8; ++c) o[c >> 2][c & 3] = cvt4_e4m3_bf16(w[c >> 1][2 * (c & 1)], w[c >> 1][2 * (c & 1) + 1], sc);
        if (grow < p.M && gcol < p.N) {
          u32x4* dst = reinterpret_cast<u32x4*>(p.QC + (long)grow * p.N + gcol);
          dst[0] = o[0];
          dst[1] = o[1];
          p.SC[(long)grow * (p.N / 32) + gcol / 32] = (unsigned char)(x + 127);
        }
      }
    }
    if (qtout) {  // transposed MX copy: lane = (column pair, 32-row block), pairs consecutive across lanes
      for (int it = tid; it < (BN / 2) * (BM / 32); it += 512) {
        const int cp = it % (BN / 2), tb = it / (BN / 2);
        unsigned h[32];
        unsigned mx = 0u;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
          h[k] = *reinterpret_cast<const unsigned*>(smem + (tb * 32 + k) * RS + cp * 4);
          const unsigned a = h[k] & 0x7fff7fffu;
          mx = max(mx & 0xffffu, a & 0xffffu) | max(mx & 0xffff0000u, a & 0xffff0000u);
        }
        const int x0 = mx_exponent(__uint_as_float(mx << 16)), x1 = mx_exponent(__uint_as_float(mx & 0xffff0000u));
        const float s0 = mx_scale_pow2(x0), s1 = mx_scale_pow2(x1);
        u32x4 o0[2], o1[2];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o0[k >> 2][k & 3] = cvt4_e4m3_bf16((h[4 * k] & 0xffffu) | (h[4 * k + 1] << 16),
                                             (h[4 * k + 2] & 0xffffu) | (h[4 * k + 3] << 16), s0);
          o1[k >> 2][k & 3] = cvt4_e4m3_bf16((h[4 * k] >> 16) | (h[4 * k + 1] & 0xffff0000u),
                                             (h[4 * k + 2] >> 16) | (h[4 * k + 3] & 0xffff0000u), s1);
        }
        const int gcol = n0 + 2 * cp, grow = m0 + tb * 32;
        if (grow < p.M) {  // M % 32 == 0 (launcher): blocks are whole; N % 8: pairs are whole
          if (gcol < p.N) {
            u32x4* dst = reinterpret_cast<u32x4*>(p.QT + (long)gcol * p.ldqt + grow);
            dst[0] = o0[0];
            dst[1] = o0[1];
            p.ST[(long)gcol * (p.ldqt / 32) + grow / 32] = (unsigned char)(x0 + 127);
          }
          if (gcol + 1 < p.N) {
            u32x4* dst = reinterpret_cast<u32x4*>(p.QT + (long)(gcol + 1) * p.ldqt + grow);
            dst[0] = o1[0];
            dst[1] = o1[1];
            p.ST[(long)(gcol + 1) * (p.ldqt / 32) + grow / 32] = (unsigned char)(x1 + 127);
          }
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int NST = 2>
hipError_t launch_mx8(const F8Args& a, int tiles, hipStream_t s) {
  if (a.flags & 32)
    hipLaunchKernelGGL((gemm_mx8_kernel<BM, BN, WM, true, NST>), dim3(tiles), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_mx8_kernel<BM, BN, WM, false, NST>), dim3(tiles), dim3(512), 0, s, a);
  return hipGetLastError();
}

template <int BM, int NST>
hipError_t launch_f8(const F8Args& a, int tiles, hipStream_t s) {
  // the FF block's up projection / dA epilogues get their compile-time specialisations
  if (BM == 128 && NST == 2 && a.C == nullptr && a.bias == nullptr && a.nsplit == 1) {
    if (a.flags == (1 | 256 | 512)) {
      hipLaunchKernelGGL((gemm_mx_fp8_kernel<128, 2, 1>), dim3(tiles), dim3(256), 0, s, a);
      return hipGetLastError();
    }
    if (a.flags == (128 | 1024 | 256 | 512)) {
      hipLaunchKernelGGL((gemm_mx_fp8_kernel<128, 2, 2>), dim3(tiles), dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
  // plain f32 output (the FF weight gradients): its own instance -- the general kernel's 288
  // registers (VGPR + AGPR) left one wave per SIMD
  if (BM == 128 && NST == 2 && a.flags == 32 && a.bias == nullptr) {
    hipLaunchKernelGGL((gemm_mx_fp8_kernel<128, 2, 3>), dim3(tiles), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((gemm_mx_fp8_kernel<BM, NST, 0>), dim3(tiles), dim3(BM * 2), 0, s, a);
  return hipGetLastError();
}

// one wave, one block-scaled MFMA on raw per-lane operands (layout validation in the tests)
__global__ void debug_mfma_f8_kernel(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x4* c) {
  const int l = threadIdx.x;
  c[l] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0, sa[l], 0,
                                                          sb[l]);
}

}  // namespace

// semantics probe of the gfx950 scaled conversion v_cvt_scalef32_pk_fp8_bf16 against the
// reference path (bf16 -> f32, times 2^-x, RNE to e4m3): per element i (bf16 pair in[i], block
// exponent x[i]): out[4 i + 0..1] = reference bytes, out[4 i + 2] = scalef32 with scale 2^x,
// out[4 i + 3] = scalef32 with scale 2^-x (low bytes of each)
__global__ void debug_cvt_scalef_kernel(const unsigned* in, const int* xs, unsigned* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned w = in[i];
  const int x = xs[i];
  const float a = __uint_as_float(w << 16), b = __uint_as_float(w & 0xffff0000u);
  const float inv = ldexpf(1.f, -x);
  const unsigned ref = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(a * inv, b * inv, 0, false) & 0xffffu;
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef short s2 __attribute__((ext_vector_type(2)));
  const bf2 v = __builtin_bit_cast(bf2, w);
  s2 o1 = {0, 0}, o2 = {0, 0};
  o1 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o1, v, ldexpf(1.f, x), false);
  o2 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o2, v, inv, false);
  out[4 * i] = ref;
  out[4 * i + 1] = 0;
  out[4 * i + 2] = __builtin_bit_cast(unsigned, o1) & 0xffffu;
  out[4 * i + 3] = __builtin_bit_cast(unsigned, o2) & 0xffffu;
}

// a, b: 64 lanes x 32 bytes; sa, sb: 64 ints (scale byte in bits 0-7); c: 64 lanes x 4 floats
LJS_API int ljs_debug_cvt_scalef(const void* in, const void* xs, void* out, int n, hipStream_t stream) {
  hipLaunchKernelGGL(debug_cvt_scalef_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, (const unsigned*)in,
                     (const int*)xs, (unsigned*)out, n);
  return (int)hipGetLastError();
}

LJS_API int ljs_debug_mfma_f8(const void* a, const void* b, const void* sa, const void* sb, void* c,
                              hipStream_t stream) {
  hipLaunchKernelGGL(debug_mfma_f8_kernel, dim3(1), dim3(64), 0, stream, (const i32x8*)a, (const i32x8*)b,
                     (const int*)sa, (const int*)sb, (f32x4*)c);
  return (int)hipGetLastError();
}

// a scalar cotangent g broadcast over a row of C: its bf16 row and that row's MX-fp8 rows (every
// 32-block has amax |bf16(g)|) in one launch -- the broadcast dY of y.sum(), read by the GEMMs
// as ONE row (ld 0 / a_bcast); C % 32 == 0
__global__ void bcast_scalar_mx_kernel(const void* __restrict__ g, int g_bf16, int C, bf16_t* __restrict__ row,
                                       unsigned char* __restrict__ q, unsigned char* __restrict__ s) {
  const int c4 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (c4 >= C) return;
  const float v = bf2f(f2bf(g_bf16 ? bf2f(*reinterpret_cast<const bf16_t*>(g)) : *reinterpret_cast<const float*>(g)));
  *reinterpret_cast<u32x2*>(row + c4) = u32x2{pack_bf16x2(v, v), pack_bf16x2(v, v)};
  const int x = mx_exponent(fabsf(v));
  const float sv = v * ldexpf(1.f, -x);
  *reinterpret_cast<unsigned*>(q + c4) = pack4_e4m3(sv, sv, sv, sv);
  if ((c4 & 31) == 0) s[c4 / 32] = (unsigned char)(x + 127);
}

LJS_API int ljs_bcast_scalar_mx(const void* g, int g_bf16, int C, void* row, void* q, void* s, hipStream_t stream) {
  if (C % 32) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bcast_scalar_mx_kernel, dim3((C / 4 + 255) / 256), dim3(256), 0, stream, g, g_bf16, C,
                     (bf16_t*)row, (unsigned char*)q, (unsigned char*)s);
  return (int)hipGetLastError();
}

// x[R][K] (row stride ld elements) -> q[R][K], s[R][K/32] (+ xb[R][K] bf16 for an f32 x, when
// xb != null); K % 32 == 0, 16-byte aligned rows
LJS_API int ljs_quant_mx_rows(const void* in, int is_bf16, long ld, int R, int K, void* q, void* s, void* xb,
                              hipStream_t stream) {
  if (K % 32 || ld % 8 || (xb && (is_bf16 || ((uintptr_t)xb & 15)))) return (int)hipErrorInvalidValue;
  const long nb = (long)R * (K / 32);
  hipLaunchKernelGGL(quant_mx_rows_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, stream, in, is_bf16, ld,
                     R, K, (unsigned char*)q, (unsigned char*)s, (bf16_t*)xb);
  return (int)hipGetLastError();
}

// w[K][N] (row stride ld) -> q[N][K], s[N][K/32]
LJS_API int ljs_quant_mx_cols(const void* in, int is_bf16, long ld, int K, int N, void* q, void* s,
                              hipStream_t stream) {
  if (K % 32) return (int)hipErrorInvalidValue;
  if (is_bf16 && K % 128 == 0 && N % 64 == 0 && ld % 8 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)q & 15) == 0) {
    hipLaunchKernelGGL(quant_mx_cols_tiled_kernel<false>, dim3(N / 64, K / 128), dim3(256), 0, stream, in, ld, K, N,
                       (unsigned char*)q, (unsigned char*)s, nullptr, nullptr, nullptr);
    return (int)hipGetLastError();
  }
  dim3 grid((N + 63) / 64, K / 32);
  hipLaunchKernelGGL(quant_mx_cols_kernel, grid, dim3(64), 0, stream, in, is_bf16, ld, K, N, (unsigned char*)q,
                     (unsigned char*)s);
  return (int)hipGetLastError();
}

// C[M][N] (bf16, or f32 with flags & 32) = A . B^T of MX-fp8 operands; K % 128 == 0, N % 8 == 0.
// R (bf16 [M][N], row stride ldr) with flags 64 / 128: residual add / ReLU mask in the epilogue;
// QC / SC with flags 256: also an MX-fp8 copy of the output (N % 32 == 0); QT / ST with flags 512:
// its TRANSPOSED MX copy QT[N][M] (row stride ldqt = M, blocks along M; M % 32 == 0, bf16-path
// outputs only); flags 1024: R is e4m3 [M][N] (ReLU mask of an fp8-only activation).
// a_bcast / b_bcast: A / B (and scales) hold one row, read for every row.  nsplit > 1: split-K,
// split s writing the f32 slab C + s * sC (summed by the caller).  tile: 1282 / 1283 / 2562 /
// 2563 = BM x 128 with 2 or 3 stages (0: automatic).
LJS_API int ljs_gemm_mx_fp8(const void* A, const void* SA, const void* B, const void* SB, void* C, const void* bias,
                            int M, int N, int K, long ldc, int flags, const void* R, long ldr, void* QC, void* SC,
                            int tile, int a_bcast, int b_bcast, void* QT, void* ST, long ldqt, int nsplit, long sC,
                            void* csum, hipStream_t stream) {
  if (K % F8_BK || N % 8 || ldc % 8 || (long)M * K >= (1L << 31) || (long)N * K >= (1L << 31))
    return (int)hipErrorInvalidValue;
  if ((flags & (64 | 128)) && (!R || ldr % 8 || (((uintptr_t)R) & 15) || (flags & 32)))
    return (int)hipErrorInvalidValue;
  if ((flags & 1024) && !(flags & 128)) return (int)hipErrorInvalidValue;
  if ((flags & 256) && (!QC || !SC || N % 32)) return (int)hipErrorInvalidValue;
  if ((flags & 512) && (!QT || !ST || M % 32 || ldqt < M || ldqt % 32 || (flags & 32) || ((uintptr_t)QT & 15)))
    return (int)hipErrorInvalidValue;
  if (nsplit < 1) nsplit = 1;
  const int nkt = K / F8_BK;
  const int kps = (nkt + nsplit - 1) / nsplit;
  if (nsplit > 1 && (!(flags & 32) || (flags & (64 | 128 | 256 | 512 | 2)) || (nkt + kps - 1) / kps != nsplit))
    return (int)hipErrorInvalidValue;  // split-K: plain f32 slabs, and the caller's slab count exact
  F8Args a;
  a.A = (const unsigned char*)A; a.B = (const unsigned char*)B;
  a.SA = (const unsigned char*)SA; a.SB = (const unsigned char*)SB;
  a.C = C; a.bias = bias; a.ldc = ldc; a.M = M; a.N = N; a.K = K; a.flags = flags;
  a.R = (const bf16_t*)R; a.ldr = ldr; a.QC = (unsigned char*)QC; a.SC = (unsigned char*)SC;
  a.lda = a_bcast ? 0 : K;  // a_bcast: A / SA hold ONE row, read for every output row
  a.ldsa = a_bcast ? 0 : K / 32;
  a.ldb = b_bcast ? 0 : K;
  a.ldsb = b_bcast ? 0 : K / 32;
  a.QT = (unsigned char*)QT; a.ST = (unsigned char*)ST; a.ldqt = ldqt;
  a.kps = kps; a.nsplit = nsplit; a.sC = sC;
  a.csum = (float*)csum;
  // fused column sums: the 8-wave kernels' bf16 epilogue only
  if ((flags & 2048) && (!csum || tile < 10000 || (flags & 32))) return (int)hipErrorInvalidValue;
  if (tile == 0) tile = 1282;
  if (tile >= 10000) {  // 8-wave large tiles: tile = BM * 1000 + BN (+ 1000000 * 3: three stages)
    const int t6 = tile % 1000000;
    const int bm = t6 / 1000, bn = t6 % 1000;
    const int tl = ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * nsplit;
    switch (tile) {
      case 256256: return (int)launch_mx8<256, 256, 2>(a, tl, stream);
      case 256128: return (int)launch_mx8<256, 128, 2>(a, tl, stream);
      case 256160: return (int)launch_mx8<256, 160, 4>(a, tl, stream);
      case 128320: return (int)launch_mx8<128, 320, 2>(a, tl, stream);
      case 128256: return (int)launch_mx8<128, 256, 2>(a, tl, stream);
      case 128128: return (int)launch_mx8<128, 128, 2>(a, tl, stream);
      case 128160: return (int)launch_mx8<128, 160, 4>(a, tl, stream);
      case 3128128: return (int)launch_mx8<128, 128, 2, 3>(a, tl, stream);
      case 3128160: return (int)launch_mx8<128, 160, 4, 3>(a, tl, stream);
      case 3128256: return (int)launch_mx8<128, 256, 2, 3>(a, tl, stream);
      case 3256128: return (int)launch_mx8<256, 128, 2, 3>(a, tl, stream);
      default: return (int)hipErrorInvalidValue;
    }
  }
  const int bm = tile / 10 >= 256 ? 256 : 128;
  const int tiles = ((M + bm - 1) / bm) * ((N + 127) / 128) * nsplit;
  if (tile == 1283) return (int)launch_f8<128, 3>(a, tiles, stream);
  if (tile == 2562) return (int)launch_f8<256, 2>(a, tiles, stream);
  if (tile == 2563) return (int)launch_f8<256, 3>(a, tiles, stream);
  return (int)launch_f8<128, 2>(a, tiles, stream);
}
