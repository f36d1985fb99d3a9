// Batched bf16 GEMM on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), f32 accumulation.
//
//   C[b] = alpha * op(A[b]) @ op(B[b]) (+ bias) (relu)        (bf16 or f32 out, optional split-K)
//
// Operand layouts (template flags), covering every GEMM of the attention block's
// forward and backward without transposing anything in memory:
//   A_KC : A[m][k] at A + m*lda + k   (k contiguous)      | !A_KC : A[m][k] at A + k*lda + m
//   B_KC : B[k][n] at B + n*ldb + k   (k contiguous)      | !B_KC : B[k][n] at B + k*ldb + n
// k-contiguous operands are staged as [rows][64] LDS tiles read with ds_read_b128;
// m/n-contiguous operands as [64][rows] tiles read with the gfx950 transposing LDS read
// (ds_read_b64_tr_b16), so e.g. dW = X^T @ dY reads X and dY in their natural layouts.
//
// Structure: 256 threads = 4 waves (2x2), block tile BM x BN, BK = 64, LDS double buffer
// with register staging (issue next tile's global loads before the MFMAs, write them to
// the other LDS buffer after; one barrier per K-tile), XOR-swizzled LDS images so both
// the row reads and the transposed reads are bank-conflict free, XCD-aware tile order.
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace {

constexpr int BK = 64;

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const void* bias;
  long lda, ldb, ldc;
  long sA, sB, sC, sBias;
  int M, N, K;
  int batch, splitk, kt_per_split;
  float alpha;
  int flags;  // 1 relu, 2 bias, 4 bias f32, 8 accumulate into C (f32 out); epilogue operand R
              // (bf16 output only): 64 residual add, 128 ReLU mask (keep where R > 0), 256 R is f32
  float* psum;  // LDS-DMA kernels, bf16 out: per (item, wave) sums of the stored values, or null
  const void* res;  // R[b][row][col] at res + b * sR + row * ldr + col (ldr may be 0: one broadcast row)
  long ldr, sR;
  const bf16_t* bptr[4];  // flags & kBPtrs (slab mode): batch b's B operand (instead of B + b * sB)
  unsigned long long* trace;  // LJS_GEMM_TRACE builds only: per-wave timestamps (see gemm_trace)
};

// Timeline instrumentation of the LDS-DMA kernel (compiled in with -DLJS_GEMM_TRACE only, a
// variant library for scripts/gemm_trace.py): per wave, kTraceSlots core-clock stamps (s_memtime)
// written by lane 0 with vector stores -- kernel start, then per K-tile wait: before the counted
// vmcnt, after it, after the barrier -- and the end.
constexpr int kTraceSlots = 128;

constexpr int kResAdd = 64, kResMask = 128, kResF32 = 256;
// f32 output, m/n-contiguous operands, batch 1: split s writes its own slab C + s * sC (no
// atomics; summed by slab_reduce) and the splits need not divide the K-tiles -- the last one
// runs past K, where the buffer range check reads zeros
constexpr int kSlabs = 512;
// item order with the tile-row fastest (set by the launcher when there are fewer tile rows
// than tile columns; see decode_item)
constexpr int kMFast = 1024;
// B operand of batch b taken from bptr[b] (up to 4 separate tensors, e.g. the q / k / v
// cotangents of a weight-major fused projection) -- slab-mode LDS-DMA kernels only
constexpr int kBPtrs = 4096;
// slab mode, the block's LAST item: its f32 tile leaves through the (then idle) LDS ring as whole
// 256-byte rows (16-byte chunk XOR row), not as 64-byte pieces of 16 rows per store instruction
constexpr int kSlabVst = 8192;

// Epilogue operand R applied to 8 consecutive output values (after bias / ReLU, f32):
//   residual add: out = bf16(bf16(v) + bf16(R))   (the unfused "y = dense(x); y + R" in bf16:
//                 both roundings kept, so the fusion is bit-exact)
//   ReLU mask   : out = R > 0 ? v : 0             (the ReLU backward of a dense whose input R is a
//                 ReLU output, fused into the dX GEMM producing v)
// rb holds R's 8 values as bf16 pairs (bf16 R) or rf their f32 values (f32 R).
__device__ __forceinline__ void apply_res8(float* v, int flags, const u32x4& rb, const u32x4& rf0,
                                           const u32x4& rf1) {
  float r[8];
  if (flags & kResF32) {
#pragma unroll
    for (int e = 0; e < 4; ++e) { r[e] = __uint_as_float(rf0[e]); r[4 + e] = __uint_as_float(rf1[e]); }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r[2 * e] = __uint_as_float(rb[e] << 16);
      r[2 * e + 1] = __uint_as_float(rb[e] & 0xffff0000u);
    }
  }
  if (flags & kResAdd) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e])) + bf2f(f2bf(r[e]));
  } else if (flags & kResMask) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = r[e] > 0.f ? v[e] : 0.f;
  }
}

// swizzled 8-byte-chunk index for the m/n-contiguous image (rows of R bf16)
template <int R>
__device__ __forceinline__ int swz_mn(int krow, int c8) {
  int f;
  if constexpr (R >= 128) f = ((krow & 3) | (((krow >> 3) & 1) << 2)) << 2;
  else f = ((((krow >> 1) & 1)) | (((krow >> 3) & 1) << 1)) << 2;
  return c8 ^ f;
}

// swizzled 16-byte-chunk index for the k-contiguous image (rows of 64 bf16 = 8 chunks)
__device__ __forceinline__ int swz_k(int row, int c16) { return c16 ^ ((row >> 1) & 7); }

template <int R, bool KC>
struct Stage {
  static constexpr int CHUNKS = R * BK * 2 / 16 / 256;  // 16-byte chunks per thread
  u32x4 v[CHUNKS];

  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, int r0, int k0, int R_lim,
                                       int K, int tid) {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i) {
      int c = tid + 256 * i;
      if constexpr (KC) {
        int row = c >> 3, kc = c & 7;
        int gr = r0 + row, gk = k0 + kc * 8;
        if (gr < R_lim && gk < K)
          v[i] = *reinterpret_cast<const u32x4*>(base + (long)gr * ld + gk);
        else
          v[i] = u32x4{0, 0, 0, 0};
      } else {
        constexpr int CPR = R / 8;  // 16B chunks per k-row
        int krow = c / CPR, mc = c % CPR;
        int gk = k0 + krow, gr = r0 + mc * 8;
        if (gk < K && gr < R_lim)
          v[i] = *reinterpret_cast<const u32x4*>(base + (long)gk * ld + gr);
        else
          v[i] = u32x4{0, 0, 0, 0};
      }
    }
  }

  __device__ __forceinline__ void store(bf16_t* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i) {
      int c = tid + 256 * i;
      if constexpr (KC) {
        int row = c >> 3, kc = c & 7;
        *reinterpret_cast<u32x4*>(lds + row * BK + swz_k(row, kc) * 8) = v[i];
      } else {
        constexpr int CPR = R / 8;
        int krow = c / CPR, mc = c % CPR;
        *reinterpret_cast<u32x4*>(lds + krow * R + swz_mn<R>(krow, mc * 2) * 4) = v[i];
      }
    }
  }
};

// MFMA operand fragment: 16 rows (m or n) starting at rb, k-step ks (32 deep)
template <int R, bool KC>
__device__ __forceinline__ bf16x8 frag(const bf16_t* lds, int rb, int ks, int lane) {
  if constexpr (KC) {
    int row = rb + (lane & 15);
    int kc = ks * 4 + (lane >> 4);
    u32x4 raw = *reinterpret_cast<const u32x4*>(lds + row * BK + swz_k(row, kc) * 8);
    return __builtin_bit_cast(bf16x8, raw);
  } else {
    int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    int kr0 = ks * 32 + 8 * g + q;
    int c8 = (rb >> 2) + p;
    s16x4 lo = lds_read_tr16(lds + kr0 * R + swz_mn<R>(kr0, c8) * 4);
    int kr1 = kr0 + 4;
    s16x4 hi = lds_read_tr16(lds + kr1 * R + swz_mn<R>(kr1, c8) * 4);
    return join_bf16x8(lo, hi);
  }
}

template <int BM, int BN, bool A_KC, bool B_KC, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmArgs p) {
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 MFMA tiles per wave (2x2 waves)
  constexpr int A_TILE = BM * BK, B_TILE = BN * BK;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (A_TILE + B_TILE)];
  // (pointer arrays into LDS would become static initializers: index arithmetically)
#define As(i) (smem + (i) * A_TILE)
#define Bs(i) (smem + 2 * A_TILE + (i) * B_TILE)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm_i = tile / ntn, tn_i = tile % ntn;
  if (tm_i >= ntm) return;
  const int bz = blockIdx.y;
  const int b = bz / p.splitk, split = bz % p.splitk;
  const int m0 = tm_i * BM, n0 = tn_i * BN;

  const bf16_t* Ab = p.A + (long)b * p.sA;
  const bf16_t* Bb = p.B + (long)b * p.sB;

  const int nkt_total = (p.K + BK - 1) / BK;
  const int kt_begin = split * p.kt_per_split;
  const int kt_end = min(nkt_total, kt_begin + p.kt_per_split);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage<BM, A_KC> sa;
  Stage<BN, B_KC> sb;
  if (kt_begin < kt_end) {
    sa.load(Ab, p.lda, m0, kt_begin * BK, p.M, p.K, tid);
    sb.load(Bb, p.ldb, n0, kt_begin * BK, p.N, p.K, tid);
    sa.store(As(0), tid);
    sb.store(Bs(0), tid);
  }
  __syncthreads();

  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int cur = (kt - kt_begin) & 1;
    const bool more = kt + 1 < kt_end;
    if (more) {
      sa.load(Ab, p.lda, m0, (kt + 1) * BK, p.M, p.K, tid);
      sb.load(Bb, p.ldb, n0, (kt + 1) * BK, p.N, p.K, tid);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<BM, A_KC>(As(cur), wr * (BM / 2) + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag<BN, B_KC>(Bs(cur), wc * (BN / 2) + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      sa.store(As(cur ^ 1), tid);
      sb.store(Bs(cur ^ 1), tid);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const bool relu = p.flags & 1;
  const bool has_bias = (p.flags & 2) && p.splitk == 1;
  const bool bias_f32 = p.flags & 4;
  const bool accumulate = p.flags & 8;
  if constexpr (!OUT_F32) {
    // bf16 output: stage the tile in LDS (the K loop's last barrier freed it), then write whole
    // rows with 16-byte stores instead of 2-byte scattered accumulator-layout stores.
    constexpr int LDC = BN + 8;
    bf16_t* ct = smem;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wc * (BN / 2) + j * 16 + (lane & 15);
      const int col = n0 + cl;
      float bv = 0.f;
      if (has_bias && col < p.N) {
        const long bo = (long)b * p.sBias + col;
        bv = bias_f32 ? reinterpret_cast<const float*>(p.bias)[bo]
                      : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[bo]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] * p.alpha + bv;
          if (relu) v = fmaxf(v, 0.f);
          ct[(wr * (BM / 2) + i * 16 + (lane >> 4) * 4 + r) * LDC + cl] = f2bf(v);
        }
    }
    __syncthreads();
    bf16_t* Cb = reinterpret_cast<bf16_t*>(p.C) + (long)b * p.sC;
    constexpr int CPR = BN / 8;
    const bool vec_ok = (p.ldc % 8 == 0) && ((((uintptr_t)Cb) & 15) == 0);
    for (int c = tid; c < BM * CPR; c += 256) {
      const int rl = c / CPR, cc = c % CPR;
      const int row = m0 + rl, col = n0 + cc * 8;
      if (row >= p.M || col >= p.N) continue;
      const bf16_t* src = ct + rl * LDC + cc * 8;
      bf16_t* dst = Cb + (long)row * p.ldc + col;
      if (p.flags & (kResAdd | kResMask)) {
        float v[8];
        u32x4 rb = {0, 0, 0, 0}, rf0 = {0, 0, 0, 0}, rf1 = {0, 0, 0, 0};
        const long ro = (long)b * p.sR + (long)row * p.ldr + col;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = bf2f(src[e]);
          if (col + e < p.N) {
            if (p.flags & kResF32) {
              const float rv = reinterpret_cast<const float*>(p.res)[ro + e];
              if (e < 4) rf0[e] = __float_as_uint(rv); else rf1[e - 4] = __float_as_uint(rv);
            } else {
              const unsigned rv = reinterpret_cast<const bf16_t*>(p.res)[ro + e];
              rb[e >> 1] |= (e & 1) ? (rv << 16) : rv;
            }
          }
        }
        apply_res8(v, p.flags, rb, rf0, rf1);
        if (vec_ok && col + 8 <= p.N)
          *reinterpret_cast<u32x4*>(dst) = u32x4{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                 pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
        else
          for (int e = 0; e < 8 && col + e < p.N; ++e) dst[e] = f2bf(v[e]);
      } else if (vec_ok && col + 8 <= p.N) {
        *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
      } else {
        for (int e = 0; e < 8 && col + e < p.N; ++e) dst[e] = src[e];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
      if (col >= p.N) continue;
      float bv = 0.f;
      if (has_bias) {
        const long bo = (long)b * p.sBias + col;
        bv = bias_f32 ? reinterpret_cast<const float*>(p.bias)[bo]
                      : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[bo]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (row >= p.M) continue;
        float v = acc[i][j][r] * p.alpha + bv;
        if (relu) v = fmaxf(v, 0.f);
        const long off = (long)b * p.sC + (long)row * p.ldc + col;
        if constexpr (OUT_F32) {
          float* C = reinterpret_cast<float*>(p.C);
          if (p.splitk > 1) atomicAdd(C + off, v);
          else if (accumulate) C[off] += v;
          else C[off] = v;
        } else {
          reinterpret_cast<bf16_t*>(p.C)[off] = f2bf(v);
        }
      }
    }
  }
}

#undef As
#undef Bs

// ============================================================================ LDS-DMA GEMM
// Persistent, pipelined MFMA GEMM for the large bench shapes.
//  * Staging by the buffer LDS-DMA (buffer_load_dwordx4 ... lds): global -> LDS with no VGPRs
//    and no ds_write (the VGPR->LDS transfer, ~79 B/clk/CU, bounds a register-staged loop).
//    Swizzles are applied on the SOURCE address (the DMA writes a wave's 64 x 16 B
//    contiguously), so the LDS images are those of the kernel above (conflict-free reads).
//  * Persistent blocks walk a FLATTENED (work item, K-tile) sequence through an NST-deep LDS
//    ring with one raw s_barrier per K-tile and a counted vmcnt, so the next item's first
//    tiles are already in flight while the current item's epilogue runs: no per-tile
//    prologue bubble (K = 512/640 projections have only 8-10 K-tiles per item).
//  * The MFMA operands are swapped (C^T = B^T A^T per 16x16 block), so each lane ends with 4
//    CONSECUTIVE columns of one output row: bf16 results leave as packed 8-byte stores and
//    f32 as 16-byte stores straight from the accumulators (no LDS round trip).
//  * Work items are ordered (split, batch, tiles; the dimension of fewer tiles fastest) and
//    dealt XCD-aware, so blocks sharing an XCD's L2 work on neighbouring tiles (shared panels).
// Edges: rows/cols past M/N read garbage that only reaches discarded outputs; the buffer
// descriptor's range check turns every out-of-range read into 0 without faulting; K must be a
// multiple of 64 and the split must divide the K-tiles (checked by the launcher) except in
// slab mode (kSlabs), whose last split reads zeros past K.

// XOR applied to the 16-byte chunk index of k-row `krow` of an m/n-contiguous image (R rows)
template <int R>
__device__ __forceinline__ int swz_mn16(int krow) {
  // (rows of 128 or 256 bf16 start on the same bank; rows of 64 alternate halves)
  if constexpr (R >= 128) return ((krow & 3) | (((krow >> 3) & 1) << 2)) << 1;
  else return ((((krow >> 1) & 1)) | (((krow >> 3) & 1) << 1)) << 1;
}


// s_waitcnt vmcnt with a wave-uniform runtime count (a jump over immediates; counts above 47
// wait for 47, which is only stricter)
template <int N>
__device__ __forceinline__ void wait_vm_imm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
#define LJS_W(k) case k: wait_vm_imm<k>(); return;
    LJS_W(0) LJS_W(1) LJS_W(2) LJS_W(3) LJS_W(4) LJS_W(5) LJS_W(6) LJS_W(7) LJS_W(8) LJS_W(9) LJS_W(10)
    LJS_W(11) LJS_W(12) LJS_W(13) LJS_W(14) LJS_W(15) LJS_W(16) LJS_W(17) LJS_W(18) LJS_W(19) LJS_W(20)
    LJS_W(21) LJS_W(22) LJS_W(23) LJS_W(24) LJS_W(25) LJS_W(26) LJS_W(27) LJS_W(28) LJS_W(29) LJS_W(30)
    LJS_W(31) LJS_W(32) LJS_W(33) LJS_W(34) LJS_W(35) LJS_W(36) LJS_W(37) LJS_W(38) LJS_W(39) LJS_W(40)
    LJS_W(41) LJS_W(42) LJS_W(43) LJS_W(44) LJS_W(45) LJS_W(46)
#undef LJS_W
    default: wait_vm_imm<47>(); return;
  }
}

// One operand tile (R rows x BK) of one K-tile: its 1 KiB DMA pieces, split over NW waves.
// Per-lane offsets are relative to (row 0, k 0); the tile origin goes in the scalar offset.
template <int R, bool KC, int NW>
struct DmaTile {
  static constexpr int PIECES = R * BK * 2 / 1024;
  static constexpr int PER_WAVE = PIECES / NW;
  static_assert(PIECES % NW == 0, "pieces must split evenly over the waves");
  int voff[PER_WAVE];

  __device__ __forceinline__ void init(long ld, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int q = wave + NW * i;
      long e;
      if constexpr (KC) {
        const int row = 8 * q + (lane >> 3), slot = lane & 7;
        e = (long)row * ld + 8 * (slot ^ ((row >> 1) & 7));
      } else {
        constexpr int CPR = R / 8;     // 16 B chunks per k-row
        constexpr int KPP = 64 / CPR;  // k-rows per piece
        const int krow = KPP * q + lane / CPR, slot = lane % CPR;
        e = (long)krow * ld + 8 * (slot ^ swz_mn16<R>(krow));
      }
      voff[i] = (int)(e * 2);
    }
  }

  // soff: byte offset of the tile origin (row r0, k-tile kt), wave-uniform
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, bf16_t* lds, int soff, int wave) const {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_PTR(void))(lds + (wave + NW * i) * 512), 16, voff[i], soff,
                                               0, 0);
  }
};

struct WorkItem {
  int b, m0, n0, kt0, split;
};

// item order (split, batch, tile-row, tile-col) with the dimension of FEWER tiles fastest: with
// the XCD-aware deal an XCD's blocks then share one K-range (split) and cover a compact block
// of tiles -- all of the narrow operand's panels and a slice of the wide one's -- so its L2
// holds both (the FF weight gradient dW_in [640 x 2560] read every dA panel on every XCD with
// the tile-col-fastest order: 80 us vs 63 for the transposed dW_out)
__device__ __forceinline__ WorkItem decode_item(const GemmArgs& p, int item, int ntm, int ntn) {
  WorkItem w;
  int tm_i, tn_i, r;
  if (p.flags & kMFast) {
    tm_i = item % ntm;
    r = item / ntm;
    tn_i = r % ntn;
    r /= ntn;
  } else {
    tn_i = item % ntn;
    r = item / ntn;
    tm_i = r % ntm;
    r /= ntm;
  }
  w.b = r % p.batch;
  w.split = r / p.batch;
  w.m0 = tm_i;
  w.n0 = tn_i;
  w.kt0 = w.split * p.kt_per_split;
  return w;
}

constexpr int kSC1 = 16;  // buffer-instruction cache policy bit: sc1 (gfx940-family CPol::SC1)

// RES: epilogue operand R (bf16 output only; see apply_res8): 0 none, 1 bf16 R, 2 f32 R.  A
// template parameter so kernels without it keep their register allocation.
// (a 4-wave kernel whose LDS ring lets two blocks share a CU is told so: the pipelined main loop's
// second fragment set and the epilogue registers would otherwise push VGPR + AGPR past 256 and
// halve the resident blocks)
// (the body of gemm_dma_kernel; `bid` / `G` are the block's index and the grid as far as this
// GEMM is concerned -- a grouped launch, gemm_dma_group2_kernel, runs two GEMMs' items in one grid)
template <int BM, int BN, int WM, int WN, int NST, bool A_KC, bool B_KC, bool OUT_F32, int RES = 0>
__device__ __forceinline__ void gemm_dma_body(const GemmArgs& p, const int bid, const int G) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_TILE = BM * BK, B_TILE = BN * BK, STAGE = A_TILE + B_TILE;
  using TA = DmaTile<BM, A_KC, NW>;
  using TB = DmaTile<BN, B_KC, NW>;
  constexpr int L = TA::PER_WAVE + TB::PER_WAVE;   // vector-memory instructions per wave per K-tile
  // Operands swapped (C^T = B^T A^T per 16x16 block): each lane ends with 4 CONSECUTIVE
  // columns of one output row.  bf16 output: lanes pair up into 16-byte row chunks and leave
  // through exactly S_EPI buffer stores per lane (masked lanes get an out-of-range offset, so
  // the count is exact and the next K-step's counted vmcnt stays valid).  f32 output (split-K
  // slabs / atomics, weight grads): one 16-byte store (or 4 atomics) per block, full drain after.
  constexpr bool SWAP = true;
  static_assert(OUT_F32 || TN % 2 == 0, "column blocks pair up for 16-byte stores");
  constexpr int S_EPI = TM * TN / 2;
  static_assert(L * (NST - 1) + S_EPI + 1 <= 63, "vmcnt immediate range");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int items = p.batch * p.splitk * ntm * ntn;
  const int slot = xcd_remap(bid, G);   // same-XCD blocks take neighbouring items
  const int my_items = slot < items ? (items - slot + G - 1) / G : 0;
  const int nk = p.kt_per_split;               // K-tiles per item (the split divides them)
  const int total = my_items * nk;
#ifdef LJS_GEMM_TRACE
  unsigned long long* trc = p.trace ? p.trace + ((long)bid * NW + wave) * kTraceSlots : nullptr;
  int trn = 0;
  auto stamp = [&]() {
    if (trc && trn < kTraceSlots - 1) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) trc[trn] = t;
    }
    ++trn;
  };
  auto stamp_end = [&]() {
    if (trc) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) trc[kTraceSlots - 1] = t;
    }
  };
#else
  auto stamp = [&]() {};
  auto stamp_end = [&]() {};
#endif
  stamp();

  constexpr int AES = 2;  // A element bytes
  const long a_bytes = AES * (A_KC ? (long)(p.M - 1) * p.lda + p.K : (long)(p.K - 1) * p.lda + p.M);
  const long b_bytes = 2 * (B_KC ? (long)(p.N - 1) * p.ldb + p.K : (long)(p.K - 1) * p.ldb + p.N);
  const long a_kt = A_KC ? (long)BK * AES : (long)BK * p.lda * 2;  // bytes per K-tile step
  const long b_kt = B_KC ? (long)BK * 2 : (long)BK * p.ldb * 2;

  TA ta;
  TB tb;
  ta.init(p.lda, wave, lane);
  tb.init(p.ldb, wave, lane);

  // issue-side cursor: the item whose K-tiles are being fetched, advanced incrementally with
  // 32-bit scalar offsets (the launcher guarantees operand extents < 2^30 bytes)
  int is_item = 0, is_kt = 0;
  __amdgpu_buffer_rsrc_t ra, rb;
  int a_off = 0, b_off = 0;
  const int a_step = (int)a_kt, b_step = (int)b_kt;
  auto load_item = [&](int k) {
    const WorkItem w = decode_item(p, slot + G * k, ntm, ntn);
    ra = make_rsrc(reinterpret_cast<const unsigned char*>(p.A) + (long)w.b * p.sA * AES, a_bytes);
    rb = make_rsrc((p.flags & kBPtrs) ? p.bptr[w.b] : p.B + (long)w.b * p.sB, b_bytes);
    a_off = __builtin_amdgcn_readfirstlane(
        (int)((A_KC ? (long)w.m0 * BM * p.lda : (long)w.m0 * BM) * AES + w.kt0 * a_kt));
    b_off = __builtin_amdgcn_readfirstlane(
        (int)((B_KC ? (long)w.n0 * BN * p.ldb : (long)w.n0 * BN) * 2 + w.kt0 * b_kt));
  };
  auto issue_a = [&](int st) { ta.issue(ra, smem + st * STAGE, a_off, wave); };
  auto issue_b = [&](int st) { tb.issue(rb, smem + st * STAGE + A_TILE, b_off, wave); };
  auto issue_next = [&](int st) {
    if (is_kt == 0) load_item(is_item);
    issue_a(st);
    issue_b(st);
    a_off += a_step;
    b_off += b_step;
    if (++is_kt == nk) { is_kt = 0; ++is_item; }
  };
  // the same in two halves (A pieces, then B pieces + cursor advance)
  auto issue_half = [&](int st, bool second) {
    if (!second) {
      if (is_kt == 0) load_item(is_item);
      issue_a(st);
      a_off += a_step;
    } else {
      issue_b(st);
      b_off += b_step;
      if (++is_kt == nk) { is_kt = 0; ++is_item; }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < total) issue_next(s);

  // RES 3 (PLAIN): alpha 1, no bias / ReLU / fused sum -- a compile-time epilogue, so the kernel
  // carries one store loop with nothing but the pair exchange, the bf16 packing and the stores;
  // for f32 output: f32 split-K slabs only (no atomics, accumulate, bias, bf16 slabs)
  // RES 4 (BSUM): alpha 1, an f32 bias, no ReLU (the out-projection: bias + fused loss sum)
  constexpr bool PLAIN = RES == 3, BSUM = RES == 4, NOALPHA = PLAIN || BSUM;
  constexpr bool HAS_R = RES == 1 || RES == 2;
  const bool relu = !PLAIN && !BSUM && (p.flags & 1);
  const bool has_bias = BSUM || (!PLAIN && (p.flags & 2) && p.splitk == 1);
  const bool bias_f32 = BSUM || (p.flags & 4);
  const bool accumulate = !PLAIN && (p.flags & 8);
  // flags & 32: output stores with sc1, which drop the written lines from the XCD's L2 (plain
  // stores keep them) so the output stream does not evict the operand panels other blocks reuse
  const bool st_sc1 = p.flags & 32;
  const bool psum_on = !OUT_F32 && !PLAIN && p.psum != nullptr;
  float tsum = 0.f;
  const bool slabs = OUT_F32 && (PLAIN || (p.flags & kSlabs));  // (f32 PLAIN: slab mode only)
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(
      p.C, (OUT_F32 ? 4 : 2) *
               ((long)((slabs ? p.splitk * p.batch : p.batch) - 1) * p.sC + (long)(p.M - 1) * p.ldc + p.N));
  bool after_epi = false;

  // K-tile g landed in LDS for every wave, and every wave's fragment reads of tile g - 1
  // completed (so its stage may be refilled): this wave's pieces of g (the younger tiles' pieces
  // and, right after an epilogue, its S_EPI stores may stay in flight), then the barrier
  auto wait_landed = [&](int g) {
    stamp();
    const bool tail = g + NST - 2 >= total;
    if constexpr (NST >= 3) {
      if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (SWAP && after_epi && psum_on)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2) + S_EPI + 1) : "memory");
      else if (SWAP && after_epi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2) + S_EPI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2)) : "memory");
    } else {
      if (SWAP && after_epi && psum_on) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S_EPI + 1) : "memory");
      else if (SWAP && after_epi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S_EPI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    after_epi = false;
    stamp();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stamp();
  };
  // Software-pipelined by half a K-tile: the fragments of k-step 0 of tile g + 1 are read (and
  // tile g + 1's barrier passed) while the k-step 1 MFMAs of tile g are still to issue, so the
  // MFMA pipe never waits for a barrier plus an LDS round trip at a tile boundary (it did, once
  // per K-tile per wave).  ka/kb: k-step 0 fragments, la/lb: k-step 1.
  bf16x8 ka[TM], kb[TN], la[TM], lb[TN];
  auto read_frags = [&](int g, int ks, bf16x8* af, bf16x8* bfr) {
    const bf16_t* As_ = smem + (g % NST) * STAGE;
    const bf16_t* Bs_ = As_ + A_TILE;
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) af[ii] = frag<BM, A_KC>(As_, wr * (BM / WM) + ii * 16, ks, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag<BN, B_KC>(Bs_, wc * (BN / WN) + j * 16, ks, lane);
  };
  auto mfmas = [&](const bf16x8* af, const bf16x8* bfr) {
#pragma unroll
    for (int ii = 0; ii < TM; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (SWAP) acc[ii][j] = mfma16x16x32(bfr[j], af[ii], acc[ii][j]);  // C^T block
        else acc[ii][j] = mfma16x16x32(af[ii], bfr[j], acc[ii][j]);
      }
  };
  static_assert(BK == 64, "two k-steps per K-tile");
  // LJS_GEMM_PIN (off: neutral at B=64, +0.7 us on the 8-wave 128x128 QKV at B=8, gpurun_out/r4p):
  // the k-step 1 fragments (la / lb) are redefined through an empty asm right after
  // the k-step 0 MFMAs (a sched_barrier keeps it there).  The compiler then places its lgkmcnt
  // wait for them at that point, where their reads are long done, instead of in front of the
  // k-step 1 MFMAs -- where, with the next tile's fragment reads issued after the barrier still
  // in flight (and an SMEM load on the item-change path), it could only emit lgkmcnt(0) and so
  // exposed the new reads' LDS latency once per K-tile.
#ifndef LJS_GEMM_PIN
#define LJS_GEMM_PIN 0
#endif
  auto pin = [&](bf16x8* af, bf16x8* bfr) {
#if LJS_GEMM_PIN
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) asm volatile("" : "+v"(af[ii]));
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
#endif
  };
  // (wave tiles with more than 8 fragments per k-step -- 128x160's 32x160 -- keep the plain
  // loop: two fragment sets would not fit beside their epilogue registers; so do the
  // transposed-read weight-gradient kernels, 1-2 % slower pipelined while the k-contiguous
  // forward / dX kernels gain 3-4 %: QKV 2561 45.3 -> 43.7 us, 1282 48.1 -> 46.1 us)
  // (one 8-wave block per CU has 256 VGPRs per wave: 10 fragments fit twice beside 24 accumulators)
  // (one 4-wave block per CU -- the wide wave tiles 128x64 .. 128x128 -- has 512 registers per
  // wave: both fragment sets fit beside up to 256 accumulators)
  constexpr bool ONE_PER_CU = !(NW == 4 && NST * (BM + BN) * 64 * 2 <= 80 * 1024);
  constexpr bool PIPE = (TM + TN <= 8 || (NW == 8 && TM + TN <= 10) || (NW == 4 && ONE_PER_CU && TM + TN <= 16)) &&
                        A_KC && B_KC;   // (the last clause: 4-wave wide wave tiles, none instantiated since r5b)
  if (PIPE && total > 0) {
    wait_landed(0);
    read_frags(0, 0, ka, kb);
    if (NST - 1 < total) issue_next((NST - 1) % NST);
  }

  for (int it = 0, f = 0; it < my_items; ++it) {
  for (int kk = 0; kk < nk; ++kk, ++f) {
    if constexpr (!PIPE) {
      // barrier for tile f, then per k-step: fragment reads, half of tile f + NST - 1's DMA
      // pieces (their issue time overlaps the LDS latency), MFMAs
      wait_landed(f);
      const bool more = f + NST - 1 < total;
      const int nst = (f + NST - 1) % NST;
      read_frags(f, 0, ka, kb);
      if (more) issue_half(nst, false);
      mfmas(ka, kb);
      read_frags(f, 1, la, lb);
      if (more) issue_half(nst, true);
      mfmas(la, lb);
      continue;
    }
    read_frags(f, 1, la, lb);
    mfmas(ka, kb);
    pin(la, lb);
    // inside an item: DMA of tile f + NST into the stage of tile f (free once barrier f + 1 is
    // passed), issued in two halves around the k-step 1 MFMAs.  An item's last tile does this
    // after its epilogue instead (below), so no fragments are live across the epilogue.
    const bool inner = kk + 1 < nk;
    const bool more = inner && f + NST < total;
    if (inner) {
      wait_landed(f + 1);
      read_frags(f + 1, 0, ka, kb);
      if (more) issue_half(f % NST, false);
    }
    mfmas(la, lb);
    if (more) issue_half(f % NST, true);
  }

    // ------------------------------------------------------------ epilogue of this item
    const WorkItem w = decode_item(p, slot + G * it, ntm, ntn);
    const int m0 = w.m0 * BM + wr * (BM / WM), n0 = w.n0 * BN + wc * (BN / WN);
    const int g = lane >> 4;
    if constexpr (!OUT_F32) {
      // lane holds C[16 ii + (lane & 15)][16 j + 4 g + 0..3]; lanes g, g^1 trade halves so
      // even g owns cols 16 j0 + 4 g .. +7 and odd g owns 16 j1 + 4 (g - 1) .. +7
      const bool even = (g & 1) == 0;
      // epilogue operand: one row block (ii) of R chunks in flight at a time (all of an item's
      // chunks at once cost the second resident block its registers); rows / columns past
      // M / N read 0 through the buffer range check, and the compiler's counted vmcnt waits
      // for them at first use
      // (two row blocks in registers: block ii + 1's loads are issued before block ii is
      // processed, so only the first block's latency is exposed per item)
      u32x4 rv[2][TN / 2][RES == 2 ? 2 : 1];
      __amdgpu_buffer_rsrc_t rr;
      if constexpr (HAS_R)
        rr = make_rsrc(p.res, (RES == 2 ? 4 : 2) * ((long)(p.batch - 1) * p.sR + (long)(p.M - 1) * p.ldr + p.N));
      auto load_r = [&](int ii) {
        if constexpr (HAS_R) {
#pragma unroll
          for (int q = 0; q < TN / 2; ++q) {
            const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
            const int row = m0 + ii * 16 + (lane & 15);
            const bool ok = row < p.M && col < p.N;
            const int off = ok ? (int)(((long)w.b * p.sR + (long)row * p.ldr + col) * (RES == 2 ? 4 : 2)) : 0x7ffffff0;
            rv[ii & 1][q][0] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
            if constexpr (RES == 2)
              rv[ii & 1][q][RES == 2 ? 1 : 0] = __builtin_amdgcn_raw_buffer_load_b128(rr, ok ? off + 16 : off, 0, 0);
          }
        }
      };
      load_r(0);
      float bvs[TN / 2][8];
      // bias: this lane's 8 consecutive columns as one or two 16-byte loads (aligned bias rows;
      // N % 8 == 0 here) instead of 8 scalar loads of each width
      const bool bias_vec = has_bias && ((((uintptr_t)p.bias) & 15) == 0) && (p.sBias % 8) == 0;
#pragma unroll
      for (int q = 0; q < TN / 2; ++q) {
        const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
        const long bo = (long)w.b * p.sBias + col;
        if (bias_vec && col + 8 <= p.N) {
          if (bias_f32) {
            const f32x4 lo = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.bias) + bo);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.bias) + bo + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bvs[q][e] = lo[e];
              bvs[q][4 + e] = hi[e];
            }
          } else {
            const u32x4 u = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(p.bias) + bo);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bvs[q][2 * e] = __uint_as_float(u[e] << 16);
              bvs[q][2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
            }
          }
          continue;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bvs[q][e] = 0.f;
          if (has_bias && col + e < p.N) {
            bvs[q][e] = bias_f32 ? reinterpret_cast<const float*>(p.bias)[bo + e]
                                 : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[bo + e]);
          }
        }
      }
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) {
        if (ii + 1 < TM) load_r(ii + 1);
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {  // both halves of a row's 128 B back to back
          const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
          const float* bv = bvs[q];
          const f32x4 a0 = NOALPHA ? acc[ii][2 * q] : acc[ii][2 * q] * p.alpha;
          const f32x4 a1 = NOALPHA ? acc[ii][2 * q + 1] : acc[ii][2 * q + 1] * p.alpha;
          acc[ii][2 * q] = f32x4{0.f, 0.f, 0.f, 0.f};
          acc[ii][2 * q + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
          float v[8];
          pair_rows16(a0, a1, even, v);
          u32x4 pk;
          if constexpr (!PLAIN) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              v[e] += bv[e];
              if (relu) v[e] = fmaxf(v[e], 0.f);
            }
          }
          if constexpr (HAS_R) apply_res8(v, p.flags, rv[ii & 1][q][0], rv[ii & 1][q][0], rv[ii & 1][q][RES == 2 ? 1 : 0]);
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
          const int row = m0 + ii * 16 + (lane & 15);
          const bool ok = row < p.M && col < p.N;  // N % 8 == 0 (launcher): chunks are whole
          const int off = ok ? (int)(((long)w.b * p.sC + (long)row * p.ldc + col) * 2) : 0x7ffffff0;
          if (st_sc1) __builtin_amdgcn_raw_buffer_store_b128(pk, rc, off, 0, kSC1);
          else __builtin_amdgcn_raw_buffer_store_b128(pk, rc, off, 0, 0);
          if (psum_on && ok) {
#pragma unroll
            for (int e = 0; e < 4; ++e) tsum += __uint_as_float(pk[e] << 16) + __uint_as_float(pk[e] & 0xffff0000u);
          }
        }
      }
      if (psum_on) {
        // fused loss reduction: this wave's share of sum(C) -- of the bf16 values just stored --
        // to its own slot (one store per wave, counted in the next K-step's vmcnt)
        tsum = warp_sum64(tsum);
        if (lane == 0) p.psum[(long)(slot + G * it) * NW + wave] = tsum;
        tsum = 0.f;
      }
      after_epi = true;
    } else {
      // lane holds C[16 ii + (lane & 15)][16 j + 4 g + 0..3]
      const bool vec = (p.ldc & 3) == 0 && (p.sC & 3) == 0 && ((((uintptr_t)p.C) & 15) == 0);
      if constexpr (BN / WN == 64 && WM * WN * (BM / WM) * 256 <= NST * STAGE * 2) {
        if (slabs && vec && (p.flags & kSlabVst) && it + 1 == my_items && !has_bias && !relu && !accumulate) {
          // no DMA is in flight after the block's last item: once every wave's last fragment reads
          // are done the ring holds this wave's 64-column f32 rows (wave-private image)
          __syncthreads();
          unsigned char* img = reinterpret_cast<unsigned char*>(smem) + wave * (BM / WM) * 256;
#pragma unroll
          for (int ii = 0; ii < TM; ++ii) {
            const int r = ii * 16 + (lane & 15);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              *reinterpret_cast<f32x4*>(img + r * 256 + (((4 * j + g) ^ (r & 7)) << 4)) = PLAIN ? acc[ii][j] : acc[ii][j] * p.alpha;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const long cb = (long)(w.split * p.batch + w.b) * p.sC;
#pragma unroll
          for (int q = 0; q < (BM / WM) / 4; ++q) {
            const int r = 4 * q + (lane >> 4), c = lane & 15;
            const f32x4 v = *reinterpret_cast<const f32x4*>(img + r * 256 + ((c ^ (r & 7)) << 4));
            const int row = m0 + r, col = n0 + 4 * c;
            if (row < p.M && col + 4 <= p.N) {
              const u32x4 bits = __builtin_bit_cast(u32x4, v);
              __builtin_amdgcn_raw_buffer_store_b128(bits, rc, (int)((cb + (long)row * p.ldc + col) * 4), 0, 0);
            } else if (row < p.M) {
              float* C = reinterpret_cast<float*>(p.C) + cb + (long)row * p.ldc + col;
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (col + e < p.N) C[e] = v[e];
            }
          }
          continue;  // the block's last item: nothing follows
        }
      }
      // this item's output block (slab mode: slab (split, batch b) = split * batch + b, so the
      // slabs of a batch of weight gradients are [S][batch][M][N]: one slab_reduce combines all)
      const long cb = (long)(slabs ? w.split * p.batch + w.b : w.b) * p.sC;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + j * 16 + 4 * g;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (has_bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (col + e >= p.N) continue;
            const long bo = (long)w.b * p.sBias + col + e;
            bv[e] = bias_f32 ? reinterpret_cast<const float*>(p.bias)[bo]
                             : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[bo]);
          }
        }
#pragma unroll
        for (int ii = 0; ii < TM; ++ii) {
          const int row = m0 + ii * 16 + (lane & 15);
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = PLAIN ? acc[ii][j][e] : acc[ii][j][e] * p.alpha + bv[e];
            if (relu) v[e] = fmaxf(v[e], 0.f);
          }
          acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (row >= p.M || col >= p.N) continue;
          float* C = reinterpret_cast<float*>(p.C) + cb + (long)row * p.ldc + col;
          if (p.splitk > 1 && !slabs) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (col + e < p.N) atomicAdd(C + e, v[e]);
          } else if (vec && col + 4 <= p.N) {
            if (accumulate) v += *reinterpret_cast<const f32x4*>(C);
            const int off = (int)((cb + (long)row * p.ldc + col) * 4);
            const u32x4 bits = __builtin_bit_cast(u32x4, v);
            if (st_sc1) __builtin_amdgcn_raw_buffer_store_b128(bits, rc, off, 0, kSC1);
            else __builtin_amdgcn_raw_buffer_store_b128(bits, rc, off, 0, 0);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (col + e < p.N) C[e] = accumulate ? C[e] + v[e] : v[e];
          }
        }
      }
      // drain before the next item's counted waits; after the block's last item the wave just
      // ends (its stores complete on their own and the CU is free for the next block sooner)
      if (it + 1 < my_items) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // the next item's first tile (f): its barrier, k-step 0 fragments and the DMA of tile
    // f + NST - 1 (the stage of tile f - 1, read by every wave before this barrier)
    if (PIPE && f < total) {
      wait_landed(f);
      read_frags(f, 0, ka, kb);
      if (f + NST - 1 < total) issue_next((f + NST - 1) % NST);
    }
  }
  stamp_end();
}

template <int BM, int BN, int WM, int WN, int NST, bool A_KC, bool B_KC, bool OUT_F32, int RES = 0>
__global__ __launch_bounds__(WM * WN * 64, (WM * WN == 4 && NST * (BM + BN) * 64 * 2 <= 80 * 1024) ? 2 : 1) void
gemm_dma_kernel(GemmArgs p) {
  gemm_dma_body<BM, BN, WM, WN, NST, A_KC, B_KC, OUT_F32, RES>(p, blockIdx.x, gridDim.x);
}

// Two GEMMs of the same kernel instance in ONE grid, one block per work item: blocks [0, g0) take
// p0's items, the rest p1's.  The weight-gradient GEMMs of a layer at the reference shape (dW_qkv
// and dW_o, 240 short items each) are latency-bound launches; grouped they share one round of
// resident blocks instead of running back to back (ops/linear.py dW grouping).
template <int BM, int BN, int WM, int WN, int NST, bool A_KC, bool B_KC, bool OUT_F32, int RES = 0>
__global__ __launch_bounds__(WM * WN * 64, (WM * WN == 4 && NST * (BM + BN) * 64 * 2 <= 80 * 1024) ? 2 : 1) void
gemm_dma_group2_kernel(GemmArgs p0, GemmArgs p1, int g0) {
  if ((int)blockIdx.x < g0)
    gemm_dma_body<BM, BN, WM, WN, NST, A_KC, B_KC, OUT_F32, RES>(p0, blockIdx.x, g0);
  else
    gemm_dma_body<BM, BN, WM, WN, NST, A_KC, B_KC, OUT_F32, RES>(p1, blockIdx.x - g0, gridDim.x - g0);
}

// ============================================================================ lean K-loop GEMM
// The persistent LDS-DMA GEMM's k-contiguous, bf16-output path (forward projections and dX GEMMs)
// with the per-K-tile bookkeeping out of the K-loop.  A DMA / MFMA / barrier probe
// (scripts/probe_dma_mfma.hip, profiles/r5_probe_dma_mfma.txt) measured what a K-tile of this
// structure costs per SIMD: 32 MFMAs per wave alone 1180 cycles; + 6 DMA pieces and 16 fragment
// reads + one barrier 1440; + ~90 scalar instructions and 6 branches per K-tile 1850 -- and the
// general kernel above carries about that much (stage index = tile mod NST through mul_hi, the
// tail / after-epilogue / next-item tests and their vmcnt selection, all inside the loop).  Here:
//  * the stage is a rotating offset (the DMA of tile f + NST goes to tile f's stage);
//  * the K-loop of an item runs nk - 1 identical steps (one counted vmcnt, one barrier, half
//    the next tile's pieces after its k-step-0 fragment reads, half after the k-step-1 MFMAs); the
//    item's last K-tile, its epilogue and the next item's first barrier are peeled;
//  * the issue cursor never tests for the end: past the block's last item it issues K-tiles that
//    read zeros (an empty-range descriptor) into stages nothing reads again, so every step's count is the same.
// Operands, images, fragment reads, MFMA orientation and the epilogue are gemm_dma_kernel's
// (bit-identical results: tests/test_kernels_gpu.py::test_gemm_lean_bit_exact).
// The issue cursor's K-tiles past the block's last item go through a buffer descriptor with an
// empty range: every lane is out of range whatever its offsets, so the pieces read zeros without a
// memory access and retire at once (the block's final vmcnt(0) does not wait for an L2 round trip).
template <int BM, int BN, int WM, int WN, int NST, int RES>
__global__ __launch_bounds__(WM * WN * 64, (WM * WN == 4 && NST * (BM + BN) * 64 * 2 <= 80 * 1024) ? 2 : 1) void
gemm_lean_kernel(GemmArgs p) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_TILE = BM * BK, B_TILE = BN * BK, STAGE = A_TILE + B_TILE;
  using TA = DmaTile<BM, true, NW>;
  using TB = DmaTile<BN, true, NW>;
  constexpr int L = TA::PER_WAVE + TB::PER_WAVE;
  static_assert(TN % 2 == 0, "column blocks pair up for 16-byte stores");
  static_assert(NST >= 2, "at least one K-tile in flight");
  constexpr int S_EPI = TM * TN / 2;
  static_assert(L * (NST - 1) + S_EPI + 1 <= 63, "vmcnt immediate range");
  constexpr bool PLAIN = RES == 3, BSUM = RES == 4, NOALPHA = PLAIN || BSUM;
  constexpr bool HAS_R = RES == 1 || RES == 2;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int items = p.batch * ntm * ntn;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  const int my_items = slot < items ? (items - slot + G - 1) / G : 0;
  if (my_items == 0) return;
  const int nk = p.kt_per_split;   // K / 64 (no split-K on this path)

  const long a_bytes = 2 * ((long)(p.M - 1) * p.lda + p.K);
  const long b_bytes = 2 * ((long)(p.N - 1) * p.ldb + p.K);
  TA ta;
  TB tb;
  ta.init(p.lda, wave, lane);
  tb.init(p.ldb, wave, lane);

  // ---- issue cursor: the item whose K-tiles are being fetched (NST K-tiles ahead of the MFMAs)
  int is_item = 0, is_kt = 0;
  __amdgpu_buffer_rsrc_t ra, rb;
  int a_off = 0, b_off = 0;
  auto load_item = [&](int k) {
    const WorkItem w = decode_item(p, slot + G * (k < my_items ? k : 0), ntm, ntn);
    ra = make_rsrc(p.A + (long)w.b * p.sA, a_bytes);
    rb = make_rsrc(p.B + (long)w.b * p.sB, b_bytes);
    a_off = __builtin_amdgcn_readfirstlane((int)((long)w.m0 * BM * p.lda * 2));
    b_off = __builtin_amdgcn_readfirstlane((int)((long)w.n0 * BN * p.ldb * 2));
    if (k >= my_items) {   // past the block's last item: an empty range (every piece reads zeros)
      ra = make_rsrc(p.A, 0);
      rb = make_rsrc(p.B, 0);
    }
  };
  auto issue_a = [&](int so) { ta.issue(ra, smem + so, a_off, wave); };
  auto issue_b = [&](int so) { tb.issue(rb, smem + so + A_TILE, b_off, wave); };
  auto advance = [&]() {
    a_off += BK * 2;
    b_off += BK * 2;
    if (++is_kt == nk) {
      is_kt = 0;
      load_item(++is_item);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_item(0);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    issue_a(s * STAGE);
    issue_b(s * STAGE);
    advance();
  }

  const bool relu = !PLAIN && !BSUM && (p.flags & 1);
  const bool has_bias = BSUM || (!PLAIN && (p.flags & 2));
  const bool bias_f32 = BSUM || (p.flags & 4);
  const bool st_sc1 = p.flags & 32;
  const bool psum_on = !PLAIN && p.psum != nullptr;
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(p.C, 2 * ((long)(p.batch - 1) * p.sC + (long)(p.M - 1) * p.ldc + p.N));

  bf16x8 ka[TM], kb[TN], la[TM], lb[TN];
  auto read_frags = [&](int so, int ks, bf16x8* af, bf16x8* bfr) {
    const bf16_t* As_ = smem + so;
    const bf16_t* Bs_ = As_ + A_TILE;
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) af[ii] = frag<BM, true>(As_, wr * (BM / WM) + ii * 16, ks, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag<BN, true>(Bs_, wc * (BN / WN) + j * 16, ks, lane);
  };
  auto mfmas = [&](const bf16x8* af, const bf16x8* bfr) {
#pragma unroll
    for (int ii = 0; ii < TM; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[ii][j] = mfma16x16x32(bfr[j], af[ii], acc[ii][j]);  // C^T block
  };
  auto next_so = [](int so) { return so + STAGE == NST * STAGE ? 0 : so + STAGE; };
  auto barrier = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  // the stage of the (virtual) tile before the block's first: the first item start issues the
  // DMA of tile NST - 1 into it
  int so = (NST - 1) * STAGE;
  // item start: tile f = the item's first (stage nso) landed -- this wave's pieces of the younger
  // tiles and, after an epilogue, its S_EPI (+1 fused-sum) stores may stay in flight -- then the
  // barrier, k-step 0 fragments, and the DMA of tile f + NST - 1 into the stage of tile f - 1
  auto item_start = [&](bool after_epi) {
    if (!after_epi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2)) : "memory");
    else if (psum_on) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2) + S_EPI + 1) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2) + S_EPI) : "memory");
    barrier();
    const int nso = next_so(so);
    read_frags(nso, 0, ka, kb);
    issue_a(so);
    issue_b(so);
    advance();
    so = nso;
  };
  item_start(false);

  float tsum = 0.f;
  for (int it = 0; it < my_items; ++it) {
    for (int kk = 0; kk + 1 < nk; ++kk) {
      read_frags(so, 1, la, lb);
      mfmas(ka, kb);
      const int nso = next_so(so);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NST - 2)) : "memory");  // tile f + 1 landed
      barrier();                                   // ... for every wave; every read of tile f done
      read_frags(nso, 0, ka, kb);
      issue_a(so);                                 // tile f + NST into tile f's stage
      mfmas(la, lb);
      issue_b(so);
      advance();
      so = nso;
    }
    // the item's last K-tile
    read_frags(so, 1, la, lb);
    mfmas(ka, kb);
    mfmas(la, lb);

    // ------------------------------------------------------------ epilogue of this item
    const WorkItem w = decode_item(p, slot + G * it, ntm, ntn);
    const int m0 = w.m0 * BM + wr * (BM / WM), n0 = w.n0 * BN + wc * (BN / WN);
    const int g = lane >> 4;
    const bool even = (g & 1) == 0;
    u32x4 rv[2][TN / 2][RES == 2 ? 2 : 1];
    __amdgpu_buffer_rsrc_t rr;
    if constexpr (HAS_R)
      rr = make_rsrc(p.res, (RES == 2 ? 4 : 2) * ((long)(p.batch - 1) * p.sR + (long)(p.M - 1) * p.ldr + p.N));
    auto load_r = [&](int ii) {
      if constexpr (HAS_R) {
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
          const int row = m0 + ii * 16 + (lane & 15);
          const bool ok = row < p.M && col < p.N;
          const int off = ok ? (int)(((long)w.b * p.sR + (long)row * p.ldr + col) * (RES == 2 ? 4 : 2)) : 0x7ffffff0;
          rv[ii & 1][q][0] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
          if constexpr (RES == 2)
            rv[ii & 1][q][RES == 2 ? 1 : 0] = __builtin_amdgcn_raw_buffer_load_b128(rr, ok ? off + 16 : off, 0, 0);
        }
      }
    };
    load_r(0);
    float bvs[TN / 2][8];
    const bool bias_vec = has_bias && ((((uintptr_t)p.bias) & 15) == 0) && (p.sBias % 8) == 0;
#pragma unroll
    for (int q = 0; q < TN / 2; ++q) {
      const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
      const long bo = (long)w.b * p.sBias + col;
      if (bias_vec && col + 8 <= p.N) {
        if (bias_f32) {
          const f32x4 lo = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.bias) + bo);
          const f32x4 hi = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.bias) + bo + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bvs[q][e] = lo[e];
            bvs[q][4 + e] = hi[e];
          }
        } else {
          const u32x4 u = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(p.bias) + bo);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bvs[q][2 * e] = __uint_as_float(u[e] << 16);
            bvs[q][2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
          }
        }
        continue;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bvs[q][e] = 0.f;
        if (has_bias && col + e < p.N) {
          bvs[q][e] = bias_f32 ? reinterpret_cast<const float*>(p.bias)[bo + e]
                               : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[bo + e]);
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) {
      if (ii + 1 < TM) load_r(ii + 1);
#pragma unroll
      for (int q = 0; q < TN / 2; ++q) {
        const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
        const float* bv = bvs[q];
        const f32x4 a0 = NOALPHA ? acc[ii][2 * q] : acc[ii][2 * q] * p.alpha;
        const f32x4 a1 = NOALPHA ? acc[ii][2 * q + 1] : acc[ii][2 * q + 1] * p.alpha;
        acc[ii][2 * q] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[ii][2 * q + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
        float v[8];
        pair_rows16(a0, a1, even, v);
        u32x4 pk;
        if constexpr (!PLAIN) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            v[e] += bv[e];
            if (relu) v[e] = fmaxf(v[e], 0.f);
          }
        }
        if constexpr (HAS_R) apply_res8(v, p.flags, rv[ii & 1][q][0], rv[ii & 1][q][0], rv[ii & 1][q][RES == 2 ? 1 : 0]);
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
        const int row = m0 + ii * 16 + (lane & 15);
        const bool ok = row < p.M && col < p.N;  // N % 8 == 0 (launcher): chunks are whole
        const int off = ok ? (int)(((long)w.b * p.sC + (long)row * p.ldc + col) * 2) : 0x7ffffff0;
        if (st_sc1) __builtin_amdgcn_raw_buffer_store_b128(pk, rc, off, 0, kSC1);
        else __builtin_amdgcn_raw_buffer_store_b128(pk, rc, off, 0, 0);
        if (psum_on && ok) {
#pragma unroll
          for (int e = 0; e < 4; ++e) tsum += __uint_as_float(pk[e] << 16) + __uint_as_float(pk[e] & 0xffff0000u);
        }
      }
    }
    if (psum_on) {
      tsum = warp_sum64(tsum);
      if (lane == 0) p.psum[(long)(slot + G * it) * NW + wave] = tsum;
      tsum = 0.f;
    }
    if (it + 1 < my_items) item_start(true);
  }
  // the DMA pieces still in flight (the cursor's past-the-end tiles) write this block's LDS: let
  // them finish before the block's LDS can be handed to another
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// explicit instantiations: hipcc (ROCm 7.2) otherwise leaves some of these kernels' host stubs
// undefined when they are only named inside launch_dma's instantiations
#define LJS_DMA_INST(BM, BN, WM, WN, NST, AK, BKc, OF) \
  template __global__ void gemm_dma_kernel<BM, BN, WM, WN, NST, AK, BKc, OF>(GemmArgs);
#define LJS_DMA_INST_LAYOUTS(NST)                                                                           \
  LJS_DMA_INST(128, 128, 2, 2, NST, true, true, false) LJS_DMA_INST(128, 128, 2, 2, NST, true, true, true)     \
  LJS_DMA_INST(128, 128, 2, 2, NST, false, false, false) LJS_DMA_INST(128, 128, 2, 2, NST, false, false, true) \
  LJS_DMA_INST(128, 128, 2, 2, NST, true, false, false) LJS_DMA_INST(128, 128, 2, 2, NST, true, false, true)   \
  LJS_DMA_INST(128, 128, 2, 2, NST, false, true, false) LJS_DMA_INST(128, 128, 2, 2, NST, false, true, true)
LJS_DMA_INST_LAYOUTS(2)
LJS_DMA_INST_LAYOUTS(4)
// f32 split-K slab kernels with the compile-time plain epilogue (weight gradients: m/n-contiguous)
template __global__ void gemm_dma_kernel<128, 128, 2, 2, 2, false, false, true, 3>(GemmArgs);
template __global__ void gemm_dma_group2_kernel<128, 128, 2, 2, 2, false, false, true, 3>(GemmArgs, GemmArgs, int);
template __global__ void gemm_dma_group2_kernel<128, 128, 2, 4, 4, false, false, true, 3>(GemmArgs, GemmArgs, int);
template __global__ void gemm_dma_group2_kernel<128, 128, 2, 4, 3, false, false, true, 3>(GemmArgs, GemmArgs, int);
template __global__ void gemm_dma_kernel<128, 128, 2, 4, 4, false, false, true, 3>(GemmArgs);
template __global__ void gemm_dma_kernel<128, 128, 2, 4, 3, false, false, true, 3>(GemmArgs);
// 64x64 tiles (4 waves of 32x32, 3 or 4 stages): the small-M GEMMs of the reference shape
// (2048 tokens), where 128x128 tiles leave most CUs idle
#define LJS_DMA_INST_64(NST)                                                                               \
  LJS_DMA_INST(64, 64, 2, 2, NST, true, true, false) LJS_DMA_INST(64, 64, 2, 2, NST, true, true, true)     \
  LJS_DMA_INST(64, 64, 2, 2, NST, false, false, false) LJS_DMA_INST(64, 64, 2, 2, NST, false, false, true) \
  LJS_DMA_INST(64, 64, 2, 2, NST, true, false, false) LJS_DMA_INST(64, 64, 2, 2, NST, true, false, true)   \
  LJS_DMA_INST(64, 64, 2, 2, NST, false, true, false) LJS_DMA_INST(64, 64, 2, 2, NST, false, true, true)
LJS_DMA_INST_64(3)
LJS_DMA_INST_64(4)
#undef LJS_DMA_INST_64
LJS_DMA_INST(256, 128, 4, 2, 3, true, true, false)
LJS_DMA_INST(256, 128, 4, 2, 3, true, true, true)
// 256x192, 8 waves of 64x96, 2 stages (112 KiB): 7 DMA pieces and 20 fragment reads per wave per
// 48 MFMAs (256x128: 6 and 16 per 32); [T][1536] outputs are 2 items per block
LJS_DMA_INST(256, 192, 4, 2, 2, true, true, false)
// weight gradients (m/n-contiguous operands, f32 slabs): 256-wide tiles, 8 waves, 3 stages, one
// block per CU -- 48 KiB of operands per 64-deep K-tile for twice the MFMA work of 128x128
LJS_DMA_INST(256, 128, 4, 2, 3, false, false, true)
LJS_DMA_INST(128, 256, 2, 4, 3, false, false, true)
// 128x160 with 4 waves stacked along M (32x160 each): N = 640 splits into 4 column tiles, so a
// [16384, 640] output is exactly 512 items = one round of 2 blocks/CU (128x128: 640 items, 1.25)
LJS_DMA_INST(128, 160, 4, 1, 2, true, true, false)
// 128x128 with 8 waves (2 x 4, 64x32 each): two waves per SIMD at one block per CU, so a
// deep (3-4 stage) ring does not cost MFMA/LDS overlap
#define LJS_DMA_INST_8W(NST)                                                                                \
  LJS_DMA_INST(128, 128, 2, 4, NST, false, false, true) LJS_DMA_INST(128, 128, 2, 4, NST, true, true, false) \
  LJS_DMA_INST(128, 128, 2, 4, NST, true, true, true)
LJS_DMA_INST_8W(3)
LJS_DMA_INST_8W(4)
#undef LJS_DMA_INST_8W
// epilogue-operand variants (bf16 output, k-contiguous operands: forward and dX GEMMs)
#define LJS_DMA_INST_RES(BM, BN, WM, WN, NST) \
  template __global__ void gemm_dma_kernel<BM, BN, WM, WN, NST, true, true, false, 1>(GemmArgs); \
  template __global__ void gemm_dma_kernel<BM, BN, WM, WN, NST, true, true, false, 2>(GemmArgs); \
  template __global__ void gemm_dma_kernel<BM, BN, WM, WN, NST, true, true, false, 3>(GemmArgs); \
  template __global__ void gemm_dma_kernel<BM, BN, WM, WN, NST, true, true, false, 4>(GemmArgs);
LJS_DMA_INST_RES(128, 160, 4, 1, 2)
LJS_DMA_INST_RES(256, 192, 4, 2, 2)
LJS_DMA_INST_RES(64, 64, 2, 2, 4)
LJS_DMA_INST_RES(256, 128, 4, 2, 3)
LJS_DMA_INST_RES(128, 128, 2, 2, 2)
LJS_DMA_INST_RES(128, 128, 2, 2, 4)
LJS_DMA_INST_RES(128, 128, 2, 4, 3)
LJS_DMA_INST_RES(128, 128, 2, 4, 4)
#undef LJS_DMA_INST_RES
// lean K-loop kernels (k-contiguous, bf16 output; every epilogue instance)
#define LJS_LEAN_INST(BM, BN, WM, WN, NST)                                  \
  template __global__ void gemm_lean_kernel<BM, BN, WM, WN, NST, 0>(GemmArgs); \
  template __global__ void gemm_lean_kernel<BM, BN, WM, WN, NST, 1>(GemmArgs); \
  template __global__ void gemm_lean_kernel<BM, BN, WM, WN, NST, 2>(GemmArgs); \
  template __global__ void gemm_lean_kernel<BM, BN, WM, WN, NST, 3>(GemmArgs); \
  template __global__ void gemm_lean_kernel<BM, BN, WM, WN, NST, 4>(GemmArgs);
LJS_LEAN_INST(256, 128, 4, 2, 3)
LJS_LEAN_INST(256, 192, 4, 2, 2)
LJS_LEAN_INST(128, 160, 4, 1, 2)
LJS_LEAN_INST(128, 128, 2, 2, 2)
LJS_LEAN_INST(128, 128, 2, 2, 4)
LJS_LEAN_INST(128, 128, 2, 4, 3)
LJS_LEAN_INST(128, 128, 2, 4, 4)
LJS_LEAN_INST(64, 64, 2, 2, 4)
#undef LJS_LEAN_INST
#undef LJS_DMA_INST_LAYOUTS
#undef LJS_DMA_INST

int g_cus = 0;
unsigned long long* g_gemm_trace = nullptr;  // LJS_GEMM_TRACE builds: the next LDS-DMA launches' stamps

template <int BM, int BN, int WM, int WN, int NST, bool AK, bool BKc, bool OF, int RES = 0>
hipError_t launch_dma(const GemmArgs& a, hipStream_t s, int blocks_per_cu) {
  if (!g_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  const int items = ntm * ntn * a.batch * a.splitk;
  GemmArgs a2 = a;
  a2.trace = g_gemm_trace;
  if (ntm < ntn) a2.flags |= kMFast;   // narrow dimension fastest: tiles sharing a panel run together
  // blocks_per_cu 0 = one block per work item (measured best at the bench shapes: the
  // dispatcher balances), else a persistent grid of blocks_per_cu x CUs
  int bpc = blocks_per_cu;
  // Persistent grid when the items fill whole rounds of the resident slots: each block then
  // walks `rounds` items with the next item's first K-tiles in flight during the current
  // item's epilogue (measured at T = 16384: QKV projection 43.8 -> 39.9 us on 128x128 x 2/CU).
  // Otherwise one block per item, which lets the dispatcher balance a ragged last round.
  constexpr int kLdsBytes = NST * (BM + BN) * BK * 2;
  constexpr int kNatural = (WM * WN == 4 && kLdsBytes <= 80 * 1024) ? 2 : 1;  // resident blocks / CU
  if (bpc == 0 && items > g_cus * kNatural && items % (g_cus * kNatural) == 0) bpc = kNatural;
  int grid = bpc > 0 ? g_cus * bpc : items;
  if (grid > items) grid = items;
  hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, NST, AK, BKc, OF, RES>), dim3(grid), dim3(WM * WN * 64), 0,
                     s, a2);
  return hipGetLastError();
}

// bf16-output k-contiguous launch with the epilogue operand variant the flags ask for
template <int BM, int BN, int WM, int WN, int NST>
hipError_t launch_dma_kk(const GemmArgs& a, hipStream_t s) {
  if (a.flags & (kResAdd | kResMask)) {
    if (a.flags & kResF32) return launch_dma<BM, BN, WM, WN, NST, true, true, false, 2>(a, s, 0);
    return launch_dma<BM, BN, WM, WN, NST, true, true, false, 1>(a, s, 0);
  }
  // plain epilogue (RES 3: compile-time instance, PERF_NOTES r4 "plain instance")
  if (a.alpha == 1.f && !(a.flags & 3) && !a.psum)
    return launch_dma<BM, BN, WM, WN, NST, true, true, false, 3>(a, s, 0);
  // bias (f32) + optional fused sum, alpha 1, no ReLU (RES 4)
  if (a.alpha == 1.f && (a.flags & 7) == 6 && a.splitk == 1)
    return launch_dma<BM, BN, WM, WN, NST, true, true, false, 4>(a, s, 0);
  return launch_dma<BM, BN, WM, WN, NST, true, true, false, 0>(a, s, 0);
}

// Grouped weight-gradient launches (ljs_gemm_group_begin / _end): while a group is open, plain f32
// slab GEMMs are recorded instead of launched; closing it launches two recorded GEMMs of the same
// kernel instance as ONE grid (gemm_dma_group2_kernel, one block per work item) and anything else
// one by one.  Same kernel body per item: bit-identical to separate launches.
struct GroupRec {
  GemmArgs a;
  int kind;   // 1: 128x128 2x2 waves 2 stages, 2: 128x128 2x4 4 stages, 3: 128x128 2x4 3 stages
};
// (per host thread: another thread's GEMMs are never recorded into this thread's open group)
static thread_local bool g_group_on = false;
static thread_local GroupRec g_group[2];
static thread_local int g_group_n = 0;

template <int BM, int BN>
GemmArgs group_prep(const GemmArgs& a, int* items) {
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  *items = ntm * ntn * a.batch * a.splitk;
  GemmArgs a2 = a;
  a2.trace = nullptr;
  if (ntm < ntn) a2.flags |= kMFast;
  return a2;
}

// weight-gradient (m/n-contiguous, f32 output) launch: the plain split-K slab instance (RES 3)
// when the slabs are f32 and nothing else is asked for
template <int BM, int BN, int WM, int WN, int NST>
hipError_t launch_slab(const GemmArgs& a, hipStream_t s) {
  if ((a.flags & kSlabs) && !(a.flags & (1 | 2 | 8 | 16)) && a.alpha == 1.f) {
    constexpr int kind = (BM == 128 && BN == 128 && WM == 2 && WN == 2 && NST == 2)   ? 1
                         : (BM == 128 && BN == 128 && WM == 2 && WN == 4 && NST == 4) ? 2
                         : (BM == 128 && BN == 128 && WM == 2 && WN == 4 && NST == 3) ? 3
                                                                                      : 0;
    if (kind && g_group_on && g_group_n < 2) {
      g_group[g_group_n].a = a;
      g_group[g_group_n].kind = kind;
      ++g_group_n;
      return hipSuccess;
    }
    return launch_dma<BM, BN, WM, WN, NST, false, false, true, 3>(a, s, 0);
  }
  return launch_dma<BM, BN, WM, WN, NST, false, false, true, 0>(a, s, 0);
}

template <int WN, int NST>
hipError_t launch_group_kind(const GroupRec* r, int n, hipStream_t s) {
  if (n == 2) {
    int i0 = 0, i1 = 0;
    const GemmArgs a0 = group_prep<128, 128>(r[0].a, &i0), a1 = group_prep<128, 128>(r[1].a, &i1);
    hipLaunchKernelGGL((gemm_dma_group2_kernel<128, 128, 2, WN, NST, false, false, true, 3>), dim3(i0 + i1),
                       dim3(2 * WN * 64), 0, s, a0, a1, i0);
    return hipGetLastError();
  }
  return launch_dma<128, 128, 2, WN, NST, false, false, true, 3>(r[0].a, s, 0);
}

hipError_t launch_rec(const GroupRec* r, int n, hipStream_t s) {
  if (r[0].kind == 1) return launch_group_kind<2, 2>(r, n, s);
  if (r[0].kind == 2) return launch_group_kind<4, 4>(r, n, s);
  return launch_group_kind<4, 3>(r, n, s);
}

// the lean K-loop kernel (k-contiguous, bf16 output, no split): same grid choice as launch_dma
template <int BM, int BN, int WM, int WN, int NST, int RES>
hipError_t launch_lean(const GemmArgs& a, hipStream_t s) {
  if (!g_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  const int items = ntm * ntn * a.batch;
  GemmArgs a2 = a;
  if (ntm < ntn) a2.flags |= kMFast;
  constexpr int kLdsBytes = NST * (BM + BN) * BK * 2;
  constexpr int kNatural = (WM * WN == 4 && kLdsBytes <= 80 * 1024) ? 2 : 1;
  int grid = items;
  if (items > g_cus * kNatural && items % (g_cus * kNatural) == 0) grid = g_cus * kNatural;
  hipLaunchKernelGGL((gemm_lean_kernel<BM, BN, WM, WN, NST, RES>), dim3(grid), dim3(WM * WN * 64), 0, s, a2);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int NST>
hipError_t launch_lean_kk(const GemmArgs& a, hipStream_t s) {
  if (a.flags & (kResAdd | kResMask)) {
    if (a.flags & kResF32) return launch_lean<BM, BN, WM, WN, NST, 2>(a, s);
    return launch_lean<BM, BN, WM, WN, NST, 1>(a, s);
  }
  if (a.alpha == 1.f && !(a.flags & 3) && !a.psum) return launch_lean<BM, BN, WM, WN, NST, 3>(a, s);
  if (a.alpha == 1.f && (a.flags & 7) == 6) return launch_lean<BM, BN, WM, WN, NST, 4>(a, s);
  return launch_lean<BM, BN, WM, WN, NST, 0>(a, s);
}

template <int BM, int BN, bool AK, bool BKc, bool OF>
hipError_t launch_t(const GemmArgs& a, hipStream_t s) {
  int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, a.batch * a.splitk);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, AK, BKc, OF>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int BM, int BN>
hipError_t dispatch_layout(const GemmArgs& a, int a_kc, int b_kc, int out_f32, hipStream_t s) {
#define LJS_CASE(AK, BK_, OF) \
  if (a_kc == AK && b_kc == BK_ && out_f32 == OF) return launch_t<BM, BN, AK, BK_, OF>(a, s);
  LJS_CASE(1, 1, 0) LJS_CASE(1, 1, 1) LJS_CASE(0, 0, 0) LJS_CASE(0, 0, 1)
  LJS_CASE(1, 0, 0) LJS_CASE(1, 0, 1) LJS_CASE(0, 1, 0) LJS_CASE(0, 1, 1)
#undef LJS_CASE
  return hipErrorInvalidValue;
}

}  // namespace

// Returns 0 on success.  Preconditions checked here (the Python wrapper checks them too):
// K % 8 == 0; for an m/n-contiguous operand its M (or N) % 8 == 0; 16-byte aligned bases
// and leading dimensions that are multiples of 8 elements.

// LJS_GEMM_TRACE builds: the LDS-DMA launches that follow write their per-wave timelines to
// `buf` (blocks x waves x kTraceSlots u64, zeroed by the caller); null turns it off.  Returns
// kTraceSlots, or 0 in a library built without the instrumentation.
LJS_API void ljs_gemm_group_begin() {
  g_group_on = true;
  g_group_n = 0;
}

// launches what the open group recorded (grouped when it is two GEMMs of one kernel instance)
LJS_API int ljs_gemm_group_end(hipStream_t stream) {
  g_group_on = false;
  const int n = g_group_n;
  g_group_n = 0;
  if (n == 0) return 0;
  if (n == 2 && g_group[0].kind == g_group[1].kind) return (int)launch_rec(g_group, 2, stream);
  for (int i = 0; i < n; ++i) {
    const hipError_t e = launch_rec(&g_group[i], 1, stream);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

LJS_API int ljs_gemm_set_trace(void* buf) {
#ifdef LJS_GEMM_TRACE
  g_gemm_trace = (unsigned long long*)buf;
  return kTraceSlots;
#else
  (void)buf;
  return 0;
#endif
}

LJS_API int ljs_gemm_bf16(const void* A, const void* B, void* C, const void* bias, int M, int N, int K,
                          long lda, long ldb, long ldc, long sA, long sB, long sC, long sBias, int batch,
                          int a_kc, int b_kc, int out_f32, int flags, float alpha, int splitk, int tile,
                          void* psum, int* psum_count, const void* res, long ldr, long sR, hipStream_t stream) {
  if (K % 8 || (!a_kc && M % 8) || (!b_kc && N % 8) || lda % 8 || ldb % 8) return (int)hipErrorInvalidValue;
  if (splitk > 1 && !out_f32) return (int)hipErrorInvalidValue;
  // the epilogue operand applies to bf16 outputs (its 16-byte loads need aligned 8-column chunks)
  if ((flags & (kResAdd | kResMask)) &&
      (out_f32 || !res || (ldr % 8) || (sR % 8) || (N % 8) || (((uintptr_t)res) & 15)))
    return (int)hipErrorInvalidValue;
  GemmArgs a;
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = C;
  a.bias = bias;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.sA = sA; a.sB = sB; a.sC = sC; a.sBias = sBias;
  a.M = M; a.N = N; a.K = K;
  a.batch = batch;
  a.alpha = alpha;
  a.flags = flags;
  a.psum = nullptr;
  a.res = res;
  a.ldr = ldr;
  a.sR = sR;
  a.trace = nullptr;
  if (flags & kBPtrs) {
    // B is a HOST array of `batch` (<= 4) device pointers, one B operand per batch
    if (batch < 1 || batch > 4 || !(flags & kSlabs)) return (int)hipErrorInvalidValue;
    const void* const* bp = (const void* const*)B;
    for (int i = 0; i < 4; ++i) a.bptr[i] = (const bf16_t*)(i < batch ? bp[i] : bp[0]);
    a.B = a.bptr[0];
  } else {
    for (int i = 0; i < 4; ++i) a.bptr[i] = nullptr;
  }
  if (psum_count) *psum_count = 0;
  // A/B: tile code + 100000 forces the lean K-loop kernel where it applies, + 200000 the general one
  const bool gen_req = tile >= 200000;
  if (gen_req) tile -= 200000;
  const bool lean_req = tile >= 100000;
  if (lean_req) tile -= 100000;
  int nkt = (K + BK - 1) / BK;
  if (splitk < 1) splitk = 1;
  if (splitk > nkt) splitk = nkt;
  a.kt_per_split = (nkt + splitk - 1) / splitk;
  a.splitk = (nkt + a.kt_per_split - 1) / a.kt_per_split;
  if (flags & 16) {  // zero C first (split-K accumulates with atomics); C must be one dense block
    if (batch > 1 && sC != (long)M * ldc) return (int)hipErrorInvalidValue;
    size_t es = out_f32 ? 4 : 2;
    size_t bytes = ((size_t)(batch - 1) * sC + (size_t)(M - 1) * ldc + N) * es;
    hipError_t me = hipMemsetAsync(C, 0, bytes, stream);
    if (me != hipSuccess) return (int)me;
  }
  hipError_t e;
  // Persistent LDS-DMA kernels (tile codes): 2561 = 256x128, 8 waves, 3 stages, 1 block/CU
  // (k-contiguous operands only); 1284 = 128x128, 4 waves, 4 stages, 1 block/CU; 1282 =
  // 128x128, 4 waves, 2 stages, 2 blocks/CU.  They need K % 64 == 0, a split that divides the
  // K-tiles and operands addressable with 32-bit byte offsets.
  const int nkt64 = K / BK;
  const bool slabs = flags & kSlabs;
  if (slabs && (!out_f32 || a_kc || b_kc || (flags & (8 | 16)) || K % BK ||
                a.splitk != splitk || !(tile > 1000 || tile == 643 || tile == 644)))
    return (int)hipErrorInvalidValue;  // the caller's slab count must be the launched split count
  const long k_ext = slabs ? (long)a.splitk * a.kt_per_split * BK : K;  // K-rows the splits address
  const bool dma_ok = K % BK == 0 && (slabs || nkt64 % a.splitk == 0) &&
                      (a_kc ? (long)M * lda : k_ext * lda) < (1L << 30) &&
                      (b_kc ? (long)N * ldb : k_ext * ldb) < (1L << 30);
  if (slabs && !dma_ok) return (int)hipErrorInvalidValue;
  const bool dma_store_ok = out_f32 || (N % 8 == 0 && ldc % 8 == 0 && (sC % 8 == 0 || batch == 1) &&
                                        (((uintptr_t)C) & 15) == 0);
  if (tile > 1000 && !(dma_ok && dma_store_ok)) tile = 128;
  // the LDS-DMA kernels carry the epilogue operand in their k-contiguous bf16 variants only
  if ((flags & (kResAdd | kResMask)) && tile > 1000 && !(a_kc && b_kc)) tile = 128;
  if ((flags & (kResAdd | kResMask)) && (tile == 643 || tile == 644)) tile = 64;
  if ((tile == 643 || tile == 644) && !(dma_ok && dma_store_ok)) tile = 64;
  if ((tile == 2563 || tile == 12856) && !(!a_kc && !b_kc && out_f32)) tile = 1282;
  if (tile == 2561 && !(a_kc && b_kc)) tile = 1284;
  if (tile == 2562 && !(a_kc && b_kc && !out_f32 && !(flags & (kResAdd | kResMask)))) tile = 1282;
  if (tile == 2562 && batch > 1) {
    // weight-major batches side by side in C over contiguous B (the fused Q/K/V projection):
    // one GEMM over N * batch columns
    if (sA == 0 && sB == (long)N * ldb && sC == N && ldc == (long)N * batch && !bias &&
        (long)N * batch * ldb < (1L << 30)) {   // (the folded B still addressable by 32-bit offsets)
      a.N = N * batch;
      a.batch = 1;
      N = a.N;
      batch = 1;
    } else {
      tile = 2561;
    }
  }
  if (tile == 1602 && !(a_kc && b_kc && !out_f32 && a.splitk == 1)) tile = 1282;
  if ((tile == 12883 || tile == 12884) && !((!a_kc && !b_kc && out_f32) || (a_kc && b_kc))) tile = 1282;
  // fused output sum (psum): LDS-DMA kernels with bf16 output only; one float per (item, wave)
  if (psum && !out_f32 && tile > 1000) {
    const int bm = (tile == 2561 || tile == 2562) ? 256 : 128;
    const int nw = (tile == 2561 || tile == 2562 || tile == 12883 || tile == 12884) ? 8 : 4;
    const int bn = tile == 1602 ? 160 : tile == 2562 ? 192 : 128;
    a.psum = (float*)psum;
    if (psum_count) *psum_count = ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch * a.splitk * nw;
  }
  // the lean K-loop kernel for the k-contiguous bf16-output LDS-DMA tiles without split-K
  // (tile code + 100000 forces the lean one, + 200000 the general one: A/B and bit-exact tests)
  if (!gen_req && a_kc && b_kc && !out_f32 && a.splitk == 1 && !(flags & kBPtrs) && dma_ok &&
      dma_store_ok) {
    if (tile == 2561) return (int)launch_lean_kk<256, 128, 4, 2, 3>(a, stream);
    if (tile == 2562) return (int)launch_lean_kk<256, 192, 4, 2, 2>(a, stream);
    // (128x160, one item per block: the general kernel measured 14.4 vs 14.8 us, gpurun_out/r5i)
    if (tile == 1602 && lean_req) return (int)launch_lean_kk<128, 160, 4, 1, 2>(a, stream);
    if (tile == 1282) return (int)launch_lean_kk<128, 128, 2, 2, 2>(a, stream);
    if (tile == 1284) return (int)launch_lean_kk<128, 128, 2, 2, 4>(a, stream);
    if (tile == 12883) return (int)launch_lean_kk<128, 128, 2, 4, 3>(a, stream);
    if (tile == 12884) return (int)launch_lean_kk<128, 128, 2, 4, 4>(a, stream);
    if (tile == 644 && !(flags & (kResAdd | kResMask))) return (int)launch_lean_kk<64, 64, 2, 2, 4>(a, stream);
  }
  if (tile == 2563) {
    e = launch_dma<256, 128, 4, 2, 3, false, false, true>(a, stream, 0);
  } else if (tile == 12856) {
    e = launch_dma<128, 256, 2, 4, 3, false, false, true>(a, stream, 0);

  } else if (tile == 1602) {
    e = launch_dma_kk<128, 160, 4, 1, 2>(a, stream);
  } else if (tile == 2562) {
    e = launch_dma_kk<256, 192, 4, 2, 2>(a, stream);
  } else if (tile == 2561) {
    if (out_f32) e = launch_dma<256, 128, 4, 2, 3, true, true, true>(a, stream, 0);
    else e = launch_dma_kk<256, 128, 4, 2, 3>(a, stream);
  } else if (tile == 12883 || tile == 12884) {
    // 128x128, 8 waves, 3 / 4 stages (weight-grad MN x MN f32, or k-contiguous operands)
    const bool d4 = tile == 12884;
    if (!a_kc) {
      if (d4) e = launch_slab<128, 128, 2, 4, 4>(a, stream);
      else e = launch_slab<128, 128, 2, 4, 3>(a, stream);
    } else if (out_f32) {
      if (d4) e = launch_dma<128, 128, 2, 4, 4, true, true, true>(a, stream, 0);
      else e = launch_dma<128, 128, 2, 4, 3, true, true, true>(a, stream, 0);
    } else {
      if (d4) e = launch_dma_kk<128, 128, 2, 4, 4>(a, stream);
      else e = launch_dma_kk<128, 128, 2, 4, 3>(a, stream);
    }
  } else if (tile == 643 || tile == 644) {
    if (a_kc && b_kc && !out_f32 && (flags & (kResAdd | kResMask))) {
      e = hipErrorInvalidValue;  // no epilogue-operand variant at 64x64: use the register-staged tile
    } else {
      // k-contiguous bf16 output: the compile-time epilogue instances (plain / bias + sum)
      if (tile == 644 && a_kc && b_kc && !out_f32) return (int)launch_dma_kk<64, 64, 2, 2, 4>(a, stream);
#define LJS_DMA(AK, BK_, OF)                                                                   \
  if (a_kc == AK && b_kc == BK_ && out_f32 == OF) {                                            \
    if (tile == 644) return (int)launch_dma<64, 64, 2, 2, 4, AK, BK_, OF>(a, stream, 0);       \
    return (int)launch_dma<64, 64, 2, 2, 3, AK, BK_, OF>(a, stream, 0);                        \
  }
      LJS_DMA(1, 1, 0) LJS_DMA(1, 1, 1) LJS_DMA(0, 0, 0) LJS_DMA(0, 0, 1)
      LJS_DMA(1, 0, 0) LJS_DMA(1, 0, 1) LJS_DMA(0, 1, 0) LJS_DMA(0, 1, 1)
#undef LJS_DMA
      e = hipErrorInvalidValue;
    }
  } else if (tile == 1284 || tile == 1282) {
    if (tile == 1282 && !a_kc && !b_kc && out_f32) return (int)launch_slab<128, 128, 2, 2, 2>(a, stream);
    // (plain if/else, not ?: -- see the explicit-instantiation note above)
    if (a_kc && b_kc && !out_f32) {
      if (tile == 1284) return (int)launch_dma_kk<128, 128, 2, 2, 4>(a, stream);
      return (int)launch_dma_kk<128, 128, 2, 2, 2>(a, stream);
    }
#define LJS_DMA(AK, BK_, OF)                                                              \
  if (a_kc == AK && b_kc == BK_ && out_f32 == OF) {                                       \
    if (tile == 1284) return (int)launch_dma<128, 128, 2, 2, 4, AK, BK_, OF>(a, stream, 0); \
    return (int)launch_dma<128, 128, 2, 2, 2, AK, BK_, OF>(a, stream, 0);                  \
  }
    LJS_DMA(1, 1, 0) LJS_DMA(1, 1, 1) LJS_DMA(0, 0, 0) LJS_DMA(0, 0, 1)
    LJS_DMA(1, 0, 0) LJS_DMA(1, 0, 1) LJS_DMA(0, 1, 0) LJS_DMA(0, 1, 1)
#undef LJS_DMA
    e = hipErrorInvalidValue;
  } else if (tile == 64) {
    e = dispatch_layout<64, 64>(a, a_kc, b_kc, out_f32, stream);
  } else {
    e = dispatch_layout<128, 128>(a, a_kc, b_kc, out_f32, stream);
  }
  return (int)e;
}

// ============================================================================ f32 GEMM
// Exact-f32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain, no
// reduced-precision path).  Arbitrary element strides, so any transpose is free; operands are
// read straight from global (this serves the small f32 matmuls of cases 1-4 and generic
// f32 dot_general; large GEMMs run in bf16 above).  One wave per 16x16 output tile, 2x2 waves.
namespace {
struct GemmF32Args {
  const float* A; const float* B; float* C;
  long a_rs, a_cs, b_rs, b_cs, c_rs;
  long sA, sB, sC;
  int M, N, K;
};

__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32Args p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 32 + (wave >> 1) * 16, n0 = blockIdx.y * 32 + (wave & 1) * 16;
  const int b = blockIdx.z;
  const float* A = p.A + b * p.sA;
  const float* B = p.B + b * p.sB;
  const int am = m0 + (lane & 15), bn = n0 + (lane & 15), kk = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < p.K; k0 += 4) {
    const int k = k0 + kk;
    float a = (am < p.M && k < p.K) ? A[am * p.a_rs + k * p.a_cs] : 0.f;
    float bb = (bn < p.N && k < p.K) ? B[k * p.b_rs + bn * p.b_cs] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, acc, 0, 0, 0);
  }
  const int col = n0 + (lane & 15);
  if (col >= p.N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + (lane >> 4) * 4 + r;
    if (row < p.M) p.C[b * p.sC + row * p.c_rs + col] = acc[r];
  }
}
}  // namespace

LJS_API int ljs_gemm_f32(const void* A, const void* B, void* C, int M, int N, int K, long a_rs, long a_cs, long b_rs,
                         long b_cs, long c_rs, long sA, long sB, long sC, int batch, hipStream_t stream) {
  GemmF32Args p;
  p.A = (const float*)A; p.B = (const float*)B; p.C = (float*)C;
  p.a_rs = a_rs; p.a_cs = a_cs; p.b_rs = b_rs; p.b_cs = b_cs; p.c_rs = c_rs;
  p.sA = sA; p.sB = sB; p.sC = sC;
  p.M = M; p.N = N; p.K = K;
  dim3 grid((M + 31) / 32, (N + 31) / 32, batch);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}
