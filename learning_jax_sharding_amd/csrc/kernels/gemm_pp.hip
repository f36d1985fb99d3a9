// Ping-pong bf16 GEMM on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16, f32 accumulation).
//
//   C[b] = alpha * op(A[b]) @ op(B[b]) (+ bias) (relu)     bf16 out, or f32 split-K slabs
//
// Why a second GEMM kernel: the 4-wave LDS-DMA kernel of gemm.hip runs its two waves per SIMD in
// lockstep - both read fragments, both wait at the same barrier, both issue MFMAs - and measured
// ~24-30 % MFMA busy with 0 LDS bank conflicts and ~50 % of wave time waiting
// (profiles/r3ac_step_pmc.txt).  Here each 512-thread block holds TWO wave groups of 4 waves
// (one wave of each group per SIMD) that alternate roles every barrier interval:
//
//     interval:   1        2        3        4     ...
//     group 0:    R(0,0)   M(0,0)   R(0,1)   M(0,1) ...     R = LDS fragment reads + DMA issue
//     group 1:    -        R(0,0)   M(0,0)   R(0,1) ...     M = MFMAs of one 32-deep k-step
//
// Group 1 starts one barrier late (a "stagger"), so on every SIMD one wave's MFMAs cover its
// partner's fragment reads, DMA issue and barrier wait: the matrix pipe is fed by one wave or the
// other in every interval (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_programming.md §5
// 8-phase template with the `wr == 1` stagger).
//
// Staging: 1 KiB LDS-DMA pieces (buffer_load_dwordx4 ... lds) into an NST-deep ring of K-tiles
// (BK = 64), swizzled on the SOURCE address so the fragment reads are conflict-free (the images of
// gemm.hip: k-contiguous rows read with ds_read_b128, m/n-contiguous tiles with
// ds_read_b64_tr_b16).  The (work item, K-tile) sequence of a persistent block is flattened, so
// the next item's first tiles are in flight while the current item's epilogue runs, and each
// group's epilogue sits in its own R interval (its partner is still in its last MFMAs).
//
// Waits: tile t must have landed before the barrier that opens group 0's R(t,0).  Each wave
// waits for ITS pieces of tile t with a counted vmcnt (younger tiles' pieces and the previous
// epilogue's stores may stay in flight) right before that barrier; the stage of tile t-1 is
// refilled only after both groups' reads of it completed (lgkmcnt(0) closes every R interval).
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace {

constexpr int BK = 64;

struct PPArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const void* bias;
  long lda, ldb, ldc;
  long sA, sB, sC, sBias;
  int M, N, K;
  int batch, splitk, kt_per_split;
  float alpha;
  int flags;              // kRelu | kBias | kBiasF32 | kSC1Out | kSlabs | kMFast | kBPtrs
  const bf16_t* bptr[4];  // flags & kBPtrs: batch b's B operand
  float* psum;            // bf16 out: per (item, wave) sum of the stored values (the fused loss sum), or null
  bf16_t* acopy;          // AF32: the bf16 rounding of A ([M][K], dense) for the backward, or null
};

constexpr int kRelu = 1, kBias = 2, kBiasF32 = 4, kSC1Out = 32, kSlabs = 512, kMFast = 1024, kBPtrs = 4096;
constexpr int kSC1 = 16;  // buffer-instruction cache policy bit sc1

// 16-byte chunk XOR of a k-contiguous row (128 B = 8 chunks): conflict-free ds_read_b128
__device__ __forceinline__ int swzk(int row) { return (row >> 1) & 7; }
// XOR of an m/n-contiguous k-row (R bf16 per row), in 16-byte chunks (DMA side)
template <int R>
__device__ __forceinline__ int swzmn16(int krow) {
  if constexpr (R >= 128) return ((krow & 3) | (((krow >> 3) & 1) << 2)) << 1;
  else return ((((krow >> 1) & 1)) | (((krow >> 3) & 1) << 1)) << 1;
}

// MFMA operand fragment: 16 rows (m or n) from rb, 32-deep k-step ks of a 64-deep K-tile
template <int R, bool KC>
__device__ __forceinline__ bf16x8 frag(const bf16_t* lds, int rb, int ks, int lane) {
  if constexpr (KC) {
    const int row = rb + (lane & 15);
    const int kc = ks * 4 + (lane >> 4);
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + row * BK + ((kc ^ swzk(row)) << 3)));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int kr0 = ks * 32 + 8 * g + q, kr1 = kr0 + 4;
    const int c8 = (rb >> 2) + pp;  // 8-byte chunk (4 bf16) of the row
    const s16x4 lo = lds_read_tr16(lds + kr0 * R + ((c8 ^ (swzmn16<R>(kr0) << 1)) << 2));
    const s16x4 hi = lds_read_tr16(lds + kr1 * R + ((c8 ^ (swzmn16<R>(kr1) << 1)) << 2));
    return join_bf16x8(lo, hi);
  }
}

// per-lane source offset (elements, relative to the tile origin) of DMA piece q of an operand
// tile of R rows (k-contiguous: 8 rows x 128 B per piece; m/n-contiguous: 64 / (R / 8) k-rows)
template <int R, bool KC>
__device__ __forceinline__ long piece_src(int q, int lane, long ld) {
  if constexpr (KC) {
    const int row = 8 * q + (lane >> 3), slot = lane & 7;
    return (long)row * ld + 8 * (slot ^ swzk(row));
  } else {
    constexpr int CPR = R / 8, KPP = 64 / CPR;
    static_assert(64 % CPR == 0, "m/n-contiguous tiles of 64, 128, 256 or 512 rows");
    const int krow = KPP * q + lane / CPR, slot = lane % CPR;
    return (long)krow * ld + 8 * (slot ^ swzmn16<R>(krow));
  }
}

// f32 k-contiguous operand (AF32): rows of 64 f32 = 256 B, 1 KiB pieces of 4 rows; 16-byte chunk
// c of row r lands at chunk c ^ (r & 15), so the 2 x ds_read_b128 of a fragment are conflict-free
__device__ __forceinline__ long piece_src_f32(int q, int lane, long ld) {
  const int row = 4 * q + (lane >> 4), slot = lane & 15;
  return (long)row * ld + 4 * (slot ^ (row & 15));
}
// bf16 MFMA operand (8 consecutive k of row rb + lane & 15, k-step ks) from the f32 image, rounded
// to nearest-even like cast_f32_bf16; also returns the packed bits (the backward's bf16 copy)
__device__ __forceinline__ u32x4 frag_f32_bits(const bf16_t* lds, int rb, int ks, int lane) {
  const int row = rb + (lane & 15);
  const int kc = ks * 4 + (lane >> 4);
  const unsigned char* base = reinterpret_cast<const unsigned char*>(lds) + row * 256;
  const f32x4 lo = *reinterpret_cast<const f32x4*>(base + (((2 * kc) ^ (row & 15)) << 4));
  const f32x4 hi = *reinterpret_cast<const f32x4*>(base + (((2 * kc + 1) ^ (row & 15)) << 4));
  return u32x4{pack_bf16x2(lo[0], lo[1]), pack_bf16x2(lo[2], lo[3]), pack_bf16x2(hi[0], hi[1]),
               pack_bf16x2(hi[2], hi[3])};
}

// 64 lanes x 16 B from rsrc + soff + voff (per lane) to LDS [lds, lds + 1 KiB); invisible to the
// compiler's waitcnt pass (see common.h dma_lds_x4): waited for with explicit counted vmcnt
__device__ __forceinline__ void dma16(const u32x4& rs, int voff, int soff, const void* lds) {
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(LDS_PTR(const void))lds);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :: "v"(voff), "s"(rs), "s"(soff), "s"(m) : "memory", "m0");
}

struct Item {
  int b, tm, tn, split;
};

__device__ __forceinline__ Item decode(const PPArgs& p, int item, int ntm, int ntn) {
  Item w;
  int r;
  if (p.flags & kMFast) {
    w.tm = item % ntm;
    r = item / ntm;
    w.tn = r % ntn;
    r /= ntn;
  } else {
    w.tn = item % ntn;
    r = item / ntn;
    w.tm = r % ntm;
    r /= ntm;
  }
  w.b = r % p.batch;
  w.split = r / p.batch;
  return w;
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// vmcnt with a wave-uniform runtime count (a jump over immediates; counts above 47 wait for 47)
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
#define LJS_W(k) case k: wait_vm<k>(); return;
    LJS_W(0) LJS_W(1) LJS_W(2) LJS_W(3) LJS_W(4) LJS_W(5) LJS_W(6) LJS_W(7) LJS_W(8) LJS_W(9) LJS_W(10)
    LJS_W(11) LJS_W(12) LJS_W(13) LJS_W(14) LJS_W(15) LJS_W(16) LJS_W(17) LJS_W(18) LJS_W(19) LJS_W(20)
    LJS_W(21) LJS_W(22) LJS_W(23) LJS_W(24) LJS_W(25) LJS_W(26) LJS_W(27) LJS_W(28) LJS_W(29) LJS_W(30)
    LJS_W(31) LJS_W(32) LJS_W(33) LJS_W(34) LJS_W(35) LJS_W(36) LJS_W(37) LJS_W(38) LJS_W(39) LJS_W(40)
    LJS_W(41) LJS_W(42) LJS_W(43) LJS_W(44) LJS_W(45) LJS_W(46)
#undef LJS_W
    default: wait_vm<47>(); return;
  }
}

// BM x BN block tile; GSN: the two wave groups split the tile's columns (else its rows); WVM:
// waves of a group along M (4 / WVM along N); NST: LDS ring depth in K-tiles.
// BIAS: the launch may carry a bias (<= kBiasMax columns), staged once per block in LDS - a
// per-item global load would be waited for with vmcnt(0) by the compiler (it cannot count the
// DMA pieces issued from asm) and drain the whole ring at every epilogue.
constexpr int kBiasMax = 4096;

// AF32: A is f32 (k-contiguous), rounded to bf16 as the fragments are read (the activation cast
// fused into the GEMM: the reference's f32 input under a bf16 Dense, case6_attention.py:96-99);
// the items of tile column 0 also write A's bf16 rounding from those registers (p.acopy).
template <int BM, int BN, bool GSN, int WVM, int NST, bool A_KC, bool B_KC, bool OUT_F32, bool BIAS = false,
          bool AF32 = false>
__global__ __launch_bounds__(512, 2) void gemm_pp_kernel(PPArgs p) {
  constexpr int GM = GSN ? BM : BM / 2, GN = GSN ? BN / 2 : BN;
  constexpr int WVN = 4 / WVM;
  constexpr int WTM = GM / WVM, WTN = GN / WVN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(WVM * WVN == 4 && WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(BM % 64 == 0 && BN % 64 == 0, "DMA pieces split evenly over 8 waves");
  static_assert(OUT_F32 || TN % 2 == 0, "bf16 output: column blocks pair up into 16-byte row chunks");
  static_assert(!AF32 || (A_KC && !OUT_F32), "f32 A: k-contiguous, bf16 output");
  constexpr int AES = AF32 ? 4 : 2;                                          // A element bytes
  constexpr int A_TILE = BM * BK * AES / 2, B_TILE = BN * BK, STAGE = A_TILE + B_TILE;  // bf16 units
  constexpr int LA = BM * AES / 128, LB = BN / 64, L = LA + LB;              // DMA pieces per wave per K-tile
  constexpr int S_EPI = OUT_F32 ? TM * TN : TM * TN / 2;                     // epilogue stores per wave
  constexpr int S_AC = AF32 ? 2 * TM : 0;                                    // acopy stores per wave per K-tile
  static_assert(L * (NST - 1) + S_EPI + S_AC + 1 <= 63, "vmcnt immediate range");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NST * STAGE + (BIAS ? 2 * kBiasMax : 0)];
  float* bias_lds = reinterpret_cast<float*>(smem + NST * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, w4 = wave & 3;
  const int wm = w4 / WVN, wn = w4 % WVN;
  const int r0w = (GSN ? 0 : grp * GM) + wm * WTM;  // the wave's tile inside the block tile
  const int c0w = (GSN ? grp * GN : 0) + wn * WTN;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int items = p.batch * p.splitk * ntm * ntn;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  const int my_items = slot < items ? (items - slot + G - 1) / G : 0;
  const int nk = p.kt_per_split;
  const int total = my_items * nk;

  // ---- DMA: per-lane source offsets of this wave's pieces (A piece wave + 8 i, B likewise)
  const long a_bytes = AES * (A_KC ? (long)(p.M - 1) * p.lda + p.K : (long)(p.K - 1) * p.lda + p.M);
  const long b_bytes = 2 * (B_KC ? (long)(p.N - 1) * p.ldb + p.K : (long)(p.K - 1) * p.ldb + p.N);
  const int a_step = A_KC ? BK * AES : (int)(BK * p.lda * 2);
  const int b_step = B_KC ? BK * 2 : (int)(BK * p.ldb * 2);
  int va[LA], vb[LB];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    if constexpr (AF32) va[i] = (int)(4 * piece_src_f32(wave + 8 * i, lane, p.lda));
    else va[i] = (int)(2 * piece_src<BM, A_KC>(wave + 8 * i, lane, p.lda));
  }
#pragma unroll
  for (int i = 0; i < LB; ++i) vb[i] = (int)(2 * piece_src<BN, B_KC>(wave + 8 * i, lane, p.ldb));

  int is_item = 0, is_kt = 0, a_off = 0, b_off = 0;
  u32x4 ra, rb;
  auto load_item = [&](int k) {
    const Item w = decode(p, slot + G * k, ntm, ntn);
    ra = rsrc_u4(reinterpret_cast<const unsigned char*>(p.A) + (long)w.b * p.sA * AES, a_bytes);
    rb = rsrc_u4((p.flags & kBPtrs) ? p.bptr[w.b] : p.B + (long)w.b * p.sB, b_bytes);
    const int kt0 = w.split * nk;
    a_off = __builtin_amdgcn_readfirstlane(
        (int)((A_KC ? (long)w.tm * BM * p.lda : (long)w.tm * BM) * AES + (long)kt0 * a_step));
    b_off = __builtin_amdgcn_readfirstlane(
        (int)((B_KC ? (long)w.tn * BN * p.ldb : (long)w.tn * BN) * 2 + (long)kt0 * b_step));
  };
  // piece i (< L) of the current issue-side K-tile into stage st: A pieces first, then B
  auto piece = [&](int st, int i) {
    const bf16_t* base = smem + st * STAGE;
    if (i < LA) dma16(ra, va[i], a_off, base + (wave + 8 * i) * 512);
    else dma16(rb, vb[i - LA], b_off, base + A_TILE + (wave + 8 * (i - LA)) * 512);
  };
  auto advance = [&]() {
    a_off += a_step;
    b_off += b_step;
    if (++is_kt == nk) {
      is_kt = 0;
      ++is_item;
    }
  };
  auto issue_next = [&](int st) {
    if (is_kt == 0) load_item(is_item);
#pragma unroll
    for (int i = 0; i < L; ++i) piece(st, i);
    advance();
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[TM], fb[TN];

  // AF32 bf16 copy of A: written by group 0's waves of the first wave column (each A row read once
  // per block tile) in the items of tile column 0 (each A row block once in all)
  __amdgpu_buffer_rsrc_t rac;
  if constexpr (AF32) rac = make_rsrc(p.acopy, p.acopy ? 2 * (long)p.M * p.K : 0);
  const bool ac_wave = AF32 && p.acopy != nullptr && grp == 0 && wn == 0;
  int ac_row0 = 0, ac_k0 = 0;   // the current item's first A row and K-tile (AF32 copy)
  auto read_frags = [&](int st, int ks, bool ac) {
    const bf16_t* As = smem + st * STAGE;
    const bf16_t* Bs = As + A_TILE;
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = frag<BN, B_KC>(Bs, c0w + 16 * j, ks, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (AF32) {
        const u32x4 bits = frag_f32_bits(As, r0w + 16 * i, ks, lane);
        fa[i] = __builtin_bit_cast(bf16x8, bits);
        if (ac) {
          const int row = ac_row0 + r0w + 16 * i + (lane & 15);
          const int k = ac_k0 + ks * 32 + (lane >> 4) * 8;
          const int off = row < p.M ? (int)(((long)row * p.K + k) * 2) : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b128(bits, rac, off, 0, 0);
        }
      } else {
        fa[i] = frag<BM, A_KC>(As, r0w + 16 * i, ks, lane);
      }
    }
  };
  auto mfmas = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);  // C^T block
    __builtin_amdgcn_s_setprio(0);
  };
  // NST >= 3: the K-tile two ahead is DMA'd from the M intervals, its pieces spread between the
  // MFMAs (one LDS-DMA issue costs ~60 cycles among bare MFMAs but 100-185 inside a phase full of
  // LDS reads and other pieces, MI355X_MICROARCH.md "LDS-DMA piece issue cost"): half the pieces
  // in each of the tile's two M intervals, so the R intervals hold only the fragment reads
  constexpr int H0 = L / 2, H1 = L - H0;
  constexpr int NMF = TM * TN;
  auto mfmas_dma = [&](int st, auto half_c) {
    constexpr int HALF = decltype(half_c)::value;
    constexpr int NP = HALF == 0 ? H0 : H1, P0 = HALF == 0 ? 0 : H0;
    constexpr int STEP = NMF / (NP + 1) > 0 ? NMF / (NP + 1) : 1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < NMF; ++m) {
      const int i = m / TN, j = m % TN;
      acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
      if ((m + 1) % STEP == 0 && (m + 1) / STEP <= NP) {
        __builtin_amdgcn_sched_barrier(0);
        piece(st, P0 + (m + 1) / STEP - 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (NMF / STEP < NP) {
#pragma unroll
      for (int q = NMF / STEP; q < NP; ++q) piece(st, P0 + q);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  using H0_ = std::integral_constant<int, 0>;
  using H1_ = std::integral_constant<int, 1>;

  // ---- epilogue of item k (accumulators -> C), then zero the accumulators
  const bool psum_on = !OUT_F32 && p.psum != nullptr;
  const bool has_bias = (p.flags & kBias) && p.splitk == 1;
  const bool bias_f32 = p.flags & kBiasF32;
  const bool slabs = OUT_F32 && (p.flags & kSlabs);
  const __amdgpu_buffer_rsrc_t rcd = make_rsrc(
      p.C, (OUT_F32 ? 4 : 2) * ((long)((slabs ? p.splitk * p.batch : p.batch) - 1) * p.sC + (long)(p.M - 1) * p.ldc + p.N));
  // (relu and the store cache policy as compile-time arguments: runtime flags inside the
  // unrolled epilogue became one branch per element)
  auto epilogue_t = [&](int k, auto relu_c, auto sc1_c) {
    constexpr bool relu = decltype(relu_c)::value;
    constexpr int cpol = decltype(sc1_c)::value ? kSC1 : 0;
    const Item w = decode(p, slot + G * k, ntm, ntn);
    const int m0 = w.tm * BM + r0w, n0 = w.tn * BN + c0w;
    const int g = lane >> 4;
    if constexpr (!OUT_F32) {
      const bool even = (g & 1) == 0;
      float tsum = 0.f;
      f32x4 bv[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (BIAS) {
          const int col = n0 + 16 * j + 4 * g;
          if (has_bias) bv[j] = *reinterpret_cast<const f32x4*>(bias_lds + (col < kBiasMax ? col : 0));
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = m0 + 16 * i + (lane & 15);
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          f32x4 x = acc[i][2 * q], y = acc[i][2 * q + 1];
          unsigned px[2], py[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float x0 = x[2 * h] * p.alpha + bv[2 * q][2 * h], x1 = x[2 * h + 1] * p.alpha + bv[2 * q][2 * h + 1];
            float y0 = y[2 * h] * p.alpha + bv[2 * q + 1][2 * h];
            float y1 = y[2 * h + 1] * p.alpha + bv[2 * q + 1][2 * h + 1];
            if constexpr (relu) {
              x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); y0 = fmaxf(y0, 0.f); y1 = fmaxf(y1, 0.f);
            }
            px[h] = pack_bf16x2(x0, x1);
            py[h] = pack_bf16x2(y0, y1);
            // rows (16-lane groups) g, g^1 trade: even g ends with block 2q's 8 columns
            // 4g .. 4g + 7, odd g with block 2q + 1's 4(g - 1) .. 4g + 3
            const auto s = __builtin_amdgcn_permlane16_swap(px[h], py[h], false, false);
            px[h] = s[0];
            py[h] = s[1];
          }
          const int col = n0 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);
          const bool ok = row < p.M && col < p.N;  // N % 8 == 0 (launcher): chunks are whole
          const int off = ok ? (int)(((long)w.b * p.sC + (long)row * p.ldc + col) * 2) : 0x7ffffff0;
          const u32x4 v = {px[0], px[1], py[0], py[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v, rcd, off, 0, cpol);
          if (psum_on && ok) {
#pragma unroll
            for (int e = 0; e < 4; ++e) tsum += __uint_as_float(v[e] << 16) + __uint_as_float(v[e] & 0xffff0000u);
          }
        }
      }
      if (psum_on) {
        // fused loss reduction: this wave's share of sum(C) - of the bf16 values just stored - to
        // its own slot (one more store, counted by the next wait)
        tsum = warp_sum64(tsum);
        if (lane == 0) p.psum[(long)(slot + G * k) * 8 + wave] = tsum;
      }
    } else {
      const long cb = (long)(slabs ? w.split * p.batch + w.b : w.b) * p.sC;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = m0 + 16 * i + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + 16 * j + 4 * g;
          f32x4 v = acc[i][j] * p.alpha;
          if constexpr (relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          const bool ok = row < p.M && col < p.N;  // N % 4 == 0 (launcher)
          const int off = ok ? (int)((cb + (long)row * p.ldc + col) * 4) : 0x7ffffff0;
          const u32x4 bits = __builtin_bit_cast(u32x4, v);
          __builtin_amdgcn_raw_buffer_store_b128(bits, rcd, off, 0, cpol);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool relu_on = p.flags & kRelu, sc1_on = p.flags & kSC1Out;
  auto epilogue = [&](int k) {
    if (relu_on) {
      if (sc1_on) epilogue_t(k, T_{}, T_{});
      else epilogue_t(k, T_{}, F_{});
    } else {
      if (sc1_on) epilogue_t(k, F_{}, T_{});
      else epilogue_t(k, F_{}, F_{});
    }
  };

  // tile f + 1 has landed (this wave's pieces of it; counted: younger tiles' pieces and, right
  // after an epilogue, its stores may stay in flight)
  auto wait_next = [&](bool after_epi, bool ac) {
    if constexpr (AF32) {
      if (ac) {   // this tile's bf16 copy stores (both k-steps) are younger than the next tile's pieces
        if (after_epi && psum_on) wait_vm<L * (NST - 2) + S_EPI + 1 + S_AC>();
        else if (after_epi) wait_vm<L * (NST - 2) + S_EPI + S_AC>();
        else wait_vm<L * (NST - 2) + S_AC>();
        return;
      }
    }
    if (after_epi && psum_on) wait_vm<L * (NST - 2) + S_EPI + 1>();
    else if (after_epi) wait_vm<L * (NST - 2) + S_EPI>();
    else wait_vm<L * (NST - 2)>();
  };

  // ---- prologue: tiles 0 .. NST - 2 in flight, tile 0 landed for everyone, then the stagger
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < total) issue_next(s);
  if constexpr (BIAS) {
    // the bias row (batch 0; sBias must be 0), read behind the prologue's DMA
    if (has_bias) {
      for (int c = tid; c < p.N; c += 512)
        bias_lds[c] = bias_f32 ? reinterpret_cast<const float*>(p.bias)[c]
                               : bf2f(reinterpret_cast<const bf16_t*>(p.bias)[c]);
    }
  }
  if (total > 0) {
    if (NST - 1 <= total) wait_vm<L * (NST - 2)>();
    else wait_vm<0>();
  }
  bar();
  if (grp == 1) bar();

  constexpr bool DM = NST >= 3;   // DMA from the M intervals (else from R(f, 0))
  for (int it = 0, f = 0; it < my_items; ++it) {
    for (int kk = 0; kk < nk; ++kk, ++f) {
      const int st = f % NST;
      // R(f, 0): refill the stage of tile f - 1 with tile f + NST - 1 (NST 2), the previous item's
      // epilogue (this group's partner is in its last MFMAs of it), k-step 0 fragments
      const bool dma = f + NST - 1 < total;
      if constexpr (!DM) {
        if (dma) issue_next((f + NST - 1) % NST);
      }
      const bool epi = kk == 0 && it > 0;
      if (epi) epilogue(it - 1);
      bool ac = false;
      if constexpr (AF32) {
        if (ac_wave) {
          if (kk == 0) {
            const Item w = decode(p, slot + G * it, ntm, ntn);
            ac_row0 = w.tn == 0 && w.b == 0 ? w.tm * BM : -1;
            ac_k0 = w.split * nk * BK;
          }
          ac = ac_row0 >= 0;
        }
      }
      read_frags(st, 0, ac);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
      // M(f, 0)
      const int dst = (f + NST - 1) % NST;
      if constexpr (DM) {
        if (dma) {
          if (is_kt == 0) load_item(is_item);
          mfmas_dma(dst, H0_{});
        } else {
          mfmas();
        }
      } else {
        mfmas();
      }
      bar();
      // R(f, 1)
      read_frags(st, 1, ac);
      if constexpr (AF32) {
        if (ac) ac_k0 += BK;   // the copy's next K-tile
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const bool more = f + 1 < total;
      // vector-memory ops younger than tile f + 1's pieces at this wave's wait (they may stay in
      // flight): the epilogue's stores (+ fused-sum store), the bf16 copy of A, and - DMA from the
      // M intervals - tile f + 2's pieces issued so far (group 1 waits before its M(f, 1))
      const int young_common = (epi ? S_EPI + (psum_on ? 1 : 0) : 0) + (ac ? S_AC : 0);
      if (grp == 1 && more) {
        if constexpr (DM) wait_vm_n(young_common + (dma ? H0 : 0));
        else if (f + NST - 1 >= total) wait_vm<0>();
        else wait_next(epi, ac);
      }
      bar();
      // M(f, 1)
      if constexpr (DM) {
        if (dma) {
          mfmas_dma(dst, H1_{});
          advance();
        } else {
          mfmas();
        }
      } else {
        mfmas();
      }
      if (grp == 0 && more) {
        if constexpr (DM) wait_vm_n(young_common + (dma ? L : 0));
        else if (f + NST - 1 >= total) wait_vm<0>();
        else wait_next(epi, ac);
      }
      bar();
    }
  }
  if (my_items > 0) epilogue(my_items - 1);
  if (grp == 0) bar();  // group 1 passed one extra barrier (the stagger)
}

#define LJS_PP_INST(BM, BN, GSN, WVM, NST, AK, BKc, OF) \
  template __global__ void gemm_pp_kernel<BM, BN, GSN, WVM, NST, AK, BKc, OF, false>(PPArgs);
// k-contiguous bf16 GEMMs of the attention block at T = 16384 (one or two rounds of 256 blocks)
LJS_PP_INST(128, 384, true, 2, 2, true, true, false)   // QKV projection  [T x 640] x [640 x 1536]
LJS_PP_INST(128, 320, true, 4, 2, true, true, false)   // out-projection  [T x 512] x [512 x 640]
template __global__ void gemm_pp_kernel<128, 320, true, 4, 2, true, true, false, true>(PPArgs);
// f32 A (the activation cast fused in): QKV projection of the reference's f32 input, 160 KiB LDS
template __global__ void gemm_pp_kernel<128, 384, true, 2, 2, true, true, false, false, true>(PPArgs);
LJS_PP_INST(128, 256, true, 2, 3, true, true, false)   // dh              [T x 640] x [640 x 512]
LJS_PP_INST(128, 256, true, 2, 2, true, true, false)
LJS_PP_INST(256, 256, false, 1, 2, true, true, false)  // 4096-class GEMMs
// weight gradients: m/n-contiguous operands, f32 split-K slabs
LJS_PP_INST(128, 256, true, 2, 3, false, false, true)
LJS_PP_INST(256, 128, false, 2, 3, false, false, true)
LJS_PP_INST(128, 128, true, 4, 3, false, false, true)
#undef LJS_PP_INST

int g_cus = 0;

template <int BM, int BN, bool GSN, int WVM, int NST, bool AK, bool BKc, bool OF, bool BIAS = false,
          bool AF32 = false>
hipError_t launch(PPArgs a, hipStream_t s) {
  if (!g_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  const int items = ntm * ntn * a.batch * a.splitk;
  if (ntm < ntn) a.flags |= kMFast;
  const int grid = items < g_cus ? items : g_cus;
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_pp_kernel<BM, BN, GSN, WVM, NST, AK, BKc, OF, BIAS, AF32>), dim3(grid), dim3(512), 0, s, a);
  return hipGetLastError();
}

}  // namespace

// Configurations (cfg): 1 = 128x384 (QKV), 2 = 128x320 (out-projection), 3 = 128x256 3-stage,
// 4 = 128x256 2-stage, 5 = 256x256 - all k-contiguous, bf16 out; 11 = 128x256, 12 = 256x128,
// 13 = 128x128 - m/n-contiguous operands, f32 out (split-K slabs with flags & 512, else one
// split).  Preconditions (checked): K % 64 == 0, N % 8 == 0, ldc % 8 == 0 (bf16 out), the split
// divides the K-tiles unless slab mode, operand extents < 2^31 bytes, 16-byte aligned bases.
LJS_API int ljs_gemm_pp(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, long lda,
                        long ldb, long ldc, long sA, long sB, long sC, long sBias, int batch, int flags, float alpha,
                        int splitk, int cfg, void* psum, int* psum_count, void* acopy, hipStream_t stream) {
  if (psum_count) *psum_count = 0;
  const bool af32 = cfg == 21;   // f32 A: the QKV configuration with the cast fused in
  if (af32) {
    if (lda % 4 || (((uintptr_t)A) & 15) || batch != 1 || (flags & (kBias | kSlabs | kBPtrs)) || splitk > 1 ||
        (long)M * lda * 4 >= (1L << 31))
      return (int)hipErrorInvalidValue;
    cfg = 1;
  } else if (acopy) {
    return (int)hipErrorInvalidValue;
  }
  const bool kc = cfg < 10;
  const bool out_f32 = !kc;
  if (K % BK || N % 8 || lda % 8 || ldb % 8 || batch < 1) return (int)hipErrorInvalidValue;
  if (!out_f32 && (ldc % 8 || (batch > 1 && sC % 8) || (((uintptr_t)C) & 15))) return (int)hipErrorInvalidValue;
  if (out_f32 && (ldc % 4 || (((uintptr_t)C) & 15) || (batch > 1 && sC % 4))) return (int)hipErrorInvalidValue;
  if (!kc && M % 8) return (int)hipErrorInvalidValue;
  PPArgs a;
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = C;
  a.bias = bias;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.sA = sA; a.sB = sB; a.sC = sC; a.sBias = sBias;
  a.M = M; a.N = N; a.K = K;
  a.batch = batch;
  a.alpha = alpha;
  a.flags = flags & ~kMFast;
  a.psum = out_f32 ? nullptr : (float*)psum;
  a.acopy = (bf16_t*)acopy;
  if (flags & kBPtrs) {
    if (batch > 4 || !(flags & kSlabs)) return (int)hipErrorInvalidValue;
    const void* const* bp = (const void* const*)B;
    for (int i = 0; i < 4; ++i) a.bptr[i] = (const bf16_t*)(i < batch ? bp[i] : bp[0]);
    a.B = a.bptr[0];
  } else {
    for (int i = 0; i < 4; ++i) a.bptr[i] = nullptr;
  }
  const int nkt = K / BK;
  if (splitk < 1) splitk = 1;
  if (splitk > nkt) splitk = nkt;
  a.kt_per_split = (nkt + splitk - 1) / splitk;
  a.splitk = (nkt + a.kt_per_split - 1) / a.kt_per_split;
  const bool slabs = flags & kSlabs;
  if (slabs && (!out_f32 || a.splitk != splitk)) return (int)hipErrorInvalidValue;
  if (!slabs && nkt % a.splitk) return (int)hipErrorInvalidValue;
  if (!slabs && a.splitk > 1) return (int)hipErrorInvalidValue;  // no atomics here: slabs only
  const long k_ext = slabs ? (long)a.splitk * a.kt_per_split * BK : K;
  const long ea = kc ? (long)M * lda : k_ext * lda, eb = kc ? (long)N * ldb : k_ext * ldb;
  if ((af32 ? 4 : 2) * (ea + (long)(batch - 1) * sA) >= (1L << 31) || 2 * eb >= (1L << 31))
    return (int)hipErrorInvalidValue;
  if (af32) return (int)launch<128, 384, true, 2, 2, true, true, false, false, true>(a, stream);
  if (!(flags & kBPtrs) && 2 * (eb + (long)(batch - 1) * sB) >= (1L << 31)) return (int)hipErrorInvalidValue;
  if (a.psum && psum_count) {
    // one partial per (item, wave): items of the configuration's tile
    const int bm = 128, bn = cfg == 1 ? 384 : cfg == 2 ? 320 : cfg == 5 ? 256 : 256;
    *psum_count = ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch * 8;
    if (cfg == 5) *psum_count = ((M + 255) / 256) * ((N + 255) / 256) * batch * 8;
  }
  if (flags & kBias) {
    // bias staged in LDS once per block: one row (sBias 0), at most kBiasMax columns, and only
    // the configurations instantiated with it
    if (sBias != 0 || N > kBiasMax || !bias || cfg != 2) return (int)hipErrorInvalidValue;
    return (int)launch<128, 320, true, 4, 2, true, true, false, true>(a, stream);
  }
  switch (cfg) {
    case 1: return (int)launch<128, 384, true, 2, 2, true, true, false>(a, stream);
    case 2: return (int)launch<128, 320, true, 4, 2, true, true, false>(a, stream);
    case 3: return (int)launch<128, 256, true, 2, 3, true, true, false>(a, stream);
    case 4: return (int)launch<128, 256, true, 2, 2, true, true, false>(a, stream);
    case 5: return (int)launch<256, 256, false, 1, 2, true, true, false>(a, stream);
    case 11: return (int)launch<128, 256, true, 2, 3, false, false, true>(a, stream);
    case 12: return (int)launch<256, 128, false, 2, 3, false, false, true>(a, stream);
    case 13: return (int)launch<128, 128, true, 4, 3, false, false, true>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
