// LJS_HIPCC_FLAGS: -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans
// Fused multi-head attention for gfx950 (head_dim 64), forward and backward.
//
// Semantics (case6_attention.py:120-133): scores = f32(q) . f32(k) * scale, f32 softmax over
// keys, probabilities rounded to bf16, P . V with f32 accumulation, bf16 output.  q and k
// are bf16 values, so bf16 MFMA products accumulated in f32 equal the f32 einsum up to
// summation order.  The S x S score matrix is never materialised (flash-style online
// softmax); the forward stores the per-row log-sum-exp for the backward's recompute.
//
// Layout trick (CDNA4 MFMA 16x16x32): compute S^T = K . Q^T so each lane owns ONE query
// (the accumulator column) and 16 of its keys in registers.  The row softmax is then
// in-lane + two xor-shuffles, and P^T goes straight from the accumulator registers into the
// B operand of O^T = V^T . P^T (the MFMA k-order is permuted identically on both operands),
// with V^T delivered by the transposing LDS read (ds_read_b64_tr_b16).  The backward uses
// the same trick for every product: dV^T = dO^T P, dK^T = Q^T dS (one kernel per key block)
// and dQ^T = K^T dS^T (one kernel per query block), so no atomics and no S x S buffers.
//
// VALU budget (D = 64 gives only 256 MFMA FLOPs per softmax element, so these kernels are
// VALU-bound unless the per-element work is minimal): masking is compiled only into the
// boundary tiles (MASK template), the softmax scale is folded into one FMA before the raw
// v_exp_f32 (no libm range reduction), and the MFMA accumulators stay in VGPRs
// (-amdgpu-mfma-vgpr-form) so no AGPR<->VGPR copies surround the softmax.
//
// Tensors are (batch, seq, heads, 64) with arbitrary batch/seq/head strides (d contiguous),
// so Q/K/V can be column slices of the fused QKV GEMM output.
#include "common.h"

#include <type_traits>

namespace {

constexpr int D = 64;      // head dim
constexpr int BLK = 64;    // queries / keys per tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr int FKR = 256;   // max keys of the K/V-resident forward

// Division by a launch constant without the integer-division sequence (~20 scalar instructions
// each on gfx950): q = (umulhi(n, m) + n) >> s for n < 2^31, m and s from the host (Granlund-
// Montgomery; d = 1 gives m = 1, s = 0).  The resident forward's 8 waves each decode their tile
// in their prologue, so this is per-wave latency before the K/V DMA can issue.
struct FastDiv {
  unsigned m;
  int s, d;
};
static inline FastDiv make_fastdiv(int d) {
  int s = 0;
  while ((1L << s) < d) ++s;
  const unsigned long long m = ((1ULL << 32) * ((1ULL << s) - (unsigned long long)d)) / (unsigned long long)d + 1;
  return FastDiv{(unsigned)m, s, d};
}
struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* o; const bf16_t* dout;
  bf16_t* out;                     // fwd: O ; bwd dkv: dK ; bwd dq: dQ
  bf16_t* out2;                    // bwd dkv: dV
  bf16_t* out3;                    // bwd fused: dQ (out = dK, out2 = dV)
  float* lse;                      // [B][H][Sq], log2 domain of scaled scores
  const float* delta;              // [B][H][Sq], NEGATED: -rowsum(dO o O) (it seeds dP accumulators)
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh;
  long do_sb, do_ss, do_sh, out_sb, out_ss, out_sh, out2_sb, out2_ss, out2_sh, out3_sb, out3_ss, out3_sh;
  int Sq, Sk, H;
  float scale, scale_log2;
  int causal, q_offset;
  int flags32;       // attn_bwd_pair32_kernel's dQ blocks: 128 queries (dq32_body), else 64
  // forward only: running-output merge across key blocks (ring / blockwise context parallelism).
  // acc_mode 0: plain (bf16 out + lse); 1: first block -> f32 oacc + lse; 2: merge into oacc + lse
  // by log-sum-exp; 3: merge, write the FINAL bf16 out (+ lse).  oacc: f32, d contiguous.
  float* oacc;
  long oa_sb, oa_ss, oa_sh;
  int acc_mode;
  int vst;           // outputs 16-byte aligned with row strides % 8 == 0: row tiles leave through an
                     // LDS image as full 128-byte rows (stage_rows16 / flush_rows)
  FastDiv fd_nx, fd_h;  // resident forward: its query-block count and H as launch-constant divisors
  unsigned long long* trace;   // LJS_ATTN_BWD_TRACE builds: fused-backward phase stamps
};
#ifndef LJS_ATTN_BWD_TRACE
#define LJS_ATTN_BWD_TRACE 0   // (diagnostic build define) fused backward: stamps per (block, wave)
#endif

// A/B switches (compile-time): the resident forward's key loop fully unrolled at 256 keys, and
// the fused backward's dQ slices without per-slice guards when all 256 keys are valid
#ifndef LJS_ATTN_FWD_UNROLL
#define LJS_ATTN_FWD_UNROLL 1
#endif
#ifndef LJS_ATTN_DQ_UNGUARD
#define LJS_ATTN_DQ_UNGUARD 1
#endif

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// f32 pair arithmetic of the softmax / dS: packed v_pk_* (LJS_ATTN_PK=1) or two scalar ops
// (LJS_ATTN_PK=0; the build adds -fno-slp-vectorize so the compiler does not re-pack them).
// MI355X_MICROARCH.md prices packed f32 VALU beside MFMAs above the scalar pair; measured A/B in
// profiles/PERF_NOTES.md.
#ifndef LJS_ATTN_PK
#define LJS_ATTN_PK 1
#endif
__device__ __forceinline__ f32x2 pk_fms(const f32x2 a, const f32x2 b, const f32x2 c) {  // a * b - c
#if LJS_ATTN_PK
  return a * b - c;
#else
  f32x2 r;
  r[0] = fmaf(a[0], b[0], -c[0]);
  r[1] = fmaf(a[1], b[1], -c[1]);
  return r;
#endif
}
__device__ __forceinline__ f32x2 pk_mul(const f32x2 a, const f32x2 b) {
#if LJS_ATTN_PK
  return a * b;
#else
  f32x2 r;
  r[0] = a[0] * b[0];
  r[1] = a[1] * b[1];
  return r;
#endif
}
__device__ __forceinline__ f32x2 pk_add(const f32x2 a, const f32x2 b) {
#if LJS_ATTN_PK
  return a + b;
#else
  f32x2 r;
  r[0] = a[0] + b[0];
  r[1] = a[1] + b[1];
  return r;
#endif
}



// XCD-aware 3-D tile index of a 1-D grid of nx * H * B blocks: blocks sharing an XCD (dealt
// round-robin by block id) take CONSECUTIVE tiles, so the query blocks of one (batch, head)
// run on one XCD and re-read that head's K/V from its L2 instead of from HBM/MALL once per XCD.
struct Tile3 {
  int x, h, b;
};
__device__ __forceinline__ Tile3 tile3(int nx, int H) {
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  Tile3 r;
  r.x = t % nx;
  r.h = (t / nx) % H;
  r.b = t / (nx * H);
  return r;
}

__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s);
}
__device__ __forceinline__ Tile3 tile3f(const FastDiv& nx, const FastDiv& H) {
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int q1 = fdiv(t, nx), q2 = fdiv(q1, H);
  Tile3 r;
  r.x = t - q1 * nx.d;
  r.h = q1 - q2 * H.d;
  r.b = q2;
  return r;
}

// ---- LDS image: [64 rows][64 d] bf16, 128-byte rows.  16-byte chunk XOR 2*((row>>1)&3):
// bank-conflict free for BOTH the ds_read_b128 row reads (MFMA operand rows) and the
// ds_read_b64_tr_b16 transposed reads (found by exhaustive bank simulation of both patterns).
__device__ __forceinline__ int img16(int row, int c16) { return row * D + ((c16 ^ (((row >> 1) & 3) << 1)) << 3); }
__device__ __forceinline__ int img8(int row, int c8) { return img16(row, c8 >> 1) + ((c8 & 1) << 2); }

// register-staged tile: rows [r0, r0+64) of a (seq, d) slab with row stride ld
struct TileRegs {
  u32x4 v[2];
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, int r0, int rlim, int tid) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + 256 * i, row = c >> 3, c16 = c & 7;
      int r = r0 + row;
      v[i] = r < rlim ? *reinterpret_cast<const u32x4*>(base + (long)r * ld + c16 * 8) : u32x4{0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + 256 * i, row = c >> 3, c16 = c & 7;
      *reinterpret_cast<u32x4*>(lds + img16(row, c16)) = v[i];
    }
  }
};

// MFMA operand from rows [rb, rb+16) of an image, k-step ks (d 32ks..32ks+31)
__device__ __forceinline__ bf16x8 frag_rows(const bf16_t* lds, int rb, int ks, int lane) {
  int row = rb + (lane & 15);
  int c16 = ks * 4 + (lane >> 4);
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + img16(row, c16)));
}

// MFMA A operand A[m = d][k = row]: d = db + (lane&15); elements 0..3 = rows base0+0..3,
// elements 4..7 = rows base1+0..3 (base0/base1 already include the lane group's offset)
__device__ __forceinline__ bf16x8 frag_tr(const bf16_t* lds, int base0, int base1, int db, int lane) {
  int i = lane & 15, q = i >> 2, p = i & 3;
  int c8 = (db >> 2) + p;
  s16x4 lo = lds_read_tr16(lds + img8(base0 + q, c8));
  s16x4 hi = lds_read_tr16(lds + img8(base1 + q, c8));
  return join_bf16x8(lo, hi);
}

// dS^T image of the fused backward ([keys][64 queries] bf16): 8-byte piece c8 of row r sits at
// c8 ^ fs(r & 15), fs a permutation of 0..15.  Its ds_write_b64 (16 contiguous lanes = 16 keys at
// one c8 per bank group, bank = dword mod 32) hit only 4 distinct piece positions under img8's
// 16-byte swizzle: 4-way conflicts, 24.5 % of the kernel's LDS cycles (profiles/r5j_step_pmc.md).
// With fs the 16 keys cover all 16 positions, and the transposed reads (rows 0..7 / 8..15 per
// half-wave, 4 consecutive pieces per row) still see distinct fs >> 2 per row parity: both
// conflict-free.  Row offsets that are multiples of 16 do not change the swizzle.
__device__ __forceinline__ int fs_swz(int row) { return (((row >> 1) & 3) << 2) | ((row & 1) << 1) | ((row >> 3) & 1); }
__device__ __forceinline__ int imgS(int row, int c8) { return row * D + ((c8 ^ fs_swz(row & 15)) << 2); }
__device__ __forceinline__ int trS_off(int db, int lane) {
  const int i = lane & 15, g = lane >> 4;
  return imgS(4 * g + (i >> 2), (db >> 2) + (i & 3));
}

// frag_tr with the row base split off: rows R0 + (4g + q) and R0 + 16 + (4g + q) for R0 a multiple
// of 8 (the swizzle depends on (row >> 1) & 3 only, which R0 does not change), so the lane part
// `off` = tr_off(db, lane) is computed once per kernel and R0 becomes an immediate LDS offset.
__device__ __forceinline__ int tr_off(int db, int lane) {
  const int i = lane & 15, g = lane >> 4;
  return img8(4 * g + (i >> 2), (db >> 2) + (i & 3));
}
__device__ __forceinline__ bf16x8 frag_tr_o(const bf16_t* lds, int R0, int off) {
  s16x4 lo = lds_read_tr16(lds + R0 * D + off);
  s16x4 hi = lds_read_tr16(lds + (R0 + 16) * D + off);
  return join_bf16x8(lo, hi);
}

// B operand from two accumulator tiles (rows t0: elements 0..3, rows t1: elements 4..7)
__device__ __forceinline__ bf16x8 frag_acc(const f32x4& t0, const f32x4& t1) {
  u32x4 u;
  u[0] = pack_bf16x2(t0[0], t0[1]);
  u[1] = pack_bf16x2(t0[2], t0[3]);
  u[2] = pack_bf16x2(t1[0], t1[1]);
  u[3] = pack_bf16x2(t1[2], t1[3]);
  return __builtin_bit_cast(bf16x8, u);
}

// a lane's 16-byte row fragment (8 consecutive d) straight from global memory
__device__ __forceinline__ bf16x8 load_row_frag(const bf16_t* __restrict__ rowp, bool ok, int ks, int lane) {
  if (!ok) return __builtin_bit_cast(bf16x8, u32x4{0, 0, 0, 0});
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(rowp + 32 * ks + 8 * (lane >> 4)));
}

// store 16 d-values of a lane (dt tiles, 4 consecutive d each) for one (seq) row
__device__ __forceinline__ void store_row_T(bf16_t* rowp, const f32x4 (&acc)[4], float mul, int lane) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    u32x2 w;
    w[0] = pack_bf16x2(acc[dt][0] * mul, acc[dt][1] * mul);
    w[1] = pack_bf16x2(acc[dt][2] * mul, acc[dt][3] * mul);
    *reinterpret_cast<u32x2*>(rowp + 16 * dt + 4 * (lane >> 4)) = w;
  }
}

// The same row tile through LDS: store_row_T issues 4 dwordx2 per lane, each covering 32 bytes of
// 16 different rows, and a wave's stores of a tile queue behind each other (the epilogue store tail
// is store-ISSUE bound, MI355X_MICROARCH "attention epilogue store tail").  Staged into a wave-
// private [rows][64] bf16 image (16-byte chunk c of local row r at chunk c ^ (r & 7): the 16 rows
// of a ds_write_b64 spread over 8 chunk positions) and read back as 16-byte row chunks, the tile
// leaves as dwordx4 stores of 8 whole 128-byte rows each (half the store instructions).
// Local row of this lane: rbase + (lane & 15).
__device__ __forceinline__ void stage_rows16(bf16_t* img, int rbase, const f32x4 (&acc)[4], float mul, int lane) {
  const int r = rbase + (lane & 15), g = lane >> 4;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    u32x2 w;
    w[0] = pack_bf16x2(acc[dt][0] * mul, acc[dt][1] * mul);
    w[1] = pack_bf16x2(acc[dt][2] * mul, acc[dt][3] * mul);
    const int c = (2 * dt + (g >> 1)) ^ (r & 7);
    *reinterpret_cast<u32x2*>(img + r * D + c * 8 + 4 * (g & 1)) = w;
  }
}
// NR staged rows -> global rows row0 + r (row stride ld elements; rows >= rlim skipped)
template <int NR>
__device__ __forceinline__ void flush_rows(const bf16_t* img, bf16_t* base, long ld, int row0, int rlim, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's image writes done (wave-private)
  u32x4 v[NR / 8];
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    const int r = 8 * i + (lane >> 3), c = lane & 7;
    v[i] = *reinterpret_cast<const u32x4*>(img + r * D + ((c ^ (r & 7)) << 3));
  }
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    const int r = 8 * i + (lane >> 3), c = lane & 7;
    if (row0 + r < rlim) *reinterpret_cast<u32x4*>(base + (long)(row0 + r) * ld + c * 8) = v[i];
  }
}

// ============================================================================ forward
struct FwdState {
  f32x4 o[4];
  float m, l;
};

template <bool MASK>
__device__ __forceinline__ void fwd_tile(const AttnArgs& a, FwdState& st, const bf16_t* Kt, const bf16_t* Vt,
                                         const bf16x8 (&qf)[2], int kbase, int qrow, int lane) {
  const int g = lane >> 4;
  f32x4 s[4];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    s[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) s[jt] = mfma16x16x32(frag_rows(Kt, 16 * jt, ks, lane), qf[ks], s[jt]);
  }
  if constexpr (MASK) {
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = kbase + 16 * jt + 4 * g + r;
        bool masked = key >= a.Sk || (a.causal && key > qrow + a.q_offset);
        s[jt][r] = masked ? -INFINITY : s[jt][r];
      }
  }
  float tmax = fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3]));
#pragma unroll
  for (int jt = 1; jt < 4; ++jt)
    tmax = fmaxf(tmax, fmaxf(fmaxf(s[jt][0], s[jt][1]), fmaxf(s[jt][2], s[jt][3])));
  tmax = row4_max(tmax);
  // scores are compared raw (scale > 0 preserves order); the scale is applied in one FMA below
  const float m_new = fmaxf(st.m, tmax * a.scale_log2);
  float m_use = m_new;
  if constexpr (MASK) m_use = m_new == -INFINITY ? 0.f : m_new;  // row fully masked so far: p = 0
  const float alpha = fast_exp2(st.m - m_use);
  // exponent arguments, the row sum and the O rescale as packed f32 pairs (v_pk_fma / v_pk_add /
  // v_pk_mul: half the VALU issues; the row sum as a pairwise tree instead of a 16-long chain)
  const f32x2 sc2 = {a.scale_log2, a.scale_log2}, mm2 = {m_use, m_use};
  f32x2 ps2 = {0.f, 0.f};
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 x = pk_fms(f32x2{s[jt][2 * h], s[jt][2 * h + 1]}, sc2, mm2);
      const f32x2 pv = {fast_exp2(x[0]), fast_exp2(x[1])};
      s[jt][2 * h] = pv[0];
      s[jt][2 * h + 1] = pv[1];
      ps2 = pk_add(ps2, pv);
    }
  const float psum = ps2[0] + ps2[1];
  // no lane's running max moved (the usual case after the first key tiles): alpha is exactly 1
  // (or the row is still all-masked with O = 0), so the O rescale is skipped wave-uniformly
  const bool rescale = !__all(m_new == st.m);
  st.l = st.l * alpha + psum;
  st.m = m_new;
  const f32x2 al2 = {alpha, alpha};
#pragma unroll
  for (int dt = 0; dt < 4 && rescale; ++dt) {
    const f32x2 lo = pk_mul(f32x2{st.o[dt][0], st.o[dt][1]}, al2), hi = pk_mul(f32x2{st.o[dt][2], st.o[dt][3]}, al2);
    st.o[dt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    bf16x8 pb = frag_acc(s[2 * s2], s[2 * s2 + 1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x8 va = frag_tr(Vt, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
      st.o[dt] = mfma16x16x32(va, pb, st.o[dt]);
    }
  }
}


// fwd_tile for TWO 16-query sub-tiles over the same 64-key tile, as the scores (fwd_s2) and the
// softmax update + P.V (fwd_pv2): each K / V fragment is read from LDS once for both sub-tiles.  Per query the same operations in
// the same order as fwd_tile<false> (no masking: Sk % 64 == 0, non-causal).
__device__ __forceinline__ void fwd_s2(f32x4 (&s)[2][4], const bf16_t* Kt, const bf16x8 (&qf)[2][2], int lane) {
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const bf16x8 k0 = frag_rows(Kt, 16 * jt, 0, lane), k1 = frag_rows(Kt, 16 * jt, 1, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
      s[t][jt] = mfma16x16x32(k0, qf[t][0], s[t][jt]);
      s[t][jt] = mfma16x16x32(k1, qf[t][1], s[t][jt]);
    }
  }
}
// the softmax update and P.V of fwd_tile2 on scores already computed by fwd_s2
__device__ __forceinline__ void fwd_pv2(const AttnArgs& a, FwdState (&st)[2], f32x4 (&s)[2][4], const bf16_t* Vt,
                                        int lane) {
  const int g = lane >> 4;
  bf16x8 pb[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float tmax = fmaxf(fmaxf(s[t][0][0], s[t][0][1]), fmaxf(s[t][0][2], s[t][0][3]));
#pragma unroll
    for (int jt = 1; jt < 4; ++jt)
      tmax = fmaxf(tmax, fmaxf(fmaxf(s[t][jt][0], s[t][jt][1]), fmaxf(s[t][jt][2], s[t][jt][3])));
    tmax = row4_max(tmax);
    const float m_new = fmaxf(st[t].m, tmax * a.scale_log2);
    const float m_use = m_new;
    const float alpha = fast_exp2(st[t].m - m_use);
    const f32x2 sc2 = {a.scale_log2, a.scale_log2}, mm2 = {m_use, m_use};
    f32x2 ps2 = {0.f, 0.f};
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 x = pk_fms(f32x2{s[t][jt][2 * h], s[t][jt][2 * h + 1]}, sc2, mm2);
        const f32x2 pv = {fast_exp2(x[0]), fast_exp2(x[1])};
        s[t][jt][2 * h] = pv[0];
        s[t][jt][2 * h + 1] = pv[1];
        ps2 = pk_add(ps2, pv);
      }
    const float psum = ps2[0] + ps2[1];
    const bool rescale = !__all(m_new == st[t].m);
    st[t].l = st[t].l * alpha + psum;
    st[t].m = m_new;
    const f32x2 al2 = {alpha, alpha};
#pragma unroll
    for (int dt = 0; dt < 4 && rescale; ++dt) {
      const f32x2 lo = pk_mul(f32x2{st[t].o[dt][0], st[t].o[dt][1]}, al2);
      const f32x2 hi = pk_mul(f32x2{st[t].o[dt][2], st[t].o[dt][3]}, al2);
      st[t].o[dt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
    }
    pb[t][0] = frag_acc(s[t][0], s[t][1]);
    pb[t][1] = frag_acc(s[t][2], s[t][3]);
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 va = frag_tr(Vt, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t) st[t].o[dt] = mfma16x16x32(va, pb[t][s2], st[t].o[dt]);
    }
  }
}

// forward epilogue of one query row (this lane's 16 d-values of it): normalise, and - for
// blockwise / ring attention - merge with the running (O, lse) of the key blocks seen so far
// (log-sum-exp in the log2 domain; +inf lse marks "no unmasked key yet"), all in registers.
__device__ __forceinline__ void fwd_store(const AttnArgs& a, const f32x4 (&o)[4], float m, float lt, int b, int h,
                                          int qrow, int lane) {
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  const float lse_blk = lt > 0.f ? m + __log2f(lt) : INFINITY;
  const long lidx = ((long)b * a.H + h) * a.Sq + qrow;
  const int g = lane >> 4;
  if (a.acc_mode == 0) {
    bf16_t* op = a.out + b * a.o_sb + (long)qrow * a.o_ss + h * a.o_sh;
    store_row_T(op, o, inv, lane);
    if (g == 0 && a.lse) a.lse[lidx] = lse_blk;
    return;
  }
  float* ap = a.oacc + b * a.oa_sb + (long)qrow * a.oa_ss + h * a.oa_sh + 4 * g;
  if (a.acc_mode == 1) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(ap + 16 * dt) = o[dt] * inv;
    if (g == 0) a.lse[lidx] = lse_blk;
    return;
  }
  const float lp = a.lse[lidx];
  const float x0 = lp == INFINITY ? -INFINITY : lp, x1 = lse_blk == INFINITY ? -INFINITY : lse_blk;
  const float mx = fmaxf(x0, x1);
  float cp = 0.f, cb = 0.f, lnew = INFINITY;
  if (mx != -INFINITY) {
    const float wp = fast_exp2(x0 - mx), wb = fast_exp2(x1 - mx), tot = wp + wb;
    cp = wp / tot;
    cb = wb / tot * inv;
    lnew = mx + __log2f(tot);
  }
  if (a.acc_mode == 2) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 prev = *reinterpret_cast<const f32x4*>(ap + 16 * dt);
      *reinterpret_cast<f32x4*>(ap + 16 * dt) = prev * cp + o[dt] * cb;
    }
  } else {
    bf16_t* op = a.out + b * a.o_sb + (long)qrow * a.o_ss + h * a.o_sh;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(ap + 16 * dt) * cp + o[dt] * cb;
      u32x2 w;
      w[0] = pack_bf16x2(v[0], v[1]);
      w[1] = pack_bf16x2(v[2], v[3]);
      *reinterpret_cast<u32x2*>(op + 16 * dt + 4 * g) = w;
    }
  }
  if (g == 0) a.lse[lidx] = lnew;
}

// acc_mode 0 epilogue of a wave's 16 query rows through the LDS image img (2 KiB, wave-private)
__device__ __forceinline__ void fwd_store_vst(const AttnArgs& a, const f32x4 (&o)[4], float m, float lt, int b, int h,
                                              int qrow0, int lane, bf16_t* img) {
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  const int qrow = qrow0 + (lane & 15);
  if ((lane >> 4) == 0 && a.lse && qrow < a.Sq)
    a.lse[((long)b * a.H + h) * a.Sq + qrow] = lt > 0.f ? m + __log2f(lt) : INFINITY;
  stage_rows16(img, 0, o, inv, lane);
  flush_rows<16>(img, a.out + b * a.o_sb + h * a.o_sh, a.o_ss, qrow0, a.Sq, lane);
}

// K/V-resident forward for Sk <= 256: the whole K and V of the (batch, head) -- at most 2 x
// 32 KB -- go to LDS in ONE burst of LDS-DMA pieces (issued from asm, swizzle on the source
// address), so a block pays the HBM latency once instead of once per 64-key tile behind a
// one-tile register prefetch; the key loop then runs from LDS with no barriers.  NW waves x 16
// queries per block; K/V traffic per query falls with NW.
template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_fwd_res_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[FKR * D];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[FKR * D];
  constexpr int QB = 16 * NW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // tile decode by launch-constant divisors (Granlund-Montgomery, FastDiv): B=64 step 0.1968-0.1990
  // vs 0.1975-0.2017 ms with integer divisions, x3 interleaved (gpurun_out/r6e)
  const Tile3 tl = tile3f(a.fd_nx, a.fd_h);
  const int qb = tl.x, h = tl.h, b = tl.b;
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;

  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, a.q_offset + (qb + 1) * QB);
  const int nkt = (kend + BLK - 1) / BLK;
  // Q fragments first: the oldest loads, so the per-key-tile waits below never hold a tile's
  // compute behind them
  const int qrow = qb * QB + 16 * wave + (lane & 15);
  const bool qok = qrow < a.Sq;
  const bf16_t* qp = a.q + b * a.q_sb + (long)qrow * a.q_ss + h * a.q_sh;
  bf16x8 qf[2];
  qf[0] = load_row_frag(qp, qok, 0, lane);
  qf[1] = load_row_frag(qp, qok, 1, lane);
  {
    const u32x4 rk = rsrc_u4(kb, 2 * ((long)(a.Sk - 1) * a.k_ss + D));
    const u32x4 rv = rsrc_u4(vb, 2 * ((long)(a.Sk - 1) * a.v_ss + D));
    const int npieces = nkt * (BLK / 8);  // 8 rows x 128 B per 1 KiB piece, key-tile major
    // 32-bit offsets (the launcher checks (Sk - 1) x stride x 2 + 128 < 2^31 for this kernel); the
    // full 256-key case unrolled, so each piece's offset is a lane constant plus an immediate
    const int ks32 = (int)a.k_ss, vs32 = (int)a.v_ss;
    if (npieces == FKR / 8) {
#pragma unroll
      for (int i = 0; i < FKR / 8 / NW; ++i) {
        const int pc = wave + NW * i;
        const int row = 8 * pc + (lane >> 3);
        const int c = ((lane & 7) ^ (((row >> 1) & 3) << 1)) * 8;
        const bool ok = row < a.Sk;
        dma_lds_x4(rk, ok ? (row * ks32 + c) * 2 : 0x7ffffff0, Ks + pc * 512);
        dma_lds_x4(rv, ok ? (row * vs32 + c) * 2 : 0x7ffffff0, Vs + pc * 512);
      }
    } else {
      for (int pc = wave; pc < npieces; pc += NW) {
        const int row = 8 * pc + (lane >> 3);
        const int c = ((lane & 7) ^ (((row >> 1) & 3) << 1)) * 8;
        const bool ok = row < a.Sk;
        dma_lds_x4(rk, ok ? (row * ks32 + c) * 2 : 0x7ffffff0, Ks + pc * 512);
        dma_lds_x4(rv, ok ? (row * vs32 + c) * 2 : 0x7ffffff0, Vs + pc * 512);
      }
    }
  }
  FwdState st;
#pragma unroll
  for (int i = 0; i < 4; ++i) st.o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  st.m = -INFINITY;
  st.l = 0.f;
  const int qrow0 = qb * QB + 16 * wave;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if ((a.Sk % BLK) == 0 && !a.causal) {
    if (LJS_ATTN_FWD_UNROLL && nkt == FKR / BLK) {
      // 256 keys: the key loop fully unrolled, so a tile's K / V fragment reads can issue during
      // the previous tile's softmax
#pragma unroll
      for (int kt = 0; kt < FKR / BLK; ++kt)
        fwd_tile<false>(a, st, Ks + kt * BLK * D, Vs + kt * BLK * D, qf, kt * BLK, qrow, lane);
    } else {
      for (int kt = 0; kt < nkt; ++kt)
        fwd_tile<false>(a, st, Ks + kt * BLK * D, Vs + kt * BLK * D, qf, kt * BLK, qrow, lane);
    }
  } else {
    for (int kt = 0; kt < nkt; ++kt) {
      const int kbase = kt * BLK;
      if (a.causal && kbase > qrow0 + 15 + a.q_offset) break;
      const bool need_mask = kbase + BLK > a.Sk || (a.causal && kbase + BLK - 1 > qrow0 + a.q_offset);
      if (need_mask) fwd_tile<true>(a, st, Ks + kt * BLK * D, Vs + kt * BLK * D, qf, kbase, qrow, lane);
      else fwd_tile<false>(a, st, Ks + kt * BLK * D, Vs + kt * BLK * D, qf, kbase, qrow, lane);
    }
  }
  float lt = row4_sum(st.l);
  if (a.vst && a.acc_mode == 0) {
    __syncthreads();  // every wave is done with the K / V images
    fwd_store_vst(a, st.o, st.m, lt, b, h, qrow0, lane, Ks + wave * 16 * D);
  } else if (qok) {
    fwd_store(a, st.o, st.m, lt, b, h, qrow, lane);
  }
}

// ============================================================================ fused Q/K/V projection + forward
// One workgroup item = one (batch, head) of a self-attention block whose sequence is exactly 256
// tokens: the projection GEMM's 256 x 192 output tile [Q_h | K_h | V_h] (x rows b*256.., the three
// stacked transposed weights' rows h*64..) and then the attention forward of that head over it,
// from LDS.  The Q/K/V tile still goes to global memory (the backward reads it, and it is the
// dense's output), but the forward's read of it back from HBM / L2 (Q, K, V: 3/4 of the forward's
// bytes) and the separate kernel's load phase are gone, and the projection's store tail overlaps
// the attention math of the same block.
//   * GEMM: 8 waves of 64 x 96 (4 x 2), 16x16x32 bf16 MFMA with the B rows as the MFMA A operand
//     (C^T blocks), K-tiles of 64 by LDS-DMA into a two-slot ring [0, 56 KiB) / [96 KiB, 152 KiB),
//     one K-tile in flight -- the same per-element MFMA sequence as gemm_lean_kernel<256, 192>, so
//     the Q/K/V values are bit-identical to the unfused projection;
//   * epilogue: the tile into LDS images Q / K / V [256][64] (img16 swizzle) over [0, 96 KiB) --
//     the next item's first K-tile streams into the other slot -- and, after the images' barrier,
//     from the images to global [T][3N] as whole 128-byte rows, draining under the attention
//     (stores straight from the accumulators before the barrier: epilogue 7.3k vs 3.1k cycles);
//   * attention: wave w owns queries 32 w .. 32 w + 31 (two 16-query sub-tiles sharing each K / V
//     fragment read, fwd_s2 / fwd_pv2: the resident forward's per-query operations; O / lse agree
//     with it up to the f32 rounding of the running softmax state), O staged through the wave's
//     own (consumed) Q rows and stored as whole 128-byte rows.
struct QkvAttnArgs {
  const bf16_t* x;   // [T][K] bf16, row stride ldx
  const bf16_t* w;   // [3][N][K] bf16: transposed Q / K / V weights, k-contiguous
  bf16_t* qkv;       // [T][3N]: Q | K | V column blocks
  bf16_t* o;         // [T][N] = [B][S][H][D]
  float* lse;        // [B][H][S]
  int T, K, N, H, ldx;
  float scale_log2;
  unsigned long long* trace;   // LJS_QA_TRACE builds: per (block, wave, item) 4 shader-clock stamps
};

#ifndef LJS_QA_TRACE
#define LJS_QA_TRACE 0   // (diagnostic build define) phase stamps: item start, K-loop end, epilogue end, attention end
#endif

constexpr int QA_S = 256, QA_BN = 192, QA_BK = 64;
constexpr int QA_A_TILE = QA_S * QA_BK, QA_STAGE = (QA_S + QA_BN) * QA_BK;   // elements
constexpr int QA_SLOT_C = 48 * 1024;                                          // elements (96 KiB)
constexpr int QA_LDS = QA_SLOT_C + QA_STAGE;                                  // 152 KiB

__device__ __forceinline__ int qa_swz(int row, int c16) { return c16 ^ ((row >> 1) & 7); }

__global__ __launch_bounds__(512, 1) void qkv_attn_fwd_kernel(QkvAttnArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[QA_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int items = (p.T / QA_S) * p.H;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  const int my_items = slot < items ? (items - slot + G - 1) / G : 0;
  if (my_items == 0) return;
  const int nk = p.K / QA_BK;   // even (launcher): tile t of an item lands in slot C (even t) / A (odd t)

  // LDS-DMA pieces (8 rows x 128 B): A 32 per K-tile (4 per wave), B 24 (3 per wave)
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.x, 2 * ((long)(p.T - 1) * p.ldx + p.K));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.w, 2 * (3L * p.N * p.K));
  int va[4], vb[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (wave + 8 * i) + (lane >> 3), c = lane & 7;
    va[i] = (row * p.ldx + 8 * qa_swz(row, c)) * 2;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int row = 8 * (wave + 8 * i) + (lane >> 3), c = lane & 7;   // B-tile row: weight row / 64, row % 64
    vb[i] = ((((row >> 6) * p.N) + (row & 63)) * p.K + 8 * qa_swz(row, c)) * 2;
  }
  auto item_of = [&](int k) { return slot + G * k; };
  // K-tile kt of item k into its slot (the item's row / column bases as the uniform offset)
  auto issue = [&](int k, int kt) {
    const int it = item_of(k);
    const int b = it / p.H, h = it - b * p.H;
    bf16_t* st = smem + ((kt & 1) ? 0 : QA_SLOT_C);
    const int sa = __builtin_amdgcn_readfirstlane(b * QA_S * p.ldx * 2 + kt * QA_BK * 2);
    const int sb = __builtin_amdgcn_readfirstlane(h * 64 * p.K * 2 + kt * QA_BK * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_PTR(void))(st + (wave + 8 * i) * 512), 16, va[i], sa, 0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDS_PTR(void))(st + QA_A_TILE + (wave + 8 * i) * 512), 16, vb[i],
                                               sb, 0, 0);
  };
  auto frag = [&](const bf16_t* img, int rb0, int ks) {
    const int row = rb0 + (lane & 15), kc = ks * 4 + (lane >> 4);
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + row * QA_BK + qa_swz(row, kc) * 8));
  };

  AttnArgs a = {};
  a.out = p.o;
  a.lse = p.lse;
  a.H = p.H;
  a.Sq = QA_S;
  a.Sk = QA_S;
  a.o_sb = (long)QA_S * p.N;
  a.o_ss = p.N;
  a.o_sh = D;
  a.scale_log2 = p.scale_log2;
  bf16_t* const Qi = smem;               // [256][64] images, img16 swizzle
  bf16_t* const Ki = smem + QA_S * D;
  bf16_t* const Vi = smem + 2 * QA_S * D;

  auto barrier = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  bf16x8 ka[4], kb[6], la[4], lb[6];
  auto read_frags = [&](int kt, int ks, bf16x8* af, bf16x8* bfr) {
    const bf16_t* As = smem + ((kt & 1) ? 0 : QA_SLOT_C);
    const bf16_t* Bs = As + QA_A_TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(As, wr * 64 + i * 16, ks);
#pragma unroll
    for (int j = 0; j < 6; ++j) bfr[j] = frag(Bs, wc * 96 + j * 16, ks);
  };
  f32x4 acc[4][6];
  auto mfmas = [&](const bf16x8* af, const bf16x8* bfr) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);   // C^T blocks
  };

  // (diagnostic builds) lane 0 of each wave stores a shader-clock stamp: a vector store under the
  // lane-0 exec mask; items past the 8th of a block are not recorded
  auto stamp = [&](int k, int ph) {
#if LJS_QA_TRACE
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (p.trace && lane == 0 && k < 8) p.trace[(((long)blockIdx.x * 8 + wave) * 8 + k) * 4 + ph] = t;
#else
    (void)k;
    (void)ph;
#endif
  };

  issue(0, 0);
  for (int k = 0; k < my_items; ++k) {
    const int it = item_of(k);
    const int b = it / p.H, h = it - b * p.H;
    stamp(k, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the lean K-loop (gemm_lean_kernel): k-step 1's fragments are read under k-step 0's MFMAs,
    // the next tile's k-step 0 under k-step 1's; one K-tile in flight.  Item start: tile 0 landed
    // for every wave (and every wave is done with the previous item's images, which tile 1 covers)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    read_frags(0, 0, ka, kb);
    issue(k, 1);
    for (int kt = 0; kt + 1 < nk; ++kt) {
      read_frags(kt, 1, la, lb);
      mfmas(ka, kb);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile kt + 1 landed (this wave's pieces)
      barrier();                                           // ... every wave's; tile kt's reads done
      read_frags(kt + 1, 0, ka, kb);
      if (kt + 2 < nk) issue(k, kt + 2);                   // into tile kt's slot
      else if (k + 1 < my_items) issue(k + 1, 0);          // slot C (tile nk - 2's; nk is even)
      mfmas(la, lb);
    }
    read_frags(nk - 1, 1, la, lb);
    mfmas(ka, kb);
    mfmas(la, lb);
    stamp(k, 1);
    // ---- epilogue: every wave is done with the last tile's slot (A) before the images cover it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      const int g = lane >> 4;
      const bool even = (g & 1) == 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int c = wc * 96 + 16 * (even ? 2 * q : 2 * q + 1) + 4 * (g & ~1);   // 8 columns, one of Q / K / V
          float v[8];
          pair_rows16(acc[i][2 * q], acc[i][2 * q + 1], even, v);
          u32x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
          const int which = c >> 6, d = c & 63;
          *reinterpret_cast<u32x4*>(smem + which * QA_S * D + img16(r, d >> 3)) = pk;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stamp(k, 2);
    // the Q / K / V tile to global from the images as whole 128-byte rows (8 lanes per row),
    // draining under the attention below.  Wave w copies rows 32 w .. 32 w + 31 of each image: its
    // Q rows are exactly the ones it later overwrites with its own O staging (no other wave's)
#pragma unroll 4
    for (int i = 0; i < 12; ++i) {
      const int which = i >> 2, r = 32 * wave + 8 * (i & 3) + (lane >> 3), c = lane & 7;
      const u32x4 val = *reinterpret_cast<const u32x4*>(smem + which * QA_S * D + img16(r, c));
      *reinterpret_cast<u32x4*>(p.qkv + (long)(b * QA_S + r) * (3 * p.N) + which * p.N + h * D + c * 8) = val;
    }
    // ---- attention over the images: wave w, queries 32 w + 16 s + (lane & 15)
    {
      FwdState st[2];
      bf16x8 qf[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) st[s].o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        st[s].m = -INFINITY;
        st[s].l = 0.f;
        qf[s][0] = frag_rows(Qi, 32 * wave + 16 * s, 0, lane);
        qf[s][1] = frag_rows(Qi, 32 * wave + 16 * s, 1, lane);
      }
      // (key tiles in order; issuing tile kt + 1's score MFMAs before tile kt's softmax measured
      // slower: 13.2k vs 12.5k cycles per item, profiles/r6n_fused_pipe_phases.txt -- the phase is
      // bound by the SIMD's issue of MFMA + VALU + v_exp_f32, not by their serialisation)
#pragma unroll 1
      for (int kt = 0; kt < QA_S / BLK; ++kt) {
        f32x4 sc[2][4];
        fwd_s2(sc, Ki + kt * BLK * D, qf, lane);
        fwd_pv2(a, st, sc, Vi + kt * BLK * D, lane);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float lt = row4_sum(st[s].l);
        // O through this wave's own Q rows (read into qf above, by this wave only)
        fwd_store_vst(a, st[s].o, st[s].m, lt, b, h, 32 * wave + 16 * s, lane, Qi + (32 * wave + 16 * s) * D);
      }
    }
    stamp(k, 3);
    // (the next item's first barrier orders these image reads before its tile 1 covers them)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Block = 4 waves x NSUB sub-tiles of 16 queries (64 NSUB queries of one head).  Each K/V tile
// staged through LDS serves all NSUB sub-tiles of every wave (NSUB x fewer K/V loads per
// query).  Sub-tile s of wave w holds queries 16 (4 s + w) + lane,
// interleaved so causal work stays balanced across waves.
template <int NSUB>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
  constexpr int QB = BLK * NSUB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tile3 tl = tile3((a.Sq + QB - 1) / QB, a.H);
  const int qb = tl.x, h = tl.h, b = tl.b;

  bf16x8 qf[NSUB][2];
  FwdState st[NSUB];
#pragma unroll
  for (int sb = 0; sb < NSUB; ++sb) {
    const int qrow = qb * QB + 16 * (4 * sb + wave) + (lane & 15);
    const bool qok = qrow < a.Sq;
    const bf16_t* qp = a.q + b * a.q_sb + (long)qrow * a.q_ss + h * a.q_sh;
    qf[sb][0] = load_row_frag(qp, qok, 0, lane);
    qf[sb][1] = load_row_frag(qp, qok, 1, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) st[sb].o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    st[sb].m = -INFINITY;
    st[sb].l = 0.f;
  }
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;

  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, a.q_offset + (qb + 1) * QB);
  const int nkt = (kend + BLK - 1) / BLK;

  TileRegs tk, tv;
  if (nkt > 0) {
    tk.load(kb, a.k_ss, 0, a.Sk, tid);
    tv.load(vb, a.v_ss, 0, a.Sk, tid);
    tk.store(smem, tid);
    tv.store(smem + 2 * BLK * D, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      tk.load(kb, a.k_ss, (kt + 1) * BLK, a.Sk, tid);
      tv.load(vb, a.v_ss, (kt + 1) * BLK, a.Sk, tid);
    }
    const bf16_t* Kt = smem + cur * BLK * D;
    const bf16_t* Vt = smem + (2 + cur) * BLK * D;
    const int kbase = kt * BLK;
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) {
      const int qrow0 = qb * QB + 16 * (4 * sb + wave);
      // wave-uniform: tile entirely in this sub-tile's causal future -> nothing to do
      if (a.causal && kbase > qrow0 + 15 + a.q_offset) continue;
      const bool need_mask = kbase + BLK > a.Sk || (a.causal && kbase + BLK - 1 > qrow0 + a.q_offset);
      if (need_mask) fwd_tile<true>(a, st[sb], Kt, Vt, qf[sb], kbase, qrow0 + (lane & 15), lane);
      else fwd_tile<false>(a, st[sb], Kt, Vt, qf[sb], kbase, qrow0 + (lane & 15), lane);
    }
    if (more) {
      tk.store(smem + (cur ^ 1) * BLK * D, tid);
      tv.store(smem + (2 + (cur ^ 1)) * BLK * D, tid);
    }
    __syncthreads();
  }
#pragma unroll
  for (int sb = 0; sb < NSUB; ++sb) {
    const int qrow = qb * QB + 16 * (4 * sb + wave) + (lane & 15);
    float lt = st[sb].l;
    lt = row4_sum(lt);
    if (qrow < a.Sq) fwd_store(a, st[sb].o, st[sb].m, lt, b, h, qrow, lane);
  }
}

// ============================================================================ backward
// sum over 8 bf16 pairs of x[i] * y[i] in f32
__device__ __forceinline__ float dot_bf16x8(const u32x4& x, const u32x4& y) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    s = fmaf(__uint_as_float(x[k] << 16), __uint_as_float(y[k] << 16), s);
    s = fmaf(__uint_as_float(x[k] & 0xffff0000u), __uint_as_float(y[k] & 0xffff0000u), s);
  }
  return s;
}

// per-lane row constants of one 64-query block: lse/delta for queries q0 + 16t + 4g + r
struct RowConst {
  f32x4 lse[4], dl[4];
  __device__ __forceinline__ void load(const float* __restrict__ lse_row, const float* __restrict__ dl_row, int q0,
                                       int Sq, int g, bool vec) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      int q = q0 + 16 * t + 4 * g;
      if (vec && q + 4 <= Sq) {
        lse[t] = *reinterpret_cast<const f32x4*>(lse_row + q);
        dl[t] = *reinterpret_cast<const f32x4*>(dl_row + q);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          lse[t][r] = q + r < Sq ? lse_row[q + r] : INFINITY;
          dl[t][r] = q + r < Sq ? dl_row[q + r] : 0.f;
        }
      }
    }
  }
};

template <bool MASK>
__device__ __forceinline__ void dkv_tile(const AttnArgs& a, const bf16_t* Qt, const bf16_t* Ot, const RowConst& rc,
                                         const bf16x8 (&kf)[2], const bf16x8 (&vf)[2], f32x4 (&dk)[4],
                                         f32x4 (&dv)[4], int q0, int key, int lane) {
  const int g = lane >> 4;
  // S = Q K^T (rows = queries 16t + 4g + r, col = this lane's key); P; dP = dO V^T; dS
  f32x4 p[4], ds[4];
  const f32x2 sc2 = {a.scale_log2, a.scale_log2};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    // rc.dl holds -delta: dP - delta comes straight out of the MFMA chain it seeds
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = rc.dl[t];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s = mfma16x16x32(frag_rows(Qt, 16 * t, ks, lane), kf[ks], s);
      dp = mfma16x16x32(frag_rows(Ot, 16 * t, ks, lane), vf[ks], dp);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 x = pk_fms(f32x2{s[2 * h], s[2 * h + 1]}, sc2, f32x2{rc.lse[t][2 * h], rc.lse[t][2 * h + 1]});
      p[t][2 * h] = fast_exp2(x[0]);
      p[t][2 * h + 1] = fast_exp2(x[1]);
    }
    if constexpr (MASK) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int q = q0 + 16 * t + 4 * g + r;
        bool ok = q < a.Sq && key < a.Sk && !(a.causal && key > q + a.q_offset);
        p[t][r] = ok ? p[t][r] : 0.f;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 d = pk_mul(f32x2{p[t][2 * h], p[t][2 * h + 1]}, f32x2{dp[2 * h], dp[2 * h + 1]});
      ds[t][2 * h] = d[0];
      ds[t][2 * h + 1] = d[1];
    }
  }
  // dV^T += dO^T P ; dK^T += Q^T dS   (k = queries)
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    bf16x8 pb = frag_acc(p[2 * s2], p[2 * s2 + 1]);
    bf16x8 sb = frag_acc(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x8 oa = frag_tr(Ot, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
      dv[dt] = mfma16x16x32(oa, pb, dv[dt]);
      bf16x8 qa = frag_tr(Qt, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
      dk[dt] = mfma16x16x32(qa, sb, dk[dt]);
    }
  }
}

// dK, dV for one 64-key block (each wave: 16 keys), sweeping all query blocks.  INLINE_DELTA:
// delta = rowsum(dO o O) of each query block is formed here from the staged dO chunks and an O
// prefetch (into dls[2][64]), instead of read from the dQ kernel's output -- so the dQ and dK/dV
// work can run as ONE launch (attn_bwd_pair_kernel) with no ordering between them.
template <bool INLINE_DELTA>
__device__ __forceinline__ void dkv_body(const AttnArgs& a, int kblk, int h, int b, bf16_t* smem, float* dls) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int key0 = kblk * BLK + wave * 16;
  const int key = key0 + (lane & 15);
  const bool kok = key < a.Sk;
  const bf16_t* kp = a.k + b * a.k_sb + (long)key * a.k_ss + h * a.k_sh;
  const bf16_t* vp = a.v + b * a.v_sb + (long)key * a.v_ss + h * a.v_sh;
  bf16x8 kf[2] = {load_row_frag(kp, kok, 0, lane), load_row_frag(kp, kok, 1, lane)};
  bf16x8 vf[2] = {load_row_frag(vp, kok, 0, lane), load_row_frag(vp, kok, 1, lane)};
  const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* ob = a.dout + b * a.do_sb + h * a.do_sh;
  const bf16_t* oo = a.o + b * a.o_sb + h * a.o_sh;
  const float* lse = a.lse + ((long)b * a.H + h) * a.Sq;
  const float* delta = a.delta + ((long)b * a.H + h) * a.Sq;
  const bool vec = (a.Sq % 4) == 0;

  int qstart = 0;
  if (a.causal) qstart = max(0, (kblk * BLK - a.q_offset) / BLK * BLK);
  const int nqt = (a.Sq - qstart + BLK - 1) / BLK;
  // no tile of this wave needs a mask (the usual case): the sweep below runs as an instance
  // without the masked tile variant (no accumulator copies at a join of the two)
  const bool wave_mask = (a.Sq % BLK) != 0 || key0 + 16 > a.Sk || a.causal;

  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  TileRegs tq, tdo, to;
  RowConst rc;
  // delta of the query block whose dO / O chunks are in tdo / to -> dls[buf]
  auto delta_to_lds = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float s = dot_bf16x8(to.v[i], tdo.v[i]);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      const int c = tid + 256 * i;
      if ((c & 7) == 0) dls[buf * BLK + (c >> 3)] = -s;  // negated, as the dQ kernel's delta
    }
  };
  if (nqt > 0) {
    tq.load(qb, a.q_ss, qstart, a.Sq, tid);
    tdo.load(ob, a.do_ss, qstart, a.Sq, tid);
    if constexpr (INLINE_DELTA) {
      to.load(oo, a.o_ss, qstart, a.Sq, tid);
      rc.load(lse, lse, qstart, a.Sq, g, vec);
      delta_to_lds(0);
    } else {
      rc.load(lse, delta, qstart, a.Sq, g, vec);
    }
    tq.store(smem, tid);
    tdo.store(smem + 2 * BLK * D, tid);
  }
  __syncthreads();
  auto sweep = [&](auto wm) {
    constexpr bool WM = decltype(wm)::value;
    for (int it = 0; it < nqt; ++it) {
      const int cur = it & 1;
      const int q0 = qstart + it * BLK;
      const bool more = it + 1 < nqt;
      if (more) {
        tq.load(qb, a.q_ss, q0 + BLK, a.Sq, tid);
        tdo.load(ob, a.do_ss, q0 + BLK, a.Sq, tid);
        if constexpr (INLINE_DELTA) to.load(oo, a.o_ss, q0 + BLK, a.Sq, tid);
      }
      if constexpr (INLINE_DELTA) {
  #pragma unroll
        for (int t = 0; t < 4; ++t) rc.dl[t] = *reinterpret_cast<const f32x4*>(dls + cur * BLK + 16 * t + 4 * g);
      }
      const bf16_t* Qt = smem + cur * BLK * D;
      const bf16_t* Ot = smem + (2 + cur) * BLK * D;
      if constexpr (WM) {
        const bool need_mask = q0 + BLK > a.Sq || key0 + 16 > a.Sk || (a.causal && key0 + 15 > q0 + a.q_offset);
        if (need_mask) dkv_tile<true>(a, Qt, Ot, rc, kf, vf, dk, dv, q0, key, lane);
        else dkv_tile<false>(a, Qt, Ot, rc, kf, vf, dk, dv, q0, key, lane);
      } else {
        dkv_tile<false>(a, Qt, Ot, rc, kf, vf, dk, dv, q0, key, lane);
      }
      if (more) {
        if constexpr (INLINE_DELTA) {
          rc.load(lse, lse, q0 + BLK, a.Sq, g, vec);
          delta_to_lds(cur ^ 1);
        } else {
          rc.load(lse, delta, q0 + BLK, a.Sq, g, vec);
        }
        tq.store(smem + (cur ^ 1) * BLK * D, tid);
        tdo.store(smem + (2 + (cur ^ 1)) * BLK * D, tid);
      }
      __syncthreads();
    }
  };
  if (wave_mask) sweep(std::true_type{});
  else sweep(std::false_type{});
  if (kok) {
    store_row_T(a.out + b * a.out_sb + (long)key * a.out_ss + h * a.out_sh, dk, a.scale, lane);
    store_row_T(a.out2 + b * a.out2_sb + (long)key * a.out2_ss + h * a.out2_sh, dv, 1.f, lane);
  }
}

// Long-key variant: each wave owns 32 keys (two 16-key halves j), so every Q / dO fragment read
// from LDS feeds twice the MFMAs of dkv_tile (the 16-key tile re-read the 64-query operands once
// per 16 keys: at S = 4096 the split backward was bound by those LDS reads).  P and dS of a
// 32-query half are packed to bf16 as they are formed (register pressure), as in fused_tile.
template <bool MASK>
__device__ __forceinline__ void dkv32_tile(const AttnArgs& a, const bf16_t* Qt, const bf16_t* Ot, const float* lse_s,
                                           const float* dl_s, const bf16x8 (&kr)[2][2], const bf16x8 (&vr)[2][2], f32x4 (&dk)[2][4],
                                           f32x4 (&dv)[2][4], int q0, int key0, int lane) {
  const int g = lane >> 4;
  const f32x2 sc2 = {a.scale_log2, a.scale_log2};
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    u32x4 pbu[2], sbu[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * s2 + tt;
      const f32x4 lse = *reinterpret_cast<const f32x4*>(lse_s + 16 * t + 4 * g);
      const f32x4 ndl = *reinterpret_cast<const f32x4*>(dl_s + 16 * t + 4 * g);  // -delta
      const bf16x8 q0f = frag_rows(Qt, 16 * t, 0, lane), q1f = frag_rows(Qt, 16 * t, 1, lane);
      const bf16x8 o0f = frag_rows(Ot, 16 * t, 0, lane), o1f = frag_rows(Ot, 16 * t, 1, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = ndl;
        s = mfma16x16x32(q0f, kr[j][0], s);
        s = mfma16x16x32(q1f, kr[j][1], s);
        dp = mfma16x16x32(o0f, vr[j][0], dp);
        dp = mfma16x16x32(o1f, vr[j][1], dp);
        float pv[4], dsv[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 x = pk_fms(f32x2{s[2 * h], s[2 * h + 1]}, sc2, f32x2{lse[2 * h], lse[2 * h + 1]});
          pv[2 * h] = fast_exp2(x[0]);
          pv[2 * h + 1] = fast_exp2(x[1]);
        }
        if constexpr (MASK) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = q0 + 16 * t + 4 * g + r, key = key0 + 16 * j + (lane & 15);
            const bool ok = q < a.Sq && key < a.Sk && !(a.causal && key > q + a.q_offset);
            pv[r] = ok ? pv[r] : 0.f;
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 d = pk_mul(f32x2{pv[2 * h], pv[2 * h + 1]}, f32x2{dp[2 * h], dp[2 * h + 1]});
          dsv[2 * h] = d[0];
          dsv[2 * h + 1] = d[1];
        }
        pbu[j][2 * tt] = pack_bf16x2(pv[0], pv[1]);
        pbu[j][2 * tt + 1] = pack_bf16x2(pv[2], pv[3]);
        sbu[j][2 * tt] = pack_bf16x2(dsv[0], dsv[1]);
        sbu[j][2 * tt + 1] = pack_bf16x2(dsv[2], dsv[3]);
      }
    }
    bf16x8 pb[2], sb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      pb[j] = __builtin_bit_cast(bf16x8, pbu[j]);
      sb[j] = __builtin_bit_cast(bf16x8, sbu[j]);
    }
    // dV^T += dO^T P ; dK^T += Q^T dS   (k = the 32 queries of this half)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 oa = frag_tr(Ot, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
      const bf16x8 qa = frag_tr(Qt, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        dv[j][dt] = mfma16x16x32(oa, pb[j], dv[j][dt]);
        dk[j][dt] = mfma16x16x32(qa, sb[j], dk[j][dt]);
      }
    }
  }
}

// dK, dV for one 128-key block (4 waves x 32 keys), sweeping all query blocks.  The next query
// block's Q / dO / O and lse arrive by LDS-DMA (no staging registers: with them the 32-key tile
// ran out of VGPRs); delta = rowsum(dO o O) is formed from LDS once they land.
// LDS: QO = [Q0 | Q1 | dO0 | dO1] (64 x D each), Os (64 x D), rowc[2][2][64] = [buf][lse, -delta]
__device__ __forceinline__ void dkv32_body(const AttnArgs& a, int kblk, int h, int b, bf16_t* QO, bf16_t* Os,
                                           float* rowc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int key0 = kblk * (4 * 32) + wave * 32;
  bf16x8 kr[2][2], vr[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = key0 + 16 * j + (lane & 15);
    const bool kok = key < a.Sk;
    const bf16_t* kp = a.k + b * a.k_sb + (long)key * a.k_ss + h * a.k_sh;
    const bf16_t* vp = a.v + b * a.v_sb + (long)key * a.v_ss + h * a.v_sh;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kr[j][ks] = load_row_frag(kp, kok, ks, lane);
      vr[j][ks] = load_row_frag(vp, kok, ks, lane);
    }
  }
  const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* dob = a.dout + b * a.do_sb + h * a.do_sh;
  const bf16_t* ob = a.o + b * a.o_sb + h * a.o_sh;
  const float* lse = a.lse + ((long)b * a.H + h) * a.Sq;
  const u32x4 rq = rsrc_u4(qb, 2 * ((long)(a.Sq - 1) * a.q_ss + D));
  const u32x4 rdo = rsrc_u4(dob, 2 * ((long)(a.Sq - 1) * a.do_ss + D));
  const u32x4 ro = rsrc_u4(ob, 2 * ((long)(a.Sq - 1) * a.o_ss + D));
  const u32x4 rl = rsrc_u4(lse, 4L * a.Sq);
  // pieces p = wave, wave + 4 of a 64-row tile: rows 8p .. 8p + 7, img16 swizzle on the source
  auto issue = [&](int q0, int buf) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int pc = wave + 4 * pp, drow = 8 * pc + (lane >> 3);
      const int dchunk = ((lane & 7) ^ (((drow >> 1) & 3) << 1)) * 8;
      const int r = q0 + drow;
      const bool ok = r < a.Sq;
      dma_lds_x4(rq, ok ? (int)(((long)r * a.q_ss + dchunk) * 2) : 0x7ffffff0, QO + buf * BLK * D + pc * 512);
      dma_lds_x4(rdo, ok ? (int)(((long)r * a.do_ss + dchunk) * 2) : 0x7ffffff0,
                 QO + (2 + buf) * BLK * D + pc * 512);
      dma_lds_x4(ro, ok ? (int)(((long)r * a.o_ss + dchunk) * 2) : 0x7ffffff0, Os + pc * 512);
    }
    if (wave == 0) dma_lds_x1(rl, q0 + lane < a.Sq ? (q0 + lane) * 4 : 0x7ffffff0, rowc + buf * 2 * BLK);
  };
  // after the DMA of `buf` landed for every wave: -delta of its 64 queries (4 threads per row)
  auto finish = [&](int buf) {
    const int row = tid >> 2, c = tid & 3;
    float sacc = 0.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c16 = 2 * c + k;
      const u32x4 o = *reinterpret_cast<const u32x4*>(Os + img16(row, c16));
      const u32x4 d = *reinterpret_cast<const u32x4*>(QO + (2 + buf) * BLK * D + img16(row, c16));
      sacc += dot_bf16x8(o, d);
    }
    sacc += __shfl_xor(sacc, 1, 64);
    sacc += __shfl_xor(sacc, 2, 64);
    if (c == 0) rowc[buf * 2 * BLK + BLK + row] = -sacc;
  };
  int qstart = 0;
  if (a.causal) qstart = max(0, (kblk * 128 - a.q_offset) / BLK * BLK);
  const int nqt = (a.Sq - qstart + BLK - 1) / BLK;  // every wave joins every barrier
  const bool wave_mask = (a.Sq % BLK) != 0 || key0 + 32 > a.Sk || a.causal;
  const bool active = key0 < a.Sk;

  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dk[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  if (nqt > 0) issue(qstart, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nqt > 0) finish(0);
  __syncthreads();
  auto sweep = [&](auto wm) {
    constexpr bool WM = decltype(wm)::value;
    for (int it = 0; it < nqt; ++it) {
      const int cur = it & 1;
      const int q0 = qstart + it * BLK;
      const bool more = it + 1 < nqt;
      if (more) issue(q0 + BLK, cur ^ 1);
      const float* lse_s = rowc + cur * 2 * BLK;
      const bf16_t* Qt = QO + cur * BLK * D;
      const bf16_t* Ot = QO + (2 + cur) * BLK * D;
      if (active) {
        if constexpr (WM) {
          const bool need_mask = q0 + BLK > a.Sq || key0 + 32 > a.Sk || (a.causal && key0 + 31 > q0 + a.q_offset);
          if (need_mask) dkv32_tile<true>(a, Qt, Ot, lse_s, lse_s + BLK, kr, vr, dk, dv, q0, key0, lane);
          else dkv32_tile<false>(a, Qt, Ot, lse_s, lse_s + BLK, kr, vr, dk, dv, q0, key0, lane);
        } else {
          dkv32_tile<false>(a, Qt, Ot, lse_s, lse_s + BLK, kr, vr, dk, dv, q0, key0, lane);
        }
      }
      // the next block's pieces landed (this wave's, then everyone's after the barrier), and
      // every wave is done with block `cur` (its buffers are the next DMA's destination)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (more) finish(cur ^ 1);
      __syncthreads();
    }
  };
  if (wave_mask) sweep(std::true_type{});
  else sweep(std::false_type{});
  if (a.vst) {
    // every wave passed the sweep's last barrier and no DMA is in flight: the Q / dO buffers are
    // free; this wave's 32 key rows of dK / dV go through its own 4 KiB of them each
    if (active) {
      bf16_t* ik = QO + wave * 32 * D;
      bf16_t* iv = QO + (4 + wave) * 32 * D;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        stage_rows16(ik, 16 * j, dk[j], a.scale, lane);
        stage_rows16(iv, 16 * j, dv[j], 1.f, lane);
      }
      flush_rows<32>(ik, a.out + b * a.out_sb + h * a.out_sh, a.out_ss, key0, a.Sk, lane);
      flush_rows<32>(iv, a.out2 + b * a.out2_sb + h * a.out2_sh, a.out2_ss, key0, a.Sk, lane);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = key0 + 16 * j + (lane & 15);
    if (key < a.Sk) {
      store_row_T(a.out + b * a.out_sb + (long)key * a.out_ss + h * a.out_sh, dk[j], a.scale, lane);
      store_row_T(a.out2 + b * a.out2_sb + (long)key * a.out2_ss + h * a.out2_sh, dv[j], 1.f, lane);
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
  const Tile3 tl = tile3((a.Sk + BLK - 1) / BLK, a.H);
  dkv_body<false>(a, tl.x, tl.h, tl.b, smem, nullptr);
}

template <bool MASK>
__device__ __forceinline__ void dq_tile(const AttnArgs& a, const bf16_t* Kt, const bf16_t* Vt, const bf16x8 (&qf)[2],
                                        const bf16x8 (&df)[2], float lse_q, float dl_q, f32x4 (&dq)[4], int kbase,
                                        int qrow, int lane) {
  const int g = lane >> 4;
  f32x4 ds[4];
  const f32x2 sc2 = {a.scale_log2, a.scale_log2}, ls2 = {lse_q, lse_q};
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    // dl_q is -delta: it seeds the dP accumulators (dP - delta out of the MFMA chain)
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{dl_q, dl_q, dl_q, dl_q};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s = mfma16x16x32(frag_rows(Kt, 16 * jt, ks, lane), qf[ks], s);
      dp = mfma16x16x32(frag_rows(Vt, 16 * jt, ks, lane), df[ks], dp);
    }
    float pv[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 x = pk_fms(f32x2{s[2 * h], s[2 * h + 1]}, sc2, ls2);
      pv[2 * h] = fast_exp2(x[0]);
      pv[2 * h + 1] = fast_exp2(x[1]);
    }
    if constexpr (MASK) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = kbase + 16 * jt + 4 * g + r;
        bool ok = qrow < a.Sq && key < a.Sk && !(a.causal && key > qrow + a.q_offset);
        pv[r] = ok ? pv[r] : 0.f;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 d = pk_mul(f32x2{pv[2 * h], pv[2 * h + 1]}, f32x2{dp[2 * h], dp[2 * h + 1]});
      ds[jt][2 * h] = d[0];
      ds[jt][2 * h + 1] = d[1];
    }
  }
  // dQ^T += K^T dS^T   (k = keys)
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    bf16x8 sb = frag_acc(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x8 ka = frag_tr(Kt, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
      dq[dt] = mfma16x16x32(ka, sb, dq[dt]);
    }
  }
}

// dQ for one 64-query block (each wave: 16 queries), sweeping key blocks
__device__ __forceinline__ void dq_body(const AttnArgs& a, int qb, int h, int b, bf16_t* smem, bool write_delta) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qrow0 = qb * BLK + wave * 16;
  const int qrow = qrow0 + (lane & 15);
  const bool qok = qrow < a.Sq;
  const bf16_t* qp = a.q + b * a.q_sb + (long)qrow * a.q_ss + h * a.q_sh;
  const bf16_t* dop = a.dout + b * a.do_sb + (long)qrow * a.do_ss + h * a.do_sh;
  bf16x8 qf[2] = {load_row_frag(qp, qok, 0, lane), load_row_frag(qp, qok, 1, lane)};
  bf16x8 df[2] = {load_row_frag(dop, qok, 0, lane), load_row_frag(dop, qok, 1, lane)};
  const float lse_q = qok ? a.lse[((long)b * a.H + h) * a.Sq + qrow] : INFINITY;
  // delta[q] = sum_d dO[q][d] O[q][d] from the dO fragments already in registers (the 4 lane
  // groups hold d-chunks 8g..8g+7 and 32+8g..): no separate kernel; published for dK/dV.
  float dl_q;
  {
    const bf16_t* op = a.o + b * a.o_sb + (long)qrow * a.o_ss + h * a.o_sh;
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const u32x4 x = __builtin_bit_cast(u32x4, load_row_frag(op, qok, ks, lane));
      const u32x4 y = __builtin_bit_cast(u32x4, df[ks]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s = fmaf(__uint_as_float(x[k] << 16), __uint_as_float(y[k] << 16), s);
        s = fmaf(__uint_as_float(x[k] & 0xffff0000u), __uint_as_float(y[k] & 0xffff0000u), s);
      }
    }
    s = row4_sum(s);
    dl_q = -s;  // delta is kept negated (it seeds the dP accumulators)
    if (write_delta && qok && (lane >> 4) == 0) const_cast<float*>(a.delta)[((long)b * a.H + h) * a.Sq + qrow] = -s;
  }
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, a.q_offset + (qb + 1) * BLK);
  const int nkt = (kend + BLK - 1) / BLK;

  f32x4 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool wave_mask = (a.Sk % BLK) != 0 || qrow0 + 16 > a.Sq || a.causal;
  TileRegs tk, tv;
  if (nkt > 0) {
    tk.load(kb, a.k_ss, 0, a.Sk, tid);
    tv.load(vb, a.v_ss, 0, a.Sk, tid);
    tk.store(smem, tid);
    tv.store(smem + 2 * BLK * D, tid);
  }
  __syncthreads();
  auto sweep = [&](auto wm) {
    constexpr bool WM = decltype(wm)::value;
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nkt;
      if (more) {
        tk.load(kb, a.k_ss, (kt + 1) * BLK, a.Sk, tid);
        tv.load(vb, a.v_ss, (kt + 1) * BLK, a.Sk, tid);
      }
      const bf16_t* Kt = smem + cur * BLK * D;
      const bf16_t* Vt = smem + (2 + cur) * BLK * D;
      const int kbase = kt * BLK;
      if constexpr (WM) {
        const bool need_mask = kbase + BLK > a.Sk || qrow0 + 16 > a.Sq ||
                               (a.causal && kbase + BLK - 1 > qrow0 + a.q_offset);
        if (need_mask) dq_tile<true>(a, Kt, Vt, qf, df, lse_q, dl_q, dq, kbase, qrow, lane);
        else dq_tile<false>(a, Kt, Vt, qf, df, lse_q, dl_q, dq, kbase, qrow, lane);
      } else {
        dq_tile<false>(a, Kt, Vt, qf, df, lse_q, dl_q, dq, kbase, qrow, lane);
      }
      if (more) {
        tk.store(smem + (cur ^ 1) * BLK * D, tid);
        tv.store(smem + (2 + (cur ^ 1)) * BLK * D, tid);
      }
      __syncthreads();
    }
  };
  if (wave_mask) sweep(std::true_type{});
  else sweep(std::false_type{});
  if (qok) store_row_T(a.out + b * a.out_sb + (long)qrow * a.out_ss + h * a.out_sh, dq, a.scale, lane);
}

__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
  const Tile3 tl = tile3((a.Sq + BLK - 1) / BLK, a.H);
  dq_body(a, tl.x, tl.h, tl.b, smem, true);
}

// Long-key dQ variant: each wave owns 32 queries (two 16-query halves i), so every K / V
// fragment read from LDS feeds twice the MFMAs of dq_tile.
template <bool MASK>
__device__ __forceinline__ void dq32_tile(const AttnArgs& a, const bf16_t* Kt, const bf16_t* Vt,
                                          const bf16x8 (&qf)[2][2], const bf16x8 (&df)[2][2], const float (&lse_q)[2],
                                          const float (&dl_q)[2], f32x4 (&dq)[2][4], int kbase, int qrow0, int lane) {
  const int g = lane >> 4;
  const f32x2 sc2 = {a.scale_log2, a.scale_log2};
  u32x4 sbu[2][2];  // [i][s2]: dS of keys 32 s2 .. + 31 packed to bf16 (frag_acc layout)
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const bf16x8 kf0 = frag_rows(Kt, 16 * jt, 0, lane), kf1 = frag_rows(Kt, 16 * jt, 1, lane);
    const bf16x8 vf0 = frag_rows(Vt, 16 * jt, 0, lane), vf1 = frag_rows(Vt, 16 * jt, 1, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{dl_q[i], dl_q[i], dl_q[i], dl_q[i]};
      s = mfma16x16x32(kf0, qf[i][0], s);
      s = mfma16x16x32(kf1, qf[i][1], s);
      dp = mfma16x16x32(vf0, df[i][0], dp);
      dp = mfma16x16x32(vf1, df[i][1], dp);
      const f32x2 ls2 = {lse_q[i], lse_q[i]};
      float pv[4], dsv[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 x = pk_fms(f32x2{s[2 * h], s[2 * h + 1]}, sc2, ls2);
        pv[2 * h] = fast_exp2(x[0]);
        pv[2 * h + 1] = fast_exp2(x[1]);
      }
      if constexpr (MASK) {
        const int qrow = qrow0 + 16 * i + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kbase + 16 * jt + 4 * g + r;
          const bool ok = qrow < a.Sq && key < a.Sk && !(a.causal && key > qrow + a.q_offset);
          pv[r] = ok ? pv[r] : 0.f;
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 d = pk_mul(f32x2{pv[2 * h], pv[2 * h + 1]}, f32x2{dp[2 * h], dp[2 * h + 1]});
        dsv[2 * h] = d[0];
        dsv[2 * h + 1] = d[1];
      }
      sbu[i][jt >> 1][2 * (jt & 1)] = pack_bf16x2(dsv[0], dsv[1]);
      sbu[i][jt >> 1][2 * (jt & 1) + 1] = pack_bf16x2(dsv[2], dsv[3]);
    }
  }
  // dQ^T += K^T dS^T   (k = keys)
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 ka = frag_tr(Kt, 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i) dq[i][dt] = mfma16x16x32(ka, __builtin_bit_cast(bf16x8, sbu[i][s2]), dq[i][dt]);
    }
  }
}

// dQ for one 128-query block (4 waves x 32 queries), sweeping key blocks
__device__ __forceinline__ void dq32_body(const AttnArgs& a, int qb, int h, int b, bf16_t* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qrow0 = qb * 128 + wave * 32;
  bf16x8 qf[2][2], df[2][2];
  float lse_q[2], dl_q[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int qrow = qrow0 + 16 * i + (lane & 15);
    const bool qok = qrow < a.Sq;
    const bf16_t* qp = a.q + b * a.q_sb + (long)qrow * a.q_ss + h * a.q_sh;
    const bf16_t* dop = a.dout + b * a.do_sb + (long)qrow * a.do_ss + h * a.do_sh;
    const bf16_t* op = a.o + b * a.o_sb + (long)qrow * a.o_ss + h * a.o_sh;
    qf[i][0] = load_row_frag(qp, qok, 0, lane);
    qf[i][1] = load_row_frag(qp, qok, 1, lane);
    df[i][0] = load_row_frag(dop, qok, 0, lane);
    df[i][1] = load_row_frag(dop, qok, 1, lane);
    lse_q[i] = qok ? a.lse[((long)b * a.H + h) * a.Sq + qrow] : INFINITY;
    float sacc = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const u32x4 x = __builtin_bit_cast(u32x4, load_row_frag(op, qok, ks, lane));
      const u32x4 y = __builtin_bit_cast(u32x4, df[i][ks]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sacc = fmaf(__uint_as_float(x[k] << 16), __uint_as_float(y[k] << 16), sacc);
        sacc = fmaf(__uint_as_float(x[k] & 0xffff0000u), __uint_as_float(y[k] & 0xffff0000u), sacc);
      }
    }
    dl_q[i] = -row4_sum(sacc);  // delta, kept negated (it seeds the dP accumulators)
  }
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, a.q_offset + (qb + 1) * 128);
  const int nkt = (kend + BLK - 1) / BLK;
  f32x4 dq[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dq[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool wave_mask = (a.Sk % BLK) != 0 || qrow0 + 32 > a.Sq || a.causal;
  const bool active = qrow0 < a.Sq;
  TileRegs tk, tv;
  if (nkt > 0) {
    tk.load(kb, a.k_ss, 0, a.Sk, tid);
    tv.load(vb, a.v_ss, 0, a.Sk, tid);
    tk.store(smem, tid);
    tv.store(smem + 2 * BLK * D, tid);
  }
  __syncthreads();
  auto sweep = [&](auto wm) {
    constexpr bool WM = decltype(wm)::value;
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nkt;
      if (more) {
        tk.load(kb, a.k_ss, (kt + 1) * BLK, a.Sk, tid);
        tv.load(vb, a.v_ss, (kt + 1) * BLK, a.Sk, tid);
      }
      const bf16_t* Kt = smem + cur * BLK * D;
      const bf16_t* Vt = smem + (2 + cur) * BLK * D;
      const int kbase = kt * BLK;
      if (active) {
        if constexpr (WM) {
          const bool need_mask = kbase + BLK > a.Sk || qrow0 + 32 > a.Sq ||
                                 (a.causal && kbase + BLK - 1 > qrow0 + a.q_offset);
          if (need_mask) dq32_tile<true>(a, Kt, Vt, qf, df, lse_q, dl_q, dq, kbase, qrow0, lane);
          else dq32_tile<false>(a, Kt, Vt, qf, df, lse_q, dl_q, dq, kbase, qrow0, lane);
        } else {
          dq32_tile<false>(a, Kt, Vt, qf, df, lse_q, dl_q, dq, kbase, qrow0, lane);
        }
      }
      if (more) {
        tk.store(smem + (cur ^ 1) * BLK * D, tid);
        tv.store(smem + (2 + (cur ^ 1)) * BLK * D, tid);
      }
      __syncthreads();
    }
  };
  if (wave_mask) sweep(std::true_type{});
  else sweep(std::false_type{});
  if (a.vst) {
    // after the sweep's last barrier (no load in flight) the K / V tiles are free: this wave's 32
    // query rows of dQ leave through its own 4 KiB of them as whole-row stores
    if (active) {
      bf16_t* img = smem + wave * 32 * D;
#pragma unroll
      for (int i = 0; i < 2; ++i) stage_rows16(img, 16 * i, dq[i], a.scale, lane);
      flush_rows<32>(img, a.out + b * a.out_sb + h * a.out_sh, a.out_ss, qrow0, a.Sq, lane);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int qrow = qrow0 + 16 * i + (lane & 15);
    if (qrow < a.Sq) store_row_T(a.out + b * a.out_sb + (long)qrow * a.out_ss + h * a.out_sh, dq[i], a.scale, lane);
  }
}

// dQ blocks and dK/dV blocks of the split backward in ONE launch (the dK/dV blocks form delta
// themselves): at the reference shape (B = 8) the two kernels ran back to back as two half-full
// grids of 256 four-wave blocks; here all 512 blocks are resident at once.  Block ids are dealt
// XCD-major (tile3's mapping) over [dQ items | dK/dV items].
__global__ __launch_bounds__(256) void attn_bwd_pair_kernel(AttnArgs dq, AttnArgs dkv) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
  __shared__ __attribute__((aligned(16))) float dls[2 * BLK];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int nq = (dq.Sq + BLK - 1) / BLK, nk = (dkv.Sk + BLK - 1) / BLK;
  const int ndq = nq * dq.H * (gridDim.x / (nq + nk) / dq.H);
  if (t < ndq) {
    dq_body(dq, t % nq, (t / nq) % dq.H, t / (nq * dq.H), smem, false);
  } else {
    const int u = t - ndq;
    dkv_body<true>(dkv, u % nk, (u / nk) % dkv.H, u / (nk * dkv.H), smem, dls);
  }
}

// the same with 128-key dK/dV blocks (dkv32_body): long key ranges, where the 64-key blocks'
// LDS reads of the staged query tiles bound the backward
__global__ __launch_bounds__(256, 2) void attn_bwd_pair32_kernel(AttnArgs dq, AttnArgs dkv) {
  __shared__ __attribute__((aligned(16))) bf16_t QO[4 * BLK * D];  // dQ blocks: their K/V ring
  __shared__ __attribute__((aligned(16))) bf16_t Os[BLK * D];
  __shared__ __attribute__((aligned(16))) float rowc[2 * 2 * BLK];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int qbs = dq.flags32 ? 128 : BLK;  // dQ block: 128 queries (dq32_body) or 64 (dq_body)
  const int nq = (dq.Sq + qbs - 1) / qbs, nk = (dkv.Sk + 127) / 128;
  const int ndq = nq * dq.H * (gridDim.x / (nq + nk) / dq.H);
  if (t < ndq) {
    if (dq.flags32) dq32_body(dq, t % nq, (t / nq) % dq.H, t / (nq * dq.H), QO);
    else dq_body(dq, t % nq, (t / nq) % dq.H, t / (nq * dq.H), QO, false);
  } else {
    const int u = t - ndq;
    dkv32_body(dkv, u % nk, (u / nk) % dkv.H, u / (nk * dkv.H), QO, Os, rowc);
  }
}

// ---------------------------------------------------------------- fused short-key backward
// Sk <= 256: ONE workgroup (8 waves) per (batch, head) keeps K and V in LDS (each wave
// owns 32 keys for dK / dV), then sweeps the query blocks once.  S and dP are computed
// once per (query, key) -- the split dQ / dK-dV kernels compute them twice -- and dS^T goes
// through LDS ([keys][queries] image, ds_write_b64) so dQ^T = K^T dS^T reads it with the
// transposing LDS read.  delta = rowsum(dO o O) is formed while staging each query block.
constexpr int FK = 256;        // max keys
constexpr int FWAVES = 8;      // 32 keys per wave
constexpr int FT = FWAVES * 64;

// one 16-byte chunk per thread of a 64-row (seq, d) tile
struct TileRegs1 {
  u32x4 v;
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, int r0, int rlim, int tid) {
    int row = tid >> 3, c16 = tid & 7, r = r0 + row;
    v = r < rlim ? *reinterpret_cast<const u32x4*>(base + (long)r * ld + c16 * 8) : u32x4{0, 0, 0, 0};
  }
  __device__ __forceinline__ void store(bf16_t* lds, int tid) const {
    *reinterpret_cast<u32x4*>(lds + img16(tid >> 3, tid & 7)) = v;
  }
};

// S/P/dP/dS for this wave's 32 keys x 64 queries; dK^T, dV^T accumulate; dS^T -> LDS
template <bool MASK>
__device__ __forceinline__ void fused_tile(const AttnArgs& a, const bf16_t* Qt, const bf16_t* Ot,
                                           const float* lse_s, const float* dl_s, bf16_t* dSt,
                                           const bf16x8 (&kr)[2][2], const bf16x8 (&vr)[2][2], f32x4 (&dk)[2][4],
                                           f32x4 (&dv)[2][4], int q0, int key0, int lane, const int (&offtr)[4]) {
  const int g = lane >> 4;
  // two 32-query halves: P / dS of a half feed the dK/dV MFMAs right away (register pressure)
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    // P and dS leave the softmax already packed to bf16 pairs (the MFMA B-operand layout of
    // frag_acc): 16 live VGPRs instead of 32 f32, which keeps the kernel out of scratch
    u32x4 pbu[2], sbu[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * s2 + tt;
      const f32x4 lse = *reinterpret_cast<const f32x4*>(lse_s + 16 * t + 4 * g);
      const f32x4 ndl = *reinterpret_cast<const f32x4*>(dl_s + 16 * t + 4 * g);  // -delta
      const bf16x8 q0f = frag_rows(Qt, 16 * t, 0, lane), q1f = frag_rows(Qt, 16 * t, 1, lane);
      const bf16x8 o0f = frag_rows(Ot, 16 * t, 0, lane), o1f = frag_rows(Ot, 16 * t, 1, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // dP - delta straight out of the MFMA chain: its accumulator starts at -delta (a row
        // constant in the accumulator layout) -- no subtraction per element
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = ndl;
        s = mfma16x16x32(q0f, kr[j][0], s);
        s = mfma16x16x32(q1f, kr[j][1], s);
        dp = mfma16x16x32(o0f, vr[j][0], dp);
        dp = mfma16x16x32(o1f, vr[j][1], dp);
        float pv[4], dsv[4];
        // exponent arguments and dS as packed f32 pairs (v_pk_fma_f32 / v_pk_mul_f32: half the
        // VALU issues of the scalar forms; the kernel is VALU-bound at head_dim 64)
        const f32x2 sc2 = {a.scale_log2, a.scale_log2};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 x = pk_fms(f32x2{s[2 * h], s[2 * h + 1]}, sc2, f32x2{lse[2 * h], lse[2 * h + 1]});
          pv[2 * h] = fast_exp2(x[0]);
          pv[2 * h + 1] = fast_exp2(x[1]);
        }
        if constexpr (MASK) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            int q = q0 + 16 * t + 4 * g + r, key = key0 + 16 * j + (lane & 15);
            bool ok = q < a.Sq && key < a.Sk && !(a.causal && key > q + a.q_offset);
            pv[r] = ok ? pv[r] : 0.f;
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 d = pk_mul(f32x2{pv[2 * h], pv[2 * h + 1]}, f32x2{dp[2 * h], dp[2 * h + 1]});
          dsv[2 * h] = d[0];
          dsv[2 * h + 1] = d[1];
        }
        pbu[j][2 * tt] = pack_bf16x2(pv[0], pv[1]);
        pbu[j][2 * tt + 1] = pack_bf16x2(pv[2], pv[3]);
        sbu[j][2 * tt] = pack_bf16x2(dsv[0], dsv[1]);
        sbu[j][2 * tt + 1] = pack_bf16x2(dsv[2], dsv[3]);
        // dS^T row (this lane's key), queries 16t + 4g .. +3
        *reinterpret_cast<u32x2*>(dSt + imgS(key0 + 16 * j + (lane & 15), 4 * t + g)) =
            u32x2{sbu[j][2 * tt], sbu[j][2 * tt + 1]};
      }
    }
    bf16x8 pb[2], sb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      pb[j] = __builtin_bit_cast(bf16x8, pbu[j]);
      sb[j] = __builtin_bit_cast(bf16x8, sbu[j]);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x8 oa = frag_tr_o(Ot, 32 * s2, offtr[dt]);
      bf16x8 qa = frag_tr_o(Qt, 32 * s2, offtr[dt]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        dv[j][dt] = mfma16x16x32(oa, pb[j], dv[j][dt]);
        dk[j][dt] = mfma16x16x32(qa, sb[j], dk[j][dt]);
      }
    }
  }
}

// SW 1: the sweep instance of the common case alone (Sq % 64 == 0, Sk == 256, not causal, dQ
// staged: a.vst == 1), so the kernel's register allocation is that one loop's, not the maximum
// over the four sweep instances; SW 0: all four, chosen at run time
template <bool KVDMA, int SW = 0>
__global__ __launch_bounds__(FT) void attn_bwd_fused_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[FK * D];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[FK * D];
  __shared__ __attribute__((aligned(16))) bf16_t dSt[FK * BLK];
  __shared__ __attribute__((aligned(16))) bf16_t QO[4 * BLK * D];  // Q[2], dO[2]
  __shared__ __attribute__((aligned(16))) bf16_t Os[BLK * D];      // next block's O (delta only)
  __shared__ __attribute__((aligned(16))) float rowc[2][2][BLK];    // [buf][lse, delta][query]
  __shared__ __attribute__((aligned(16))) bf16_t dQs[BLK * D];      // a query block's dQ (a.vst)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int h = blockIdx.x, b = blockIdx.y;
  const int key0 = wave * 32;
  // (diagnostic builds) shader-clock stamps: 0 start, 1 first query block ready, 2 + it after
  // query block it, 7 end; a vector store from lane 0
  auto bstamp = [&](int k) {
#if LJS_ATTN_BWD_TRACE
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (a.trace && lane == 0) a.trace[(((long)b * gridDim.x + h) * (FT / 64) + wave) * 8 + k] = t;
#else
    (void)k;
#endif
  };
  bstamp(0);
  const bool active = key0 < a.Sk;
  const int nk32 = (a.Sk + 31) / 32;

  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  // K and V land by LDS-DMA (swizzle on the source address, rows past Sk read zeros), in flight
  // together with the first query block's Q / dO / O below: one exposed latency, not two (the
  // register-staged copy waited for K / V before the first block's DMA was even issued)
  if constexpr (KVDMA) {
    const u32x4 rk = rsrc_u4(kb, 2 * ((long)(a.Sk - 1) * a.k_ss + D));
    const u32x4 rv = rsrc_u4(vb, 2 * ((long)(a.Sk - 1) * a.v_ss + D));
    constexpr int NWF = FT / 64;
#pragma unroll
    for (int i = 0; i < FK / 8 / NWF; ++i) {
      const int pc = wave + NWF * i;
      const int row = 8 * pc + (lane >> 3);
      const int c = ((lane & 7) ^ (((row >> 1) & 3) << 1)) * 8;
      const bool ok = row < a.Sk;
      dma_lds_x4(rk, ok ? (int)(((long)row * a.k_ss + c) * 2) : 0x7ffffff0, Ks + pc * 512);
      dma_lds_x4(rv, ok ? (int)(((long)row * a.v_ss + c) * 2) : 0x7ffffff0, Vs + pc * 512);
    }
  } else {
    // register-staged copy (the default from 3 query blocks up: 45.98 vs 47.01 us for the
    // LDS-DMA form at B=64, gpurun_out/r3aj; the launch picks the DMA form for <= 128 queries)
#pragma unroll
    for (int i = 0; i < FK * 8 / FT; ++i) {
      int c = tid + FT * i, row = c >> 3, c16 = c & 7;
      u32x4 x = row < a.Sk ? *reinterpret_cast<const u32x4*>(kb + (long)row * a.k_ss + c16 * 8) : u32x4{0, 0, 0, 0};
      u32x4 y = row < a.Sk ? *reinterpret_cast<const u32x4*>(vb + (long)row * a.v_ss + c16 * 8) : u32x4{0, 0, 0, 0};
      *reinterpret_cast<u32x4*>(Ks + img16(row, c16)) = x;
      *reinterpret_cast<u32x4*>(Vs + img16(row, c16)) = y;
    }
  }

  const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* dob = a.dout + b * a.do_sb + h * a.do_sh;
  const bf16_t* ob = a.o + b * a.o_sb + h * a.o_sh;
  const float* lse = a.lse + ((long)b * a.H + h) * a.Sq;
  const int nqt = (a.Sq + BLK - 1) / BLK;

  // Next query block's Q / dO / O (and its log-sum-exp) arrive by LDS-DMA (buffer_load ... lds,
  // issued from inline asm -- see dma_lds_x4):
  // no staging VGPRs (those spilled the kernel to scratch, and every scratch reload's vmcnt(0)
  // waited for the whole prefetch), one 1 KiB piece per wave per tile.  The img16 swizzle is
  // applied on the SOURCE address (a wave's DMA fills 1 KiB of LDS contiguously); rows past Sq
  // get an out-of-range offset and read as zeros.
  const u32x4 rq = rsrc_u4(qb, 2 * ((long)(a.Sq - 1) * a.q_ss + D));
  const u32x4 rdo = rsrc_u4(dob, 2 * ((long)(a.Sq - 1) * a.do_ss + D));
  const u32x4 ro = rsrc_u4(ob, 2 * ((long)(a.Sq - 1) * a.o_ss + D));
  const u32x4 rl = rsrc_u4(lse, 4L * a.Sq);
  const int drow = 8 * wave + (lane >> 3);
  const int dchunk = ((lane & 7) ^ (((drow >> 1) & 3) << 1)) * 8;  // element offset in the row
  auto issue = [&](int q0, int buf) {
    const int r = q0 + drow;
    const bool ok = r < a.Sq;
    const int oq = ok ? (int)(((long)r * a.q_ss + dchunk) * 2) : 0x7ffffff0;
    const int odo = ok ? (int)(((long)r * a.do_ss + dchunk) * 2) : 0x7ffffff0;
    const int oo = ok ? (int)(((long)r * a.o_ss + dchunk) * 2) : 0x7ffffff0;
    dma_lds_x4(rq, oq, QO + buf * BLK * D + wave * 512);
    dma_lds_x4(rdo, odo, QO + (2 + buf) * BLK * D + wave * 512);
    dma_lds_x4(ro, oo, Os + wave * 512);
    if (wave == 0) dma_lds_x1(rl, q0 + lane < a.Sq ? (q0 + lane) * 4 : 0x7ffffff0, &rowc[buf][0][0]);
  };
  // after every wave's DMA of `buf` landed (vmcnt(0) + barrier): delta = rowsum(dO o O)
  auto finish = [&](int buf) {
    const int row = tid >> 3, c16 = tid & 7;  // 8 threads per query row
    const u32x4 o = *reinterpret_cast<const u32x4*>(Os + img16(row, c16));
    const u32x4 d = *reinterpret_cast<const u32x4*>(QO + (2 + buf) * BLK * D + img16(row, c16));
    float s = dot_bf16x8(o, d);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (c16 == 0) rowc[buf][1][row] = -s;  // stored negated: it seeds the dP accumulators
  };
  if (nqt > 0) issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nqt > 0) finish(0);
  __syncthreads();
  bstamp(1);

  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dk[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // this wave's 32 keys as MFMA B operands stay in registers for the whole query sweep (they
  // were re-read from LDS per 16-query tile: a third of the kernel's LDS traffic)
  bf16x8 kr[2][2], vr[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kr[j][ks] = frag_rows(Ks, key0 + 16 * j, ks, lane);
      vr[j][ks] = frag_rows(Vs, key0 + 16 * j, ks, lane);
    }
  const int qt = wave & 3, dt0 = 2 * (wave >> 2);
  int offtr[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) offtr[dt] = tr_off(16 * dt, lane);
  const int off_q = trS_off(16 * qt, lane);   // (dS^T image)
  const int off_k[2] = {tr_off(16 * dt0, lane), tr_off(16 * (dt0 + 1), lane)};
  // the query sweep as two instances: waves that never need a mask (the common case: Sq % 64 == 0,
  // all 32 keys valid, not causal) run one whose tiles are all unmasked -- with both tile variants
  // in one loop the compiler allocated dK / dV differently in each and copied all 64 accumulator
  // registers at their join on every query block.  Same trip count and barriers in both.
  const bool wave_mask = (a.Sq % BLK) != 0 || key0 + 32 > a.Sk || a.causal;
  auto sweep = [&](auto wm, auto vs) {
    constexpr bool WM = decltype(wm)::value;
    constexpr bool VS = decltype(vs)::value;  // dQ through dQs (compile-time: a runtime branch in
                                              // the sweep cost the loop its register allocation)
    for (int it = 0; it < nqt; ++it) {
      const int cur = it & 1;
      const int q0 = it * BLK;
      const bool more = it + 1 < nqt;
      if (more) issue(q0 + BLK, cur ^ 1);
      const bf16_t* Qt = QO + cur * BLK * D;
      const bf16_t* Ot = QO + (2 + cur) * BLK * D;
      if (active) {
        if constexpr (WM) {
          const bool need_mask = q0 + BLK > a.Sq || key0 + 32 > a.Sk || (a.causal && key0 + 31 > q0 + a.q_offset);
          if (need_mask) fused_tile<true>(a, Qt, Ot, rowc[cur][0], rowc[cur][1], dSt, kr, vr, dk, dv, q0, key0, lane, offtr);
          else fused_tile<false>(a, Qt, Ot, rowc[cur][0], rowc[cur][1], dSt, kr, vr, dk, dv, q0, key0, lane, offtr);
        } else {
          fused_tile<false>(a, Qt, Ot, rowc[cur][0], rowc[cur][1], dSt, kr, vr, dk, dv, q0, key0, lane, offtr);
        }
      }
      // this wave's DMA pieces of the next block landed; after the barrier everyone's have, so the
      // next block's delta is formed inside the dQ phase (two barriers per query block, not three)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (more) finish(cur ^ 1);
      // dQ^T (d tiles dt0, dt0+1) x queries 16qt..16qt+15 = K^T dS^T over all keys
      f32x4 dq[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      // unrolled over the at most FK / 32 key slices: every LDS address is a lane offset plus an
      // immediate (the rolled loop recomputed the swizzled addresses, 12 VALU per slice)
      if (LJS_ATTN_DQ_UNGUARD && nk32 == FK / 32) {
        // all key slices valid (Sk == 256): no per-slice guard, so the fragment reads of later
        // slices can issue ahead of earlier slices' MFMAs
  #pragma unroll
        for (int s2 = 0; s2 < FK / 32; ++s2) {
          bf16x8 sb = frag_tr_o(dSt, 32 * s2, off_q);
  #pragma unroll
          for (int i = 0; i < 2; ++i) {
            bf16x8 ka = frag_tr_o(Ks, 32 * s2, off_k[i]);
            dq[i] = mfma16x16x32(ka, sb, dq[i]);
          }
        }
      } else {
  #pragma unroll
        for (int s2 = 0; s2 < FK / 32; ++s2) {
          if (s2 < nk32) {
            bf16x8 sb = frag_tr_o(dSt, 32 * s2, off_q);
  #pragma unroll
            for (int i = 0; i < 2; ++i) {
              bf16x8 ka = frag_tr_o(Ks, 32 * s2, off_k[i]);
              dq[i] = mfma16x16x32(ka, sb, dq[i]);
            }
          }
        }
      }
      const int qrow = q0 + 16 * qt + (lane & 15);
      if constexpr (VS) {
        // the block's dQ is split over wave pairs (d halves): staged in dQs (16-byte chunk XOR
        // row), written as whole 128-byte rows after the barrier below
        const int r = 16 * qt + (lane & 15);
  #pragma unroll
        for (int i = 0; i < 2; ++i) {
          u32x2 w;
          w[0] = pack_bf16x2(dq[i][0] * a.scale, dq[i][1] * a.scale);
          w[1] = pack_bf16x2(dq[i][2] * a.scale, dq[i][3] * a.scale);
          const int c = (2 * (dt0 + i) + (g >> 1)) ^ (r & 7);
          *reinterpret_cast<u32x2*>(dQs + r * D + c * 8 + 4 * (g & 1)) = w;
        }
      } else if (qrow < a.Sq) {
        bf16_t* rowp = a.out3 + b * a.out3_sb + (long)qrow * a.out3_ss + h * a.out3_sh;
  #pragma unroll
        for (int i = 0; i < 2; ++i) {
          u32x2 w;
          w[0] = pack_bf16x2(dq[i][0] * a.scale, dq[i][1] * a.scale);
          w[1] = pack_bf16x2(dq[i][2] * a.scale, dq[i][3] * a.scale);
          *reinterpret_cast<u32x2*>(rowp + 16 * (dt0 + i) + 4 * g) = w;
        }
      }
      __syncthreads();
      if constexpr (VS) {
        // one 16-byte chunk per thread (64 rows x 8 chunks); the read completes before this
        // thread's store issues, i.e. before the next block's mid-sweep barrier (dQs reuse)
        const int r = tid >> 3, c = tid & 7;
        const u32x4 v = *reinterpret_cast<const u32x4*>(dQs + r * D + ((c ^ (r & 7)) << 3));
        if (q0 + r < a.Sq)
          *reinterpret_cast<u32x4*>(a.out3 + b * a.out3_sb + (long)(q0 + r) * a.out3_ss + h * a.out3_sh + c * 8) = v;
      }
      if (it < 5) bstamp(2 + it);
    }
  };
  if constexpr (SW == 1) {
    (void)wave_mask;
    sweep(std::false_type{}, std::true_type{});
  } else if (a.vst == 1) {  // (LJS_ATTN_VST=2: dK / dV staged, dQ per lane -- A/B)
    if (wave_mask) sweep(std::true_type{}, std::true_type{});
    else sweep(std::false_type{}, std::true_type{});
  } else {
    if (wave_mask) sweep(std::true_type{}, std::false_type{});
    else sweep(std::false_type{}, std::false_type{});
  }
  if (a.vst) {
    // every wave passed the sweep's last barrier: the K / V images are free; this wave's 32 key
    // rows of dK / dV go through its own rows of them
    if (active) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        stage_rows16(Ks + key0 * D, 16 * j, dk[j], a.scale, lane);
        stage_rows16(Vs + key0 * D, 16 * j, dv[j], 1.f, lane);
      }
      flush_rows<32>(Ks + key0 * D, a.out + b * a.out_sb + h * a.out_sh, a.out_ss, key0, a.Sk, lane);
      flush_rows<32>(Vs + key0 * D, a.out2 + b * a.out2_sb + h * a.out2_sh, a.out2_ss, key0, a.Sk, lane);
    }
    bstamp(7);
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int key = key0 + 16 * j + (lane & 15);
    if (key < a.Sk) {
      store_row_T(a.out + b * a.out_sb + (long)key * a.out_ss + h * a.out_sh, dk[j], a.scale, lane);
      store_row_T(a.out2 + b * a.out2_sb + (long)key * a.out2_ss + h * a.out2_sh, dv[j], 1.f, lane);
    }
  }
}

}  // namespace

// Kernel-variant switches.  The defaults are the measured winners (profiles/PERF_NOTES.md); the
// setters (ops/hip.py set_attention_*) exist so the GPU tests can run every variant and check it
// bit-exact against the default -- they are not environment knobs.
//  * split backward as ONE launch of dQ and dK/dV blocks (attn_bwd_pair_kernel), else two launches
static int g_bwd_pair = 1;
LJS_API void ljs_attn_set_bwd_pair(int v) { g_bwd_pair = v < 0 ? 1 : v; }
//  * 128-key dK/dV blocks in the split backward (S = 4096 step 1.50 -> 1.04 ms; B = 8, 256 keys:
//    0.0861-0.0873 -> 0.0852 ms), else 64-key blocks
static int g_dkv32 = 1;
LJS_API void ljs_attn_set_dkv32(int v) { g_dkv32 = v != 0; }
//  * 128-query dQ blocks beside the 128-key dK/dV blocks, else 64-query ones
static int g_dq32 = 1;
LJS_API void ljs_attn_set_dq32(int v) { g_dq32 = v != 0; }
//  * row tiles stored through LDS as whole 128-byte rows (1), per-lane 8-byte stores (0), or dK / dV
//    staged with per-lane dQ (2)
static int g_vst = 1;
LJS_API void ljs_attn_set_vst(int v) { g_vst = v < 0 ? 1 : v; }
static bool vst_ok(const void* p, const long* st) {
  return (((uintptr_t)p) & 15) == 0 && st[0] % 8 == 0 && st[1] % 8 == 0 && st[2] % 8 == 0;
}
static int g_attn_cus = 0;   // CUs of the current device (the fused projection's grid)
//  * K/V-resident forward for Sk <= 256: 8 (or 4) waves per block; 0 = the tiled kernel
static int g_fwd_res = 8;
LJS_API void ljs_attn_set_fwd_res(int v) { g_fwd_res = v < 0 ? 8 : v; }
//  * fused backward's K / V staging: 1 = LDS-DMA in flight with the first query block, 0 = register
//    copy, 2 = automatic (DMA for <= 128 queries per block)
static int g_bwd_kv_dma = 2;
LJS_API void ljs_attn_set_bwd_kv_dma(int v) { g_bwd_kv_dma = v < 0 ? 2 : v; }
//  * backward for Sk <= 256: 1 = fused single-pass kernel, 0 = split dQ + dK/dV kernels, 2 =
//    automatic by grid size
static int g_bwd_fused = 2;
LJS_API void ljs_attn_set_bwd_fused(int v) { g_bwd_fused = v < 0 ? 2 : v; }
//  * (diagnostic) the fused backward's phase-stamp buffer (LJS_ATTN_BWD_TRACE builds): [B][H][waves][8]
static unsigned long long* g_attn_trace = nullptr;
LJS_API void ljs_attn_set_trace(void* p) { g_attn_trace = (unsigned long long*)p; }

// strides are in elements, ordered (batch, seq, head); head_dim must be 64 and contiguous.
static int attn_fwd_impl(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Sq, int Sk,
                         int H, const long* qs, const long* ks, const long* vs, const long* os, float scale,
                         int causal, int q_offset, void* oacc, const long* oas, int acc_mode, hipStream_t stream) {
  AttnArgs a = {};
  a.oacc = (float*)oacc;
  a.acc_mode = acc_mode;
  if (oas) {
    a.oa_sb = oas[0]; a.oa_ss = oas[1]; a.oa_sh = oas[2];
  }
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.out = (bf16_t*)o;
  a.lse = (float*)lse;
  a.q_sb = qs[0]; a.q_ss = qs[1]; a.q_sh = qs[2];
  a.k_sb = ks[0]; a.k_ss = ks[1]; a.k_sh = ks[2];
  a.v_sb = vs[0]; a.v_ss = vs[1]; a.v_sh = vs[2];
  a.o_sb = os[0]; a.o_ss = os[1]; a.o_sh = os[2];
  a.Sq = Sq; a.Sk = Sk; a.H = H;
  a.scale = scale; a.scale_log2 = scale * LOG2E;
  a.causal = causal; a.q_offset = q_offset;
  a.vst = g_vst && vst_ok(o, os);
  if (g_fwd_res > 0 && Sk <= FKR && (long)(Sk - 1) * (ks[1] > vs[1] ? ks[1] : vs[1]) * 2 + 128 < (1L << 31)) {
    // 8 waves x 16 queries per block leave CUs idle below 256 blocks (B*H = 64 at the
    // reference shape): 4-wave blocks there (B=8: step 0.1069 -> 0.1057 ms).  (16-wave blocks,
    // a persistent double-buffered form, per-key-tile waits and two query sub-tiles per wave all
    // measured slower and were removed: PERF_NOTES rounds 2-5)
    int nw = g_fwd_res == 4 ? 4 : 8;
    if (nw == 8 && (Sq + 127) / 128 * H * B < 256) nw = 4;
    const int nqb = (Sq + 16 * nw - 1) / (16 * nw);
    a.fd_nx = make_fastdiv(nqb);
    a.fd_h = make_fastdiv(H);
    if (nw == 8) hipLaunchKernelGGL(attn_fwd_res_kernel<8>, dim3(nqb * H * B), dim3(512), 0, stream, a);
    else hipLaunchKernelGGL(attn_fwd_res_kernel<4>, dim3(nqb * H * B), dim3(256), 0, stream, a);
    return (int)hipGetLastError();
  }
  const int nqb = (Sq + BLK - 1) / BLK;
  hipLaunchKernelGGL(attn_fwd_kernel<1>, dim3(nqb * H * B), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

LJS_API int ljs_attn_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Sq, int Sk,
                         int H, const long* qs, const long* ks, const long* vs, const long* os, float scale,
                         int causal, int q_offset, hipStream_t stream) {
  return attn_fwd_impl(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, causal, q_offset, nullptr, nullptr, 0,
                       stream);
}

// blockwise forward with the running-output merge (ring attention's hop): acc_mode 1 / 2 / 3 (see
// AttnArgs); oacc f32 [.., d] with strides oas; lse read (modes 2, 3) and rewritten
LJS_API int ljs_attn_fwd_acc(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Sq, int Sk,
                             int H, const long* qs, const long* ks, const long* vs, const long* os, float scale,
                             int causal, int q_offset, void* oacc, const long* oas, int acc_mode, hipStream_t stream) {
  if (acc_mode < 1 || acc_mode > 3 || !oacc || !lse || (((uintptr_t)oacc) & 15) || oas[1] % 4 || oas[2] % 4 ||
      oas[0] % 4)
    return (int)hipErrorInvalidValue;
  return attn_fwd_impl(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, causal, q_offset, oacc, oas, acc_mode,
                       stream);
}


// fused Q/K/V projection + attention forward (qkv_attn_fwd_kernel): x [T][K] bf16 (row stride
// ldx), w [3][N][K] bf16 (the stacked transposed Q/K/V weights), N = H * 64, T = B * 256 tokens
// (sequence 256, batch-major rows); writes qkv [T][3N], o [T][N] ([B][256][H][64]) and lse
// [B][H][256] (log2 domain, as ljs_attn_fwd).  scale: the softmax scale.
LJS_API int ljs_qkv_attn_fwd(const void* x, long ldx, const void* w, void* qkv, void* o, void* lse, int T, int K, int N,
                             int H, float scale, void* trace, hipStream_t stream) {
  if (T <= 0 || T % QA_S || K < 2 * QA_BK || K % (2 * QA_BK) || N != H * D || H <= 0 || ldx < K || ldx % 8 ||
      (((uintptr_t)x | (uintptr_t)w | (uintptr_t)qkv | (uintptr_t)o) & 15) ||
      (long)T * ldx * 2 >= (1L << 31) || 3L * N * K * 2 >= (1L << 31))
    return (int)hipErrorInvalidValue;
  if (!g_attn_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_attn_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_attn_cus <= 0) g_attn_cus = 256;
  }
  QkvAttnArgs a;
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.qkv = (bf16_t*)qkv; a.o = (bf16_t*)o; a.lse = (float*)lse;
  a.T = T; a.K = K; a.N = N; a.H = H; a.ldx = (int)ldx;
  a.scale_log2 = scale * LOG2E;
  a.trace = (unsigned long long*)trace;
  const int items = T / QA_S * H;
  const int grid = items < g_attn_cus ? items : g_attn_cus;   // one 8-wave block per CU, items dealt round-robin
  hipLaunchKernelGGL(qkv_attn_fwd_kernel, dim3(grid), dim3(512), 0, stream, a);
  return (int)hipGetLastError();
}

// dq/dk/dv outputs get their own strides; delta is a [B][H][Sq] f32 workspace
LJS_API int ljs_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const void* lse, void* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int H,
                         const long* qs, const long* ks, const long* vs, const long* os, const long* dos,
                         const long* dqs, const long* dks, const long* dvs, float scale, int causal, int q_offset,
                         hipStream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (const bf16_t*)o;
  a.dout = (const bf16_t*)dout;
  a.lse = (float*)lse; a.delta = (const float*)delta;
  a.q_sb = qs[0]; a.q_ss = qs[1]; a.q_sh = qs[2];
  a.k_sb = ks[0]; a.k_ss = ks[1]; a.k_sh = ks[2];
  a.v_sb = vs[0]; a.v_ss = vs[1]; a.v_sh = vs[2];
  a.o_sb = os[0]; a.o_ss = os[1]; a.o_sh = os[2];
  a.do_sb = dos[0]; a.do_ss = dos[1]; a.do_sh = dos[2];
  a.Sq = Sq; a.Sk = Sk; a.H = H;
  a.scale = scale; a.scale_log2 = scale * LOG2E;
  a.causal = causal; a.q_offset = q_offset;
  // 2 = automatic: the fused kernel runs one workgroup per (batch, head), so below ~half a
  // workgroup per CU (B*H < 128: the reference's B = 8 x 8 heads) the split kernels' per-query-
  // block grids fill the chip better (measured: 0.1218 vs 0.1248 ms/step at B = 8, equal at 16,
  // fused far ahead from 32)
  const bool fused = g_bwd_fused == 1 || (g_bwd_fused == 2 && (long)B * H >= 128);
  if (fused && Sk <= FK) {
    AttnArgs f = a;
    f.out = (bf16_t*)dk; f.out_sb = dks[0]; f.out_ss = dks[1]; f.out_sh = dks[2];
    f.out2 = (bf16_t*)dv; f.out2_sb = dvs[0]; f.out2_ss = dvs[1]; f.out2_sh = dvs[2];
    f.out3 = (bf16_t*)dq; f.out3_sb = dqs[0]; f.out3_ss = dqs[1]; f.out3_sh = dqs[2];
    f.vst = vst_ok(dk, dks) && vst_ok(dv, dvs) && vst_ok(dq, dqs) ? g_vst : 0;
    f.trace = g_attn_trace;
    // 2 = automatic: the DMA form when a block sweeps at most two query blocks (the 2-D mesh's
    // 128 local queries against 256 gathered keys: the K / V prologue is a third of the block's
    // time there, and overlapping it with the first query block's loads measured 58.8 -> 57.1 us,
    // 2-D rehearsal step 0.2963 -> 0.2937 ms median, gpurun_out/r4ab); at 256 queries it is
    // neutral (0.2194 vs 0.2196 ms), so the register copy stays there
    const bool kv_dma = g_bwd_kv_dma == 1 || (g_bwd_kv_dma == 2 && Sq <= 2 * BLK);
    const bool sw1 = f.vst == 1 && Sq % BLK == 0 && Sk == FK && !causal;
    if (kv_dma && sw1) hipLaunchKernelGGL((attn_bwd_fused_kernel<true, 1>), dim3(H, B), dim3(FT), 0, stream, f);
    else if (kv_dma) hipLaunchKernelGGL((attn_bwd_fused_kernel<true, 0>), dim3(H, B), dim3(FT), 0, stream, f);
    else if (sw1) hipLaunchKernelGGL((attn_bwd_fused_kernel<false, 1>), dim3(H, B), dim3(FT), 0, stream, f);
    else hipLaunchKernelGGL((attn_bwd_fused_kernel<false, 0>), dim3(H, B), dim3(FT), 0, stream, f);
    return (int)hipGetLastError();
  }
  AttnArgs c = a;
  c.out = (bf16_t*)dq; c.out_sb = dqs[0]; c.out_ss = dqs[1]; c.out_sh = dqs[2];
  c.vst = g_vst && vst_ok(dq, dqs);  // (the 128-query dQ blocks use it)
  AttnArgs b = a;
  b.out = (bf16_t*)dk; b.out_sb = dks[0]; b.out_ss = dks[1]; b.out_sh = dks[2];
  b.out2 = (bf16_t*)dv; b.out2_sb = dvs[0]; b.out2_ss = dvs[1]; b.out2_sh = dvs[2];
  b.vst = g_vst && vst_ok(dk, dks) && vst_ok(dv, dvs);  // (the 128-key dK/dV blocks use it)
  const long nq = (Sq + BLK - 1) / BLK, nk = (Sk + BLK - 1) / BLK;
  if (g_dkv32 && (nq + (Sk + 127) / 128) * H * B < (1L << 30)) {
    const long nk128 = (Sk + 127) / 128;
    c.flags32 = g_dq32;
    const long nqb = c.flags32 ? (Sq + 127) / 128 : nq;
    hipLaunchKernelGGL(attn_bwd_pair32_kernel, dim3((unsigned)((nqb + nk128) * H * B)), dim3(256), 0, stream, c, b);
    return (int)hipGetLastError();
  }
  if (g_bwd_pair && (nq + nk) * H * B < (1L << 30)) {
    // one launch: dQ blocks and dK/dV blocks (which form delta themselves) side by side
    hipLaunchKernelGGL(attn_bwd_pair_kernel, dim3((unsigned)((nq + nk) * H * B)), dim3(256), 0, stream, c, b);
    return (int)hipGetLastError();
  }
  // dQ first: it also computes delta, which the dK/dV kernel consumes (stream order)
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(nq * H * B), dim3(256), 0, stream, c);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel, dim3(nk * H * B), dim3(256), 0, stream, b);
  return (int)hipGetLastError();
}
