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
// Tensors are (batch, seq, heads, 64) with arbitrary batch/seq/head strides (d contiguous),
// so Q/K/V can be column slices of the fused QKV GEMM output.
#include "common.h"

namespace {

constexpr int D = 64;      // head dim
constexpr int BLK = 64;    // queries / keys per tile
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* o; const bf16_t* dout;
  bf16_t* out;                     // fwd: O ; bwd dkv: dK ; bwd dq: dQ
  bf16_t* out2;                    // bwd dkv: dV
  float* lse;                      // [B][H][Sq], log2 domain of scaled scores
  const float* delta;              // [B][H][Sq]
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh;
  long do_sb, do_ss, do_sh, out_sb, out_ss, out_sh, out2_sb, out2_ss, out2_sh;
  int Sq, Sk, H;
  float scale, scale_log2;
  int causal, q_offset;
};

// ---- LDS images: [64 rows][64 d] bf16, 128-byte rows
// k-contiguous row reads (ds_read_b128) + transposed reads: 16-byte chunk XOR (row>>1)&7
__device__ __forceinline__ int img_k(int row, int c16) { return row * D + ((c16 ^ ((row >> 1) & 7)) << 3); }
// transposed reads only: 8-byte chunk XOR 4*((row>>1)&3) (conflict-free tr_b16 reads)
__device__ __forceinline__ int img_t(int row, int c8) { return row * D + ((c8 ^ (((row >> 1) & 3) << 2)) << 2); }

template <bool TR_ONLY>
__device__ __forceinline__ int img_chunk16(int row, int c16) {
  if constexpr (TR_ONLY) return img_t(row, c16 * 2);
  else return img_k(row, c16);
}

template <bool TR_ONLY>
__device__ __forceinline__ int img_chunk8(int row, int c8) {
  if constexpr (TR_ONLY) return img_t(row, c8);
  else return row * D + (((c8 >> 1) ^ ((row >> 1) & 7)) << 3) + ((c8 & 1) << 2);
}

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
  template <bool TR_ONLY>
  __device__ __forceinline__ void store(bf16_t* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + 256 * i, row = c >> 3, c16 = c & 7;
      *reinterpret_cast<u32x4*>(lds + img_chunk16<TR_ONLY>(row, c16)) = v[i];
    }
  }
};

// MFMA operand from rows [rb, rb+16) of a k-contiguous image, k-step ks (d 32ks..32ks+31)
__device__ __forceinline__ bf16x8 frag_rows(const bf16_t* lds, int rb, int ks, int lane) {
  int row = rb + (lane & 15);
  int c16 = ks * 4 + (lane >> 4);
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + img_k(row, c16)));
}

// MFMA A operand A[m = d][k = row]: d = db + (lane&15); elements 0..3 = rows base0+0..3,
// elements 4..7 = rows base1+0..3 (base0/base1 already include the lane group's offset)
template <bool TR_ONLY>
__device__ __forceinline__ bf16x8 frag_tr(const bf16_t* lds, int base0, int base1, int db, int lane) {
  int i = lane & 15, q = i >> 2, p = i & 3;
  int c8 = (db >> 2) + p;
  s16x4 lo = lds_read_tr16(lds + img_chunk8<TR_ONLY>(base0 + q, c8));
  s16x4 hi = lds_read_tr16(lds + img_chunk8<TR_ONLY>(base1 + q, c8));
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

// ============================================================================ forward
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
#define Ks(i) (smem + (i) * BLK * D)
#define Vs(i) (smem + (2 + (i)) * BLK * D)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int qrow = qb * BLK + wave * 16 + (lane & 15);
  const bool qok = qrow < a.Sq;

  const bf16_t* qp = a.q + b * a.q_sb + (long)qrow * a.q_ss + h * a.q_sh;
  bf16x8 qf[2] = {load_row_frag(qp, qok, 0, lane), load_row_frag(qp, qok, 1, lane)};
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;

  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, a.q_offset + (qb + 1) * BLK);
  const int nkt = (kend + BLK - 1) / BLK;

  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  TileRegs tk, tv;
  if (nkt > 0) {
    tk.load(kb, a.k_ss, 0, a.Sk, tid);
    tv.load(vb, a.v_ss, 0, a.Sk, tid);
    tk.store<false>(Ks(0), tid);
    tv.store<true>(Vs(0), tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      tk.load(kb, a.k_ss, (kt + 1) * BLK, a.Sk, tid);
      tv.load(vb, a.v_ss, (kt + 1) * BLK, a.Sk, tid);
    }
    // S^T = K Q^T : rows = keys (16jt + 4g + r), col = this lane's query
    f32x4 s[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      s[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) s[jt] = mfma16x16x32(frag_rows(Ks(cur), 16 * jt, ks, lane), qf[ks], s[jt]);
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = kt * BLK + 16 * jt + 4 * g + r;
        float x = s[jt][r] * a.scale_log2;
        bool masked = key >= a.Sk || (a.causal && key > qrow + a.q_offset);
        x = masked ? -INFINITY : x;
        s[jt][r] = x;
        tmax = fmaxf(tmax, x);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m, tmax);
    const bool dead = m_new == -INFINITY;
    const float alpha = dead ? 1.f : exp2f(m - m_new);
    float psum = 0.f;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = dead ? 0.f : exp2f(s[jt][r] - m_new);
        s[jt][r] = pv;
        psum += pv;
      }
    l = l * alpha + psum;
    m = m_new;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    // O^T += V^T P^T
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 pb = frag_acc(s[2 * s2], s[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 va = frag_tr<true>(Vs(cur), 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
        o[dt] = mfma16x16x32(va, pb, o[dt]);
      }
    }
    if (more) {
      tk.store<false>(Ks(cur ^ 1), tid);
      tv.store<true>(Vs(cur ^ 1), tid);
    }
    __syncthreads();
  }
  float lt = l;
  lt += __shfl_xor(lt, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  if (qok) {
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    bf16_t* op = a.out + b * a.o_sb + (long)qrow * a.o_ss + h * a.o_sh;
    store_row_T(op, o, inv, lane);
    if (g == 0 && a.lse) a.lse[((long)b * a.H + h) * a.Sq + qrow] = lt > 0.f ? m + log2f(lt) : INFINITY;
  }
}

// ============================================================================ backward
// delta[q] = sum_d dO[q][d] * O[q][d]   (one wave handles 64 rows, one lane per row)
__global__ void attn_bwd_delta_kernel(AttnArgs a) {
  const int b = blockIdx.z, h = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= a.Sq) return;
  const bf16_t* op = a.o + b * a.o_sb + (long)q * a.o_ss + h * a.o_sh;
  const bf16_t* dp = a.dout + b * a.do_sb + (long)q * a.do_ss + h * a.do_sh;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    u32x4 x = *reinterpret_cast<const u32x4*>(op + 8 * c);
    u32x4 y = *reinterpret_cast<const u32x4*>(dp + 8 * c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s += __uint_as_float(x[k] << 16) * __uint_as_float(y[k] << 16);
      s += __uint_as_float(x[k] & 0xffff0000u) * __uint_as_float(y[k] & 0xffff0000u);
    }
  }
  const_cast<float*>(a.delta)[((long)b * a.H + h) * a.Sq + q] = s;
}

// dK, dV for one 64-key block (each wave: 16 keys), sweeping all query blocks
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
#define Qs(i) (smem + (i) * BLK * D)
#define Os(i) (smem + (2 + (i)) * BLK * D)  // dO tiles
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int kblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int key = kblk * BLK + wave * 16 + (lane & 15);
  const bool kok = key < a.Sk;
  const bf16_t* kp = a.k + b * a.k_sb + (long)key * a.k_ss + h * a.k_sh;
  const bf16_t* vp = a.v + b * a.v_sb + (long)key * a.v_ss + h * a.v_sh;
  bf16x8 kf[2] = {load_row_frag(kp, kok, 0, lane), load_row_frag(kp, kok, 1, lane)};
  bf16x8 vf[2] = {load_row_frag(vp, kok, 0, lane), load_row_frag(vp, kok, 1, lane)};
  const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* ob = a.dout + b * a.do_sb + h * a.do_sh;
  const float* lse = a.lse + ((long)b * a.H + h) * a.Sq;
  const float* delta = a.delta + ((long)b * a.H + h) * a.Sq;

  int qstart = 0;
  if (a.causal) qstart = max(0, (kblk * BLK - a.q_offset) / BLK * BLK);
  const int nqt = (a.Sq - qstart + BLK - 1) / BLK;

  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  TileRegs tq, tdo;
  if (nqt > 0) {
    tq.load(qb, a.q_ss, qstart, a.Sq, tid);
    tdo.load(ob, a.do_ss, qstart, a.Sq, tid);
    tq.store<false>(Qs(0), tid);
    tdo.store<false>(Os(0), tid);
  }
  __syncthreads();
  for (int it = 0; it < nqt; ++it) {
    const int cur = it & 1;
    const int q0 = qstart + it * BLK;
    const bool more = it + 1 < nqt;
    if (more) {
      tq.load(qb, a.q_ss, q0 + BLK, a.Sq, tid);
      tdo.load(ob, a.do_ss, q0 + BLK, a.Sq, tid);
    }
    // S = Q K^T (rows = queries 16t + 4g + r, col = this lane's key); P; dP = dO V^T; dS
    f32x4 p[4], ds[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s = mfma16x16x32(frag_rows(Qs(cur), 16 * t, ks, lane), kf[ks], s);
        dp = mfma16x16x32(frag_rows(Os(cur), 16 * t, ks, lane), vf[ks], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int q = q0 + 16 * t + 4 * g + r;
        bool ok = q < a.Sq && kok && !(a.causal && key > q + a.q_offset);
        float pv = ok ? exp2f(s[r] * a.scale_log2 - lse[q]) : 0.f;
        float dl = ok ? delta[q] : 0.f;
        p[t][r] = pv;
        ds[t][r] = pv * (dp[r] - dl);
      }
    }
    // dV^T += dO^T P ; dK^T += Q^T dS   (k = queries)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 pb = frag_acc(p[2 * s2], p[2 * s2 + 1]);
      bf16x8 sb = frag_acc(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 oa = frag_tr<false>(Os(cur), 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
        dv[dt] = mfma16x16x32(oa, pb, dv[dt]);
        bf16x8 qa = frag_tr<false>(Qs(cur), 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
        dk[dt] = mfma16x16x32(qa, sb, dk[dt]);
      }
    }
    if (more) {
      tq.store<false>(Qs(cur ^ 1), tid);
      tdo.store<false>(Os(cur ^ 1), tid);
    }
    __syncthreads();
  }
  if (kok) {
    store_row_T(a.out + b * a.out_sb + (long)key * a.out_ss + h * a.out_sh, dk, a.scale, lane);
    store_row_T(a.out2 + b * a.out2_sb + (long)key * a.out2_ss + h * a.out2_sh, dv, 1.f, lane);
  }
}

// dQ for one 64-query block (each wave: 16 queries), sweeping key blocks
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * BLK * D];
#define Ks(i) (smem + (i) * BLK * D)
#define Vs(i) (smem + (2 + (i)) * BLK * D)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int qrow = qb * BLK + wave * 16 + (lane & 15);
  const bool qok = qrow < a.Sq;
  const bf16_t* qp = a.q + b * a.q_sb + (long)qrow * a.q_ss + h * a.q_sh;
  const bf16_t* dop = a.dout + b * a.do_sb + (long)qrow * a.do_ss + h * a.do_sh;
  bf16x8 qf[2] = {load_row_frag(qp, qok, 0, lane), load_row_frag(qp, qok, 1, lane)};
  bf16x8 df[2] = {load_row_frag(dop, qok, 0, lane), load_row_frag(dop, qok, 1, lane)};
  const float lse_q = qok ? a.lse[((long)b * a.H + h) * a.Sq + qrow] : 0.f;
  const float dl_q = qok ? a.delta[((long)b * a.H + h) * a.Sq + qrow] : 0.f;
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  int kend = a.Sk;
  if (a.causal) kend = min(a.Sk, a.q_offset + (qb + 1) * BLK);
  const int nkt = (kend + BLK - 1) / BLK;

  f32x4 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  TileRegs tk, tv;
  if (nkt > 0) {
    tk.load(kb, a.k_ss, 0, a.Sk, tid);
    tv.load(vb, a.v_ss, 0, a.Sk, tid);
    tk.store<false>(Ks(0), tid);
    tv.store<false>(Vs(0), tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      tk.load(kb, a.k_ss, (kt + 1) * BLK, a.Sk, tid);
      tv.load(vb, a.v_ss, (kt + 1) * BLK, a.Sk, tid);
    }
    f32x4 ds[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s = mfma16x16x32(frag_rows(Ks(cur), 16 * jt, ks, lane), qf[ks], s);
        dp = mfma16x16x32(frag_rows(Vs(cur), 16 * jt, ks, lane), df[ks], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = kt * BLK + 16 * jt + 4 * g + r;
        bool ok = qok && key < a.Sk && !(a.causal && key > qrow + a.q_offset);
        float pv = ok ? exp2f(s[r] * a.scale_log2 - lse_q) : 0.f;
        ds[jt][r] = pv * (dp[r] - dl_q);
      }
    }
    // dQ^T += K^T dS^T   (k = keys)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 sb = frag_acc(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 ka = frag_tr<false>(Ks(cur), 32 * s2 + 4 * g, 32 * s2 + 16 + 4 * g, 16 * dt, lane);
        dq[dt] = mfma16x16x32(ka, sb, dq[dt]);
      }
    }
    if (more) {
      tk.store<false>(Ks(cur ^ 1), tid);
      tv.store<false>(Vs(cur ^ 1), tid);
    }
    __syncthreads();
  }
  if (qok) store_row_T(a.out + b * a.out_sb + (long)qrow * a.out_ss + h * a.out_sh, dq, a.scale, lane);
}

#undef Ks
#undef Vs
#undef Qs
#undef Os
}  // namespace

// strides are in elements, ordered (batch, seq, head); head_dim must be 64 and contiguous.
LJS_API int ljs_attn_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Sq, int Sk,
                         int H, const long* qs, const long* ks, const long* vs, const long* os, float scale,
                         int causal, int q_offset, hipStream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.out = (bf16_t*)o;
  a.lse = (float*)lse;
  a.q_sb = qs[0]; a.q_ss = qs[1]; a.q_sh = qs[2];
  a.k_sb = ks[0]; a.k_ss = ks[1]; a.k_sh = ks[2];
  a.v_sb = vs[0]; a.v_ss = vs[1]; a.v_sh = vs[2];
  a.o_sb = os[0]; a.o_ss = os[1]; a.o_sh = os[2];
  a.Sq = Sq; a.Sk = Sk; a.H = H;
  a.scale = scale; a.scale_log2 = scale * LOG2E;
  a.causal = causal; a.q_offset = q_offset;
  dim3 grid((Sq + BLK - 1) / BLK, H, B);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, stream, a);
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
  hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((Sq + 255) / 256, H, B), dim3(256), 0, stream, a);
  // dK, dV
  AttnArgs b = a;
  b.out = (bf16_t*)dk; b.out_sb = dks[0]; b.out_ss = dks[1]; b.out_sh = dks[2];
  b.out2 = (bf16_t*)dv; b.out2_sb = dvs[0]; b.out2_ss = dvs[1]; b.out2_sh = dvs[2];
  hipLaunchKernelGGL(attn_bwd_dkv_kernel, dim3((Sk + BLK - 1) / BLK, H, B), dim3(256), 0, stream, b);
  // dQ
  AttnArgs c = a;
  c.out = (bf16_t*)dq; c.out_sb = dqs[0]; c.out_ss = dqs[1]; c.out_sh = dqs[2];
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((Sq + BLK - 1) / BLK, H, B), dim3(256), 0, stream, c);
  return (int)hipGetLastError();
}
