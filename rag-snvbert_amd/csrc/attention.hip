// Unmasked multi-head attention, flash-style (no L x L score matrix in HBM).
//
// Reference: model/attention/attention.py:21-31 (softmax(QK^T/sqrt(dh)) V, no
// mask — padding tokens participate) with the head split/merge of
// multi_head_attention.py:44-51.  L = 1030 for every v18 configuration.
//
// Head dim 32 (every v18 model: d384/H12, d128/H4, d64/H2): attn32_dma below.  Other head
// dims: attn_fwd_bf16 (v_mfma_f32_16x16x32_bf16), one workgroup = 4 waves = 64 queries of
// one (sequence, head); each wave owns 16 queries.  Scores are computed
// TRANSPOSED, S^T = K Q^T, so each lane holds one query's column of scores and
// the softmax row statistics need only 2 cross-lane shuffles; P^T then feeds
// the O^T = V^T P^T MFMA as the B operand straight from the accumulators
// (key order permuted consistently on the V^T side).  K is staged row-major
// (XOR-swizzled for conflict-free 16-lane reads), V transposed, both double
// buffered with register prefetch of the next 64-key tile.
//
// f32 path: exact-f32 VALU online softmax, one thread per query (parity mode).
#include "attn_common.h"

namespace snvrag {

template <int DH>
__global__ __launch_bounds__(256) void attn_fwd_bf16(int nseq, int L, int H, const bf16* __restrict__ qkv,
                                                     long ld, bf16* __restrict__ out, long ldo,
                                                     float scale_log2e, int nqb, float* __restrict__ lse,
                                                     AttnDrop drop) {
  using C = AttnCfg<DH>;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::STAGE];

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int qq = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int qb = wg % nqb, sh = wg / nqb, h = sh % H, seq = sh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const long base = (long)seq * L * ld;
  const int D = H * DH;
  const bf16* Qp = qkv + base + h * DH;
  const bf16* Kp = qkv + base + D + h * DH;
  const bf16* Vp = qkv + base + 2 * D + h * DH;

  // Q fragment (B operand of S^T = K Q^T): lane -> query q0+li, d = 32*ks + 8*lg + j
  const int q = qb * AQ + wave * 16 + li;
  bf16x8 qf[C::KS];
#pragma unroll
  for (int ks = 0; ks < C::KS; ++ks) {
    const int d0 = 32 * ks + 8 * lg;
    if (q < L && d0 < DH)
      qf[ks] = *reinterpret_cast<const bf16x8*>(Qp + (long)q * ld + d0);
    else
      qf[ks] = bf16x8{};
  }

  // tile loader: thread -> (key, 16-B chunk) for K and V; rows beyond L / DH are zero
  constexpr int CH = C::CPR;                               // chunks per key (padded)
  constexpr int NLD = (AK * CH + 255) / 256;
  u32x4 kr[NLD], vr[NLD];
  auto load_tile = [&](int t0) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int id = tid + 256 * i;
      const int key = id / CH, c = id % CH;
      const int kk = t0 + key, d0 = 8 * c;
      if (id < AK * CH && kk < L && d0 < DH) {
        kr[i] = *reinterpret_cast<const u32x4*>(Kp + (long)kk * ld + d0);
        vr[i] = *reinterpret_cast<const u32x4*>(Vp + (long)kk * ld + d0);
      } else {
        kr[i] = u32x4{0u, 0u, 0u, 0u};
        vr[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto store_tile = [&](char* st) {
    bf16* vt = reinterpret_cast<bf16*>(st + C::KBYTES);
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int id = tid + 256 * i;
      if (id < AK * CH) {
        const int key = id / CH, c = id % CH;
        *reinterpret_cast<u32x4*>(st + k_off<DH>(key, c)) = kr[i];
        const bf16x8 v = __builtin_bit_cast(bf16x8, vr[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) vt[(8 * c + j) * C::VT_LD + key] = v[j];
      }
    }
  };

  f32x4 o[C::ET];
#pragma unroll
  for (int e = 0; e < C::ET; ++e) o[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int ntile = (L + AK - 1) / AK;
  load_tile(0);
  store_tile(smem);
  __syncthreads();

  for (int t = 0; t < ntile; ++t) {
    char* st = smem + (t & 1) * C::STAGE;
    const bool more = t + 1 < ntile;
    if (more) load_tile((t + 1) * AK);

    // ---- S^T tile: 4 x (16 keys x 16 queries) ----
    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int key = 16 * kt + li;
#pragma unroll
      for (int ks = 0; ks < C::KS; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(st + k_off<DH>(key, 4 * ks + lg));
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[kt], 0, 0, 0);
      }
    }
    // ---- online softmax over the 64 keys of this tile (per query = per lane column) ----
    const int kbase = t * AK;
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kbase + 16 * kt + 4 * lg + r;
        float v = s[kt][r] * scale_log2e;
        v = key < L ? v : -INFINITY;
        s[kt][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = exp2f(m_run - m_new);
    float psum = 0.f;
    bf16x8 pb[2];
    if (drop.thresh) {
      // training dropout: the row sum keeps every probability, the PV product the kept ones
      const uint32_t dbase = drop_base(drop.seed, (uint32_t)sh);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          float dm[2];
          drop_mul2(drop, dbase, (uint32_t)q, (uint32_t)(kbase + 16 * kt + 4 * lg + r), dm[0], dm[1]);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float p = exp2f(s[kt][r + e] - m_new);
            psum += p;
            pb[kt >> 1][(kt & 1) * 4 + r + e] = (bf16)(p * dm[e]);
          }
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[kt][r] - m_new);
          psum += p;
          pb[kt >> 1][(kt & 1) * 4 + r] = (bf16)p;
        }
    }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int e = 0; e < C::ET; ++e) o[e] *= alpha;

    // ---- O^T += V^T P^T : keys of MFMA c in the order the accumulators hold them ----
    const bf16* vt = reinterpret_cast<const bf16*>(st + C::KBYTES);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int e = 0; e < C::ET; ++e) {
        const bf16* row = vt + (16 * e + li) * C::VT_LD + 32 * c + 4 * lg;
        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(row);
        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(row + 16);
        const bf16x8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        o[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[c], o[e], 0, 0, 0);
      }
    }
    if (more) store_tile(smem + ((t + 1) & 1) * C::STAGE);
    __syncthreads();
  }

  if (q < L) {
    const float inv = 1.0f / l_run;
    // training: per-row log2-sum-exp of the scaled scores, P = exp2(s*c - lse) in the backward
    if (lse && lg == 0) lse[((long)seq * H + h) * L + q] = m_run + log2f(l_run);
    bf16* op = out + (long)seq * L * ldo + (long)q * ldo + h * DH;
#pragma unroll
    for (int e = 0; e < C::ET; ++e) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[e][r] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * e + 4 * lg) = w;
    }
  }
}

// ------------------------------------------------------- bf16, head dim 32 --
// attn32: one workgroup = 4 waves x 32 queries (two 16-query MFMA column tiles per
// wave, sharing every K / V^T fragment read) of one (sequence, head); K/V stream
// through LDS in 64-key tiles, register-staged and double buffered (loads of tile
// t+1 in flight under tile t's MFMAs).  At dh = 32 the exp, not the MFMA, bounds
// the loop, so the softmax VALU is cut to one v_exp_f32 + half a cvt per score:
//  * Q arrives pre-scaled by log2(e)/sqrt(dh) (folded into W_q by the engine), or is
//    scaled once when loaded;
//  * the shift is fixed per query after the first key tile (m_q = exact max of
//    tile 0) and enters as the MFMA's C operand (S^T = K Q^T - m_q), so later
//    tiles run no max, no subtraction and no O rescale (softmax is shift-invariant;
//    m_q <= the true max, so the dominant terms never underflow);
//  * the row sum l_q comes out of an extra MFMA against a ones matrix (same
//    bf16-rounded P that multiplies V).
// If a later score exceeds m_q by more than f32 can hold (l or O not finite), that
// wave recomputes its queries with an exact online-max softmax straight from global
// memory (attn32_online) — correctness never depends on the data range.
namespace a32 {
constexpr int QPW = 32, WAVES = 4, QPB = QPW * WAVES, KT = 64;
constexpr int TB = KT * 64;                        // one K or V tile: 64 keys x 64 B
// K tile: 64-B rows, chunk XOR (-(key>>2))&3 — conflict-free for the ds_read_b128 lane groups
__device__ __forceinline__ int k_off(int key, int chunk) { return key * 64 + ((chunk ^ ((-(key >> 2)) & 3)) << 4); }
// V tile: 64-B rows, 32-B halves swapped on (key>>2)&1 — conflict-free ds_read_b64_tr_b16
__device__ __forceinline__ int v_off(int key, int half) { return key * 64 + ((half ^ ((key >> 2) & 1)) << 5); }
__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

struct State {
  f32x4 o[2][2];     // [e][qt]: O^T rows 16e + 4lg + r, query column li
  f32x4 ls[2];       // [qt]: row sums (all four entries equal)
  f32x4 negm[2];     // [qt]: -m_q broadcast (MFMA C operand)
};

// Training (TRAIN): Q is unscaled (no bf16 rounding of Q * scale, so the backward's recomputed
// P = exp2(c s - lse) matches), the shift m_q is in unscaled score units and p = exp2(c (s - m_q));
// with dropout the PV operand is bf16(p * keep / (1 - p_drop)) while the row sum keeps every p.
struct Train {
  float c;            // scale * log2(e)
  AttnDrop drop;
  uint32_t dbase;     // drop_base(seed, seq * H + h)
  int q0;             // the wave's first query
};

struct NoMid {
  __device__ void operator()() const {}
};

// One 64-key tile for a wave's 32 queries.  VAR (inference A/B, snvrag option attn_variant):
//   0  as described above;
//   1  the PV + row-sum MFMA block at s_setprio 2 (a wave with MFMAs to issue wins the SIMD's
//      issue arbitration over the co-resident waves' exp streams);
//   2  like 1, and the S MFMAs at the head of the tile as well;
//   3  K fragments passed in ``kin`` (read one tile ahead by the caller) and ``mid`` run between
//      the exps and the PV block (the caller's ring barrier + next-tile K prefetch);
//   5  the V^T fragments read right after the S MFMAs (LDS latency under the exps).
template <int NKT, bool MASK, bool FIRST, bool TRAIN = false, int VAR = 0, typename Mid = NoMid>
__device__ __forceinline__ void tile(const char* Kt, const char* Vt, int kbase, int L, const bf16x8 (&qf)[2],
                                     State& st, int li, int lg, const Train& tr = Train{},
                                     const bf16x8* kin = nullptr, Mid mid = Mid{}) {
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 s[NKT][2];
  if constexpr (VAR == 2) __builtin_amdgcn_s_setprio(2);
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const bf16x8 kf = VAR == 3 ? kin[kt] : *reinterpret_cast<const bf16x8*>(Kt + k_off(16 * kt + li, lg));
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt], FIRST ? zero : st.negm[qt], 0, 0, 0);
  }
  if constexpr (VAR == 2) __builtin_amdgcn_s_setprio(0);
  if constexpr (MASK) {
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (kbase + 16 * kt + 4 * lg + r >= L) {
          s[kt][0][r] = -INFINITY;
          s[kt][1][r] = -INFINITY;
        }
  }
  if constexpr (FIRST) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      st.negm[qt] = f32x4{-mx, -mx, -mx, -mx};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) s[kt][qt] += st.negm[qt];
    }
  }
  constexpr int NCB = (NKT + 1) / 2;
  const int tq = li >> 2, tp = li & 3;          // ds_read_b64_tr_b16: lane 4q+p -> row q, columns 4p..4p+3
  // VAR 5: the V^T fragments read right after the S MFMAs, their LDS latency under the exps
  bf16x8 vpre[VAR == 5 ? NCB : 1][2];
  if constexpr (VAR == 5) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int k0 = 32 * cb + 4 * lg + tq;
        vpre[cb][e] = cat(tr_read(Vt + v_off(k0, e) + 8 * tp), tr_read(Vt + v_off(k0 + 16, e) + 8 * tp));
      }
  }
  bf16x8 pb[NCB][2];
  bf16x8 pd[TRAIN ? NCB : 1][2];                 // TRAIN: the dropped-out PV operand
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kt = 2 * cb + (j >> 2);
        if constexpr (TRAIN)
          pb[cb][qt][j] = kt < NKT ? (bf16)__builtin_amdgcn_exp2f(tr.c * s[kt < NKT ? kt : 0][qt][j & 3]) : (bf16)0.f;
        else
          pb[cb][qt][j] = kt < NKT ? (bf16)__builtin_amdgcn_exp2f(s[kt < NKT ? kt : 0][qt][j & 3]) : (bf16)0.f;
      }
  if constexpr (TRAIN) {
    // dropout: keys 2i, 2i + 1 (one packed dword of P) share one hash; the kept halves pass the
    // AND, the 1 / (1 - p) scale is applied to O after the loop.  Hash input of (query
    // 16 qt + li, this lane's first key pair (kbase + 4 lg) / 2); dword i of block cb adds the
    // pair offset 8 kt + (i & 1), kt = 2 cb + i / 2
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const uint32_t drow = drop_row(tr.dbase, (uint32_t)(tr.q0 + 16 * qt + li), (uint32_t)((kbase >> 1) + 2 * lg));
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        u32x4 w = __builtin_bit_cast(u32x4, pb[cb][qt]);
        if (tr.drop.thresh) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            w[i] = drop_pair_apply(w[i], drop_mix24(drow + (uint32_t)(8 * (2 * cb + (i >> 1)) + (i & 1)) * DROP_C2),
                                   tr.drop.thresh);
        }
        pd[cb][qt] = __builtin_bit_cast(bf16x8, w);
      }
    }
  }
  mid();
  const bf16x8 ones = {(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};
  if constexpr (VAR == 1 || VAR == 2) __builtin_amdgcn_s_setprio(2);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int k0 = 32 * cb + 4 * lg + tq;
      const bf16x8 vf = VAR == 5 ? vpre[VAR == 5 ? cb : 0][e]
                                 : cat(tr_read(Vt + v_off(k0, e) + 8 * tp), tr_read(Vt + v_off(k0 + 16, e) + 8 * tp));
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        st.o[e][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, TRAIN ? pd[TRAIN ? cb : 0][qt] : pb[cb][qt],
                                                               st.o[e][qt], 0, 0, 0);
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) st.ls[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[cb][qt], st.ls[qt], 0, 0, 0);
  }
  if constexpr (VAR == 1 || VAR == 2) __builtin_amdgcn_s_setprio(0);
}

// TRAIN with dropout: the kept probabilities entered PV unscaled; O *= 1 / (1 - p) once
__device__ __forceinline__ void drop_scale_o(State& st, const AttnDrop& drop) {
  if (!drop.thresh) return;
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) st.o[e][qt] *= drop.scale;
}

template <bool FIRST, bool TRAIN = false>
__device__ __forceinline__ void tile_any(const char* Kt, const char* Vt, int kbase, int L, const bf16x8 (&qf)[2],
                                         State& st, int li, int lg, const Train& tr = Train{}) {
  const int rem = L - kbase;
  if (rem >= KT) tile<4, false, FIRST, TRAIN>(Kt, Vt, kbase, L, qf, st, li, lg, tr);
  else if (rem <= 16) tile<1, true, FIRST, TRAIN>(Kt, Vt, kbase, L, qf, st, li, lg, tr);
  else if (rem <= 32) tile<2, true, FIRST, TRAIN>(Kt, Vt, kbase, L, qf, st, li, lg, tr);
  else tile<4, true, FIRST, TRAIN>(Kt, Vt, kbase, L, qf, st, li, lg, tr);
}

// Exact online-max softmax for one wave's 32 queries, K/V read from global memory
// (16 keys per step).  Only runs when the fixed-shift pass overflowed.
// (TRAIN: scores scaled by tr.c here, dropout on the PV operand; st.negm returns -m / c so that
// the caller's lse = -c negm + log2 l holds for both paths)
template <bool TRAIN = false>
__device__ __forceinline__ void attn32_online(const bf16* Kp, const bf16* Vp, long ld, int L, const bf16x8 (&qf)[2],
                                           State& st, int li, int lg, const Train& tr = Train{}) {
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 2; ++e) st.o[e][0] = st.o[e][1] = zero;
  for (int k0 = 0; k0 < L; k0 += 16) {
    const int kr = k0 + li;
    const bf16x8 kf = kr < L ? *reinterpret_cast<const bf16x8*>(Kp + (long)kr * ld + 8 * lg) : bf16x8{};
    bf16x8 vf[2];
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int key = k0 + 4 * lg + j;
        vf[e][j] = (j < 4 && key < L) ? Vp[(long)key * ld + 16 * e + li] : (bf16)0.f;
      }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x4 sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt], zero, 0, 0, 0);
      if constexpr (TRAIN) sc *= tr.c;
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (k0 + 4 * lg + r >= L) sc[r] = -INFINITY;
        mx = fmaxf(mx, sc[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[qt], mx), alpha = exp2f(m[qt] - mn);
      bf16x8 pb{};
      float ps = 0.f;
      float dm[4] = {1.f, 1.f, 1.f, 1.f};
      if constexpr (TRAIN) {
        if (tr.drop.thresh) {
          drop_mul2(tr.drop, tr.dbase, (uint32_t)(tr.q0 + 16 * qt + li), (uint32_t)(k0 + 4 * lg), dm[0], dm[1]);
          drop_mul2(tr.drop, tr.dbase, (uint32_t)(tr.q0 + 16 * qt + li), (uint32_t)(k0 + 4 * lg + 2), dm[2], dm[3]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pf = exp2f(sc[r] - mn);
        const bf16 pr = (bf16)pf;
        ps += (float)pr;
        if constexpr (TRAIN)
          pb[r] = tr.drop.thresh ? (bf16)(pf * dm[r]) : pr;
        else
          pb[r] = pr;
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l[qt] = l[qt] * alpha + ps;
      m[qt] = mn;
#pragma unroll
      for (int e = 0; e < 2; ++e) st.o[e][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[e], pb, st.o[e][qt] * alpha, 0, 0, 0);
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    st.ls[qt] = f32x4{l[qt], l[qt], l[qt], l[qt]};
    const float nm = TRAIN ? -m[qt] / tr.c : -m[qt];
    st.negm[qt] = f32x4{nm, nm, nm, nm};
  }
}
}  // namespace a32

// ------------------------------------------- bf16, head dim 32, LDS-DMA ring --
// attn32_dma: the attn32 math (same tile<> bodies, same LDS images) with K/V staged by
// LDS-DMA (buffer_load ... lds) through a 4-slot ring instead of register staging.  In the
// register-staged kernel every tile paid ~25 VALU instructions of staging (zeroing the
// out-of-range rows, bounds compares, address arithmetic, the LDS stores and their
// addressing) on a loop that is VALU-issue bound (v_exp + cvt + MFMA issue), plus a
// vmcnt(0) stall when the one-tile-ahead load was not back; here a wave issues 2 LDS-DMA
// instructions per tile whose per-lane offsets are loop-invariant (the tile advance rides in
// soffset), the swizzles of k_off / v_off are applied to the SOURCE addresses, loads run 3
// tiles ahead, and the full-tile loop is unrolled by the ring depth so every LDS address is an
// instruction immediate.  Rows past L read the next sequence (finite data; their scores are
// masked to -inf and their P is 0) or, past the tensor, the buffer's out-of-range zeros.
namespace a32 {
constexpr int NS = 4;                           // ring slots
constexpr int SLOT = 2 * TB;                    // K tile + V tile
}  // namespace a32

// VAR 4: the VAR 0 tile body in 8-wave workgroups (2 waves per SIMD, 256 queries): every K/V
// tile's 8 KiB of LDS-DMA is shared by twice the queries, one DMA instruction per wave per tile
// (waves 0-3 move K, 4-7 move V) instead of two.
template <bool PRESCALED, bool TRAIN = false, int VAR = 0>
__global__ __launch_bounds__(VAR == 4 ? 512 : 256, VAR == 4 || VAR == 5 ? 4 : 1) void attn32_dma(int L, int H, const bf16* __restrict__ qkv, long ld,
                                                  bf16* __restrict__ out, long ldo, float scale_log2e, int nqb,
                                                  int* __restrict__ n_fallback, long total_rows,
                                                  float* __restrict__ lse = nullptr, AttnDrop drop = AttnDrop{}) {
  using namespace a32;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int qq = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int qb = wg % nqb, sh = wg / nqb, h = sh % H, seq = sh / H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int D = H * 32;
  const long base = (long)seq * L * ld;
  const bf16* Qp = qkv + base + h * 32;
  const bf16* Kp = qkv + base + D + h * 32;
  const bf16* Vp = qkv + base + 2 * D + h * 32;
  constexpr int NW = VAR == 4 ? 8 : WAVES;          // waves per workgroup
  constexpr int TV = VAR == 4 ? 0 : VAR;            // tile-body variant
  const int q0 = qb * (QPW * NW) + wave * QPW;
  const bool active = q0 < L;                      // wave-uniform

  bf16x8 qf[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    bf16x8 v = q < L ? *reinterpret_cast<const bf16x8*>(Qp + (long)q * ld + 8 * lg) : bf16x8{};
    if constexpr (!PRESCALED && !TRAIN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] * scale_log2e);
    }
    qf[qt] = v;
  }
  // retire the Q loads HERE: the waitcnt pass would otherwise place their wait at the first use,
  // inside the tile loop (the loop header merges the preheader's pending loads), where it
  // becomes an s_waitcnt vmcnt(0) per tile that also drains the LDS-DMA ring
  asm volatile("" : "+v"(qf[0]), "+v"(qf[1]));

  // K / V pieces: wave w moves keys 16 w .. 16 w + 15 of a tile (1 KiB of K, 1 KiB of V); lane
  // l lands at byte 16 l of the piece, i.e. key 16 w + l / 4, image chunk l % 4, so it loads the
  // source chunk that k_off / v_off put there
  const long rem = (total_rows - (long)seq * L) * ld * 2;
  const i32x4 rs = dma_rsrc(qkv + base, rem);
  const int pw = NW == 8 ? wave & 3 : wave;         // the 16-key piece this wave moves
  const int kk = 16 * pw + (lane >> 2), c4 = lane & 3;
  const int kc = c4 ^ ((-(kk >> 2)) & 3);
  const int vc = 2 * ((c4 >> 1) ^ ((kk >> 2) & 1)) + (c4 & 1);
  const int vk = (int)(kk * ld * 2) + (D + h * 32) * 2 + kc * 16;
  const int vv = (int)(kk * ld * 2) + (2 * D + h * 32) * 2 + vc * 16;
  const int tile_bytes = (int)(KT * ld * 2);
  const uint32_t lds_w = lds_addr(smem) + pw * 1024;
  // 8 waves: waves 4-7 move the V pieces (one offset and one LDS base per wave, chosen once)
  const bool vwave = NW == 8 && wave >= 4;
  const int v_mine = vwave ? vv : vk;
  const uint32_t lds_mine = lds_w + (vwave ? TB : 0);
  auto issue = [&](int t, int slot) {
    if constexpr (NW == 8) {
      dma_x4(rs, lds_mine + slot * SLOT, v_mine, t * tile_bytes);
    } else {
      dma_x4(rs, lds_w + slot * SLOT, vk, t * tile_bytes);
      dma_x4(rs, lds_w + slot * SLOT + TB, vv, t * tile_bytes);
    }
  };
  // retire this wave's pieces of tile t: y = younger tiles still in flight (<= NS - 2)
  constexpr int PPT = NW == 8 ? 1 : 2;              // DMA instructions per wave per tile
  auto wait = [&](int y) {
    if (y >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPT) : "memory");
    else if (y == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  State st;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    st.o[0][qt] = st.o[1][qt] = st.ls[qt] = zero;
    st.negm[qt] = zero;
  }
  Train tr{};
  if constexpr (TRAIN) tr = Train{scale_log2e, drop, drop.thresh ? drop_base(drop.seed, (uint32_t)sh) : 0u, q0};
  const int ntile = (L + KT - 1) / KT, nfull = L / KT;
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < ntile) issue(j, j);
  // one tile of the ring: slot S is compile-time, so the LDS reads take immediate offsets
  // (inside the unrolled loop t + NS <= nfull: NS - 2 younger tiles are in flight and tile
  // t + NS - 1 exists, so the wait and the issue are unconditional)
  auto step = [&](auto s_tag, int t) {
    constexpr int S = decltype(s_tag)::value;
    wait(NS - 2);
    __builtin_amdgcn_s_barrier();                  // tile t visible; every wave is done with t - 1
    issue(t + NS - 1, (S + NS - 1) % NS);
    // a wave past L (3 of the 4 waves of the last query block at L = 1030: 8 % of all waves) only
    // moves its DMA pieces and meets the barriers — a wave-uniform branch, not 20 idle MFMAs
    if (active) {
      const char* Kt = smem + S * SLOT;
      if (t == 0) tile<4, false, true, TRAIN, TV>(Kt, Kt + TB, 0, L, qf, st, li, lg, tr);
      else tile<4, false, false, TRAIN, TV>(Kt, Kt + TB, t * KT, L, qf, st, li, lg, tr);
    }
  };
  int t = 0;
  bool ring3 = false;
  if constexpr (VAR == 3) ring3 = nfull >= NS + 1;
  if (ring3) {
    // K of tile t + 1 read during tile t: the ring barrier moves between the exps and the PV
    // block of tile t (every wave then is done with V of t - 1 and has landed tile t + 1), the
    // look-ahead drops to 2 tiles (tile t + 3 issued into the slot of t - 1 at that barrier)
    bf16x8 kcur[4];
    wait(1);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) kcur[kt] = *reinterpret_cast<const bf16x8*>(smem + k_off(16 * kt + li, lg));
    auto step3 = [&](auto s_tag, int t) {
      constexpr int S = decltype(s_tag)::value;
      bf16x8 knext[4];
      auto mid = [&]() {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");      // this wave's pieces of tile t + 1
        __builtin_amdgcn_s_barrier();
        issue(t + NS - 1, (S + NS - 1) % NS);
        const char* Kn = smem + ((S + 1) % NS) * SLOT;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) knext[kt] = *reinterpret_cast<const bf16x8*>(Kn + k_off(16 * kt + li, lg));
      };
      const char* Kt = smem + S * SLOT;
      if (!active) mid();                           // barrier + issue only
      else if (t == 0) tile<4, false, true, TRAIN, 3>(Kt, Kt + TB, 0, L, qf, st, li, lg, tr, kcur, mid);
      else tile<4, false, false, TRAIN, 3>(Kt, Kt + TB, t * KT, L, qf, st, li, lg, tr, kcur, mid);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) kcur[kt] = knext[kt];
    };
    // full tiles whose successor is a full tile that exists and whose t + NS - 1 issue is in range
    for (; t + NS <= nfull - 1; t += NS) {
      step3(std::integral_constant<int, 0>{}, t);
      step3(std::integral_constant<int, 1>{}, t + 1);
      step3(std::integral_constant<int, 2>{}, t + 2);
      step3(std::integral_constant<int, 3>{}, t + 3);
    }
    // hand back to the plain loop: tile t's K is in LDS and visible; its barrier already passed,
    // so the plain step's barrier and issue must not repeat — run tile t here, then continue
    {
      const char* Kt = smem + (t % NS) * SLOT;
      __builtin_amdgcn_s_barrier();                  // every wave done with tile t - 1 (its V)
      if (t + NS - 1 < ntile) issue(t + NS - 1, (t + NS - 1) % NS);
      if (active) tile_any<false, TRAIN>(Kt, Kt + TB, t * KT, L, qf, st, li, lg, tr);   // t >= NS: not the first
      ++t;
    }
  } else {
  for (; t + NS <= nfull; t += NS) {
    step(std::integral_constant<int, 0>{}, t);
    step(std::integral_constant<int, 1>{}, t + 1);
    step(std::integral_constant<int, 2>{}, t + 2);
    step(std::integral_constant<int, 3>{}, t + 3);
  }
  }
  for (; t < ntile; ++t) {                         // the last < NS full tiles and the ragged tail
    wait(min(NS - 2, ntile - 1 - t));
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < ntile) issue(t + NS - 1, (t + NS - 1) % NS);
    if (active) {
      const char* Kt = smem + (t % NS) * SLOT;
      if (t == 0) tile_any<true, TRAIN>(Kt, Kt + TB, 0, L, qf, st, li, lg, tr);
      else tile_any<false, TRAIN>(Kt, Kt + TB, t * KT, L, qf, st, li, lg, tr);
    }
  }
  if (!active) return;
  if constexpr (TRAIN) drop_scale_o(st, drop);

  bool bad = false;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float l = st.ls[qt][0];
    bad |= !(l > 0.f && l < INFINITY);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int r = 0; r < 4; ++r) bad |= !__builtin_isfinite(st.o[e][qt][r]);
  }
  if (__ballot(bad)) {
    if (lane == 0 && n_fallback) atomicAdd(n_fallback, 1);
    attn32_online<TRAIN>(Kp, Vp, ld, L, qf, st, li, lg, tr);
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    if (q >= L) continue;
    const float inv = 1.0f / st.ls[qt][0];
    if constexpr (TRAIN) {
      if (lg == 0) lse[((long)seq * H + h) * L + q] = -scale_log2e * st.negm[qt][0] + log2f(st.ls[qt][0]);
    }
    bf16* op = out + (long)seq * L * ldo + (long)q * ldo + h * 32;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(st.o[e][qt][r] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * e + 4 * lg) = w;
    }
  }
}

// ---------------------------------------------------------------- f32 path --
template <int DH>
__global__ __launch_bounds__(64) void attn_fwd_f32(int nseq, int L, int H, const float* __restrict__ qkv,
                                                   long ld, float* __restrict__ out, long ldo, float scale) {
  __shared__ float ks[AK][DH];
  __shared__ float vs[AK][DH];
  const int qb = blockIdx.x, h = blockIdx.y, seq = blockIdx.z;
  const int tid = threadIdx.x;
  const int D = H * DH;
  const long base = (long)seq * L * ld;
  const int q = qb * 64 + tid;
  float qv[DH], o[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    qv[d] = q < L ? qkv[base + (long)q * ld + h * DH + d] * scale : 0.f;
    o[d] = 0.f;
  }
  float m_run = -INFINITY, l_run = 0.f;
  for (int t0 = 0; t0 < L; t0 += AK) {
    __syncthreads();
    for (int i = tid; i < AK * DH; i += 64) {
      const int key = i / DH, d = i % DH, kk = t0 + key;
      ks[key][d] = kk < L ? qkv[base + (long)kk * ld + D + h * DH + d] : 0.f;
      vs[key][d] = kk < L ? qkv[base + (long)kk * ld + 2 * D + h * DH + d] : 0.f;
    }
    __syncthreads();
    const int nk = min(AK, L - t0);
    for (int j = 0; j < nk; ++j) {
      float sc = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) sc = fmaf(qv[d], ks[j][d], sc);
      const float m_new = fmaxf(m_run, sc);
      const float a = expf(m_run - m_new), p = expf(sc - m_new);
      l_run = l_run * a + p;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] = o[d] * a + p * vs[j][d];
      m_run = m_new;
    }
  }
  if (q < L) {
    float* op = out + (long)seq * L * ldo + (long)q * ldo + h * DH;
#pragma unroll
    for (int d = 0; d < DH; ++d) op[d] = o[d] / l_run;
  }
}

// device counter of waves that took the exact online-softmax fallback (tests read it)
static int* attn_fallback_counter() {
  static int* p = nullptr;
  if (!p && hipMalloc(&p, sizeof(int)) == hipSuccess) (void)hipMemset(p, 0, sizeof(int));
  return p;
}

template <int DH>
static int launch_attn(int dtype, long nseq, long L, int H, const void* qkv, long ld, void* out,
                       long ldo, float scale, hipStream_t s) {
  evlog_begin(s);
  if (DH == 32 && dtype == SNVRAG_BF16) {
    const int nqb = cdiv(L, a32::QPB);
    const long nb = (long)nqb * H * nseq;
    SNV_CHECK_ARG(nb < (1L << 31), "grid too large");
    const float sl2 = scale * 1.4426950408889634f;
    const bool pre = fabsf(sl2 - 1.0f) < 1e-6f;      // Q already carries log2(e)/sqrt(dh)
    int* cnt = attn_fallback_counter();
    const int var = (int)options().attn_variant;
    auto kp = var == 1 ? attn32_dma<true, false, 1> : var == 2 ? attn32_dma<true, false, 2>
              : var == 3 ? attn32_dma<true, false, 3> : var == 4 ? attn32_dma<true, false, 4>
              : var == 5 ? attn32_dma<true, false, 5> : attn32_dma<true, false, 0>;
    const int nqb8 = cdiv(L, 2 * a32::QPB);
    if (pre && var == 4)
      hipLaunchKernelGGL(kp, dim3((unsigned)(nqb8 * H * nseq)), dim3(512), 0, s, (int)L, H, (const bf16*)qkv, ld,
                         (bf16*)out, ldo, 1.0f, nqb8, cnt, (long)nseq * L, nullptr, AttnDrop{});
    else if (pre)
      hipLaunchKernelGGL(kp, dim3((unsigned)nb), dim3(256), 0, s, (int)L, H, (const bf16*)qkv, ld,
                         (bf16*)out, ldo, 1.0f, nqb, cnt, (long)nseq * L, nullptr, AttnDrop{});
    else
      hipLaunchKernelGGL(attn32_dma<false>, dim3((unsigned)nb), dim3(256), 0, s, (int)L, H, (const bf16*)qkv, ld,
                         (bf16*)out, ldo, sl2, nqb, cnt, (long)nseq * L, nullptr, AttnDrop{});
  } else if (dtype == SNVRAG_BF16) {
    const int nqb = cdiv(L, AQ);
    const long nb = (long)nqb * H * nseq;
    SNV_CHECK_ARG(nb < (1L << 31), "grid too large");
    hipLaunchKernelGGL(attn_fwd_bf16<DH>, dim3((unsigned)nb), dim3(256), 0, s, (int)nseq, (int)L, H,
                       (const bf16*)qkv, ld, (bf16*)out, ldo, scale * 1.4426950408889634f, nqb, nullptr,
                       make_attn_drop(0.f, 0));
  } else {
    hipLaunchKernelGGL(attn_fwd_f32<DH>, dim3(cdiv(L, 64), H, (unsigned)nseq), dim3(64), 0, s,
                       (int)nseq, (int)L, H, (const float*)qkv, ld, (float*)out, ldo, scale);
  }
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_ATTN, 4.0 * nseq * H * (double)L * L * DH);
  return 0;
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_attention_fallbacks(int reset) {
  int* p = attn_fallback_counter();
  if (!p) return fail(__func__, "no device counter");
  int v = 0;
  SNV_HIP(hipMemcpy(&v, p, sizeof(int), hipMemcpyDeviceToHost));
  if (reset) SNV_HIP(hipMemset(p, 0, sizeof(int)));
  return v;
}

// Training forward: the generic bf16 kernel (online softmax) plus the per-row log2-sum-exp
// the backward (attention_train.hip) rebuilds P from.
extern "C" int snvrag_attention_train_fwd(int64_t nseq, int64_t L, int heads, int dh, const void* qkv,
                                          int64_t ld_qkv, void* out, int64_t ld_out, float* lse, float scale,
                                          float dropout_p, uint64_t seed, void* stream) {
  SNV_CHECK_ARG(qkv && out && lse, "null pointer");
  SNV_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout probability must be in [0, 1)");
  const AttnDrop drop = make_attn_drop(dropout_p, seed);
  SNV_CHECK_ARG(nseq >= 0 && L > 0 && heads > 0, "bad shape");
  SNV_CHECK_ARG(ld_qkv >= 3L * heads * dh && ld_out >= (long)heads * dh, "leading dims too small");
  SNV_CHECK_ARG(ld_qkv % 8 == 0 && ld_out % 4 == 0, "bf16 alignment");
  if (nseq == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int nqb = cdiv(L, AQ);
  const long nb = (long)nqb * heads * nseq;
  SNV_CHECK_ARG(nb < (1L << 31), "grid too large");
  const float sl2 = scale * 1.4426950408889634f;
  evlog_begin(s);
  if (dh == 32) {
    // the inference kernel's structure (fixed shift, ones-MFMA row sums, 32 queries per wave) with
    // unscaled Q, lse and dropout (attn32_dma<false, true>)
    const int nqb3 = cdiv(L, a32::QPB);
    const long nb3 = (long)nqb3 * heads * nseq;
    SNV_CHECK_ARG(nb3 < (1L << 31), "grid too large");
    hipLaunchKernelGGL((attn32_dma<false, true>), dim3((unsigned)nb3), dim3(256), 0, s, (int)L, heads,
                       (const bf16*)qkv, (long)ld_qkv, (bf16*)out, (long)ld_out, sl2, nqb3, attn_fallback_counter(),
                       (long)nseq * L, lse, drop);
  } else if (dh == 64)
    hipLaunchKernelGGL(attn_fwd_bf16<64>, dim3((unsigned)nb), dim3(256), 0, s, (int)nseq, (int)L, heads,
                       (const bf16*)qkv, (long)ld_qkv, (bf16*)out, (long)ld_out, sl2, nqb, lse, drop);
  else
    return fail(__func__, "training attention supports head dims 32 and 64");
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_ATTN, 4.0 * nseq * heads * (double)L * L * dh);
  return 0;
}

extern "C" int snvrag_attention(int dtype, int64_t nseq, int64_t L, int heads, int dh,
                                const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out,
                                float scale, void* stream) {
  SNV_CHECK_ARG(qkv && out, "null pointer");
  SNV_CHECK_ARG(nseq >= 0 && L > 0 && heads > 0, "bad shape");
  SNV_CHECK_ARG(ld_qkv >= 3L * heads * dh && ld_out >= (long)heads * dh, "leading dims too small");
  if (dtype == SNVRAG_BF16)
    SNV_CHECK_ARG(ld_qkv % 8 == 0 && ld_out % 4 == 0 && (heads * dh) % 8 == 0, "bf16 alignment");
  if (nseq == 0) return 0;
  hipStream_t s = as_stream(stream);
  switch (dh) {
    case 16: return launch_attn<16>(dtype, nseq, L, heads, qkv, ld_qkv, out, ld_out, scale, s);
    case 32: return launch_attn<32>(dtype, nseq, L, heads, qkv, ld_qkv, out, ld_out, scale, s);
    case 48: return launch_attn<48>(dtype, nseq, L, heads, qkv, ld_qkv, out, ld_out, scale, s);
    case 64: return launch_attn<64>(dtype, nseq, L, heads, qkv, ld_qkv, out, ld_out, scale, s);
    default: return fail(__func__, "head dim must be 16, 32, 48 or 64");
  }
}
