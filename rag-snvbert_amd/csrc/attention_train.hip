// Attention backward for training (bf16 in, f32 accumulation, bf16 gradients).
//
// Reference: model/attention/attention.py:21-31 (softmax(Q K^T / sqrt(dh)) V, no mask)
// under autograd, with the head split/merge of multi_head_attention.py:44-51.  The
// forward (attention.hip attn_fwd_bf16 with an lse pointer) stores
// lse[q] = log2 sum_k exp2(c s_qk), c = scale * log2(e); with P = exp2(c S - lse):
//   D_q  = sum_d dO[q,d] O[q,d]
//   dS   = P o (dO V^T - D)            (gradient w.r.t. the scaled scores)
//   dQ   = scale * dS K,   dK = scale * dS^T Q,   dV = P^T dO.
// Two kernels, no atomics (the FlashAttention-2 split):
//   attn_bwd_dq  : one workgroup = 64 queries of one (sequence, head), loops over key
//                  tiles.  The forward's lane layout: S^T = K Q^T and dP^T = V dO^T
//                  accumulate with one query per lane column; dS^T feeds
//                  dQ^T += K^T dS^T as the B operand straight from the accumulators.
//                  Also writes D_q for the second kernel.
//   attn_bwd_dkv : one workgroup = 64 keys, loops over query tiles.  S = Q K^T and
//                  dP = dO V^T accumulate with one key per lane column; P and dS feed
//                  dV^T += dO^T P and dK^T += Q^T dS the same way.
// MFMA v_mfma_f32_16x16x32_bf16 throughout (lane (li, lg): A row li / B column li,
// k = 8 lg + j; D[4 lg + r][li]).  Head dims 32 and 64.
#include "attn_common.h"

#include <cmath>
#include <utility>

namespace snvrag {

template <int DH>
struct BwdCfg {
  using C = AttnCfg<DH>;
  static constexpr int CH = C::CPR;                         // 16-B chunks per row
  static constexpr int NLD = (64 * CH + 255) / 256;         // loads per thread per 64-row tile
};

// XCD-aware block order (consecutive tiles of one (sequence, head) share an XCD's L2)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int qq = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  return (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
}

// load a 64-row x DH bf16 tile (rows >= L are zero) into registers
template <int DH>
__device__ __forceinline__ void tile_load(u32x4 (&r)[BwdCfg<DH>::NLD], const bf16* __restrict__ P, long ld, int t0,
                                          int L, int tid) {
  using B = BwdCfg<DH>;
#pragma unroll
  for (int i = 0; i < B::NLD; ++i) {
    const int id = tid + 256 * i;
    const int row = id / B::CH, c = id % B::CH;
    const int rr = t0 + row, d0 = 8 * c;
    if (id < 64 * B::CH && rr < L && d0 < DH) r[i] = *reinterpret_cast<const u32x4*>(P + (long)rr * ld + d0);
    else r[i] = u32x4{0u, 0u, 0u, 0u};
  }
}
// row-major swizzled store (A operand rows: MFMA reads row li, chunk 4 ks + lg)
template <int DH>
__device__ __forceinline__ void tile_store_rows(char* dst, const u32x4 (&r)[BwdCfg<DH>::NLD], int tid) {
  using B = BwdCfg<DH>;
#pragma unroll
  for (int i = 0; i < B::NLD; ++i) {
    const int id = tid + 256 * i;
    if (id < 64 * B::CH) *reinterpret_cast<u32x4*>(dst + k_off<DH>(id / B::CH, id % B::CH)) = r[i];
  }
}
// transposed store [d][row] with row stride VT_LD (A operand of the P / dS products)
template <int DH>
__device__ __forceinline__ void tile_store_t(char* dst, const u32x4 (&r)[BwdCfg<DH>::NLD], int tid) {
  using B = BwdCfg<DH>;
  using C = AttnCfg<DH>;
  bf16* t = reinterpret_cast<bf16*>(dst);
#pragma unroll
  for (int i = 0; i < B::NLD; ++i) {
    const int id = tid + 256 * i;
    if (id < 64 * B::CH) {
      const int row = id / B::CH, c = id % B::CH;
      const bf16x8 v = __builtin_bit_cast(bf16x8, r[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[(8 * c + j) * C::VT_LD + row] = v[j];
    }
  }
}
// A fragment of a transposed tile whose k = 64 rows follow the accumulator order of a
// 4 x (16-row) score block: half c covers rows 32c + 4 lg + {0..3} and 32c + 16 + 4 lg + {0..3}
template <int DH>
__device__ __forceinline__ bf16x8 t_frag(const char* tt, int e, int c, int li, int lg) {
  using C = AttnCfg<DH>;
  const bf16* row = reinterpret_cast<const bf16*>(tt) + (16 * e + li) * C::VT_LD + 32 * c + 4 * lg;
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(row);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(row + 16);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// B fragment of this lane's row r over d: k = 32 ks + 8 lg + j
template <int DH>
__device__ __forceinline__ void row_frag(bf16x8 (&f)[AttnCfg<DH>::KS], const bf16* __restrict__ P, long ld, int r,
                                         int L, int lg) {
#pragma unroll
  for (int ks = 0; ks < AttnCfg<DH>::KS; ++ks) {
    const int d0 = 32 * ks + 8 * lg;
    f[ks] = (r < L && d0 < DH) ? *reinterpret_cast<const bf16x8*>(P + (long)r * ld + d0) : bf16x8{};
  }
}

// ------------------------------------------------------------------- dQ ---
template <int DH>
__global__ __launch_bounds__(256) void attn_bwd_dq(int L, int H, const bf16* __restrict__ qkv, long ld,
                                                   const bf16* __restrict__ O, long ldo,
                                                   const bf16* __restrict__ dO, long lddo,
                                                   const float* __restrict__ lse, float* __restrict__ Dout,
                                                   bf16* __restrict__ dqkv, long ldd, float c_log2e, float scale,
                                                   int nqb, AttnDrop drop) {
  using C = AttnCfg<DH>;
  using B = BwdCfg<DH>;
  constexpr int STAGE = 2 * C::KBYTES + C::VBYTES;          // K rows, V rows, K^T
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = wg % nqb, sh = wg / nqb, h = sh % H, seq = sh / H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int D = H * DH;
  const long row0 = (long)seq * L;
  const bf16* Kp = qkv + row0 * ld + D + h * DH;
  const bf16* Vp = qkv + row0 * ld + 2 * D + h * DH;
  const int q = qb * 64 + wave * 16 + li;

  bf16x8 qf[C::KS], df[C::KS], of[C::KS];
  row_frag<DH>(qf, qkv + row0 * ld + h * DH, ld, q, L, lg);
  row_frag<DH>(df, dO + row0 * lddo + h * DH, lddo, q, L, lg);
  row_frag<DH>(of, O + row0 * ldo + h * DH, ldo, q, L, lg);
  float dq_ = 0.f;
#pragma unroll
  for (int ks = 0; ks < C::KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) dq_ += (float)df[ks][j] * (float)of[ks][j];
  dq_ += __shfl_xor(dq_, 16, 64);
  dq_ += __shfl_xor(dq_, 32, 64);
  const long srow = ((long)seq * H + h) * L;
  const float lse_q = q < L ? lse[srow + q] : 0.f;
  const uint32_t dbase = drop_base(drop.seed, (uint32_t)sh);
  if (q < L && lg == 0) Dout[srow + q] = dq_;

  u32x4 kr[B::NLD], vr[B::NLD];
  auto store = [&](char* st) {
    tile_store_rows<DH>(st, kr, tid);
    tile_store_rows<DH>(st + C::KBYTES, vr, tid);
    tile_store_t<DH>(st + 2 * C::KBYTES, kr, tid);
  };
  f32x4 acc[C::ET];
#pragma unroll
  for (int e = 0; e < C::ET; ++e) acc[e] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ntile = (L + 63) / 64;
  tile_load<DH>(kr, Kp, ld, 0, L, tid);
  tile_load<DH>(vr, Vp, ld, 0, L, tid);
  store(smem);
  __syncthreads();
  for (int t = 0; t < ntile; ++t) {
    char* st = smem + (t & 1) * STAGE;
    const bool more = t + 1 < ntile;
    if (more) {
      tile_load<DH>(kr, Kp, ld, (t + 1) * 64, L, tid);
      tile_load<DH>(vr, Vp, ld, (t + 1) * 64, L, tid);
    }
    f32x4 s[4], dp[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int key = 16 * kt + li;
#pragma unroll
      for (int ks = 0; ks < C::KS; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(st + k_off<DH>(key, 4 * ks + lg));
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(st + C::KBYTES + k_off<DH>(key, 4 * ks + lg));
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[kt], 0, 0, 0);
        dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, df[ks], dp[kt], 0, 0, 0);
      }
    }
    bf16x8 dsb[2];
    // hash input of (q, key pair (64 t + 4 lg) / 2); (kt, r) adds 8 kt + r / 2
    const uint32_t drow = drop_row(dbase, (uint32_t)q, (uint32_t)(32 * t + 2 * lg));
    // straight-line element math (raw v_exp_f32, no per-element branches); only the ragged
    // last key tile masks keys >= L
    auto elem = [&](auto mask_tag) {
      constexpr bool MASK = decltype(mask_tag)::value;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          float dm[2] = {1.f, 1.f};
          if (drop.thresh) drop_split(drop, drop_mix24(drow + (uint32_t)(8 * kt + (r >> 1)) * DROP_C2), dm[0], dm[1]);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            float p = __builtin_amdgcn_exp2f(s[kt][r + e] * c_log2e - lse_q);
            if constexpr (MASK) p = t * 64 + 16 * kt + 4 * lg + r + e < L ? p : 0.f;
            // dropout: dP = (dO V^T) o mask / (1 - p); D_q = rowsum(dO o O) is unchanged (O = P' V)
            const float dpv = dp[kt][r + e] * dm[e];
            dsb[kt >> 1][(kt & 1) * 4 + r + e] = (bf16)(p * (dpv - dq_));
          }
        }
    };
    if ((t + 1) * 64 <= L) elem(std::false_type{});
    else elem(std::true_type{});
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < C::ET; ++e)
        acc[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t_frag<DH>(st + 2 * C::KBYTES, e, c, li, lg), dsb[c],
                                                         acc[e], 0, 0, 0);
    if (more) store(smem + ((t + 1) & 1) * STAGE);
    __syncthreads();
  }
  if (q < L) {
    bf16* op = dqkv + (row0 + q) * ldd + h * DH;
#pragma unroll
    for (int e = 0; e < C::ET; ++e) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(acc[e][r] * scale);
      *reinterpret_cast<bf16x4*>(op + 16 * e + 4 * lg) = w;
    }
  }
}

// ------------------------------------------------------------------ dKV ---
template <int DH>
__global__ __launch_bounds__(256) void attn_bwd_dkv(int L, int H, const bf16* __restrict__ qkv, long ld,
                                                    const bf16* __restrict__ dO, long lddo,
                                                    const float* __restrict__ lse, const float* __restrict__ Dq,
                                                    bf16* __restrict__ dqkv, long ldd, float c_log2e, float scale,
                                                    int nkb, AttnDrop drop) {
  using C = AttnCfg<DH>;
  using B = BwdCfg<DH>;
  constexpr int STAGE = 2 * C::KBYTES + 2 * C::VBYTES + 2 * 64 * 4;   // Q, dO rows; Q^T, dO^T; lse, D
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = wg % nkb, sh = wg / nkb, h = sh % H, seq = sh / H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int D = H * DH;
  const long row0 = (long)seq * L;
  const bf16* Qp = qkv + row0 * ld + h * DH;
  const bf16* dOp = dO + row0 * lddo + h * DH;
  const long srow = ((long)seq * H + h) * L;
  const int key = kb * 64 + wave * 16 + li;
  const uint32_t dbase = drop_base(drop.seed, (uint32_t)sh);

  bf16x8 kf[C::KS], vf[C::KS];
  row_frag<DH>(kf, qkv + row0 * ld + D + h * DH, ld, key, L, lg);
  row_frag<DH>(vf, qkv + row0 * ld + 2 * D + h * DH, ld, key, L, lg);

  u32x4 qr[B::NLD], gr[B::NLD];
  float lr = 0.f, dr = 0.f;
  auto load = [&](int t0) {
    tile_load<DH>(qr, Qp, ld, t0, L, tid);
    tile_load<DH>(gr, dOp, lddo, t0, L, tid);
    if (tid < 64) {
      const int qq = t0 + tid;
      lr = qq < L ? lse[srow + qq] : 0.f;
      dr = qq < L ? Dq[srow + qq] : 0.f;
    }
  };
  auto store = [&](char* st) {
    tile_store_rows<DH>(st, qr, tid);
    tile_store_rows<DH>(st + C::KBYTES, gr, tid);
    tile_store_t<DH>(st + 2 * C::KBYTES, qr, tid);
    tile_store_t<DH>(st + 2 * C::KBYTES + C::VBYTES, gr, tid);
    float* ls = reinterpret_cast<float*>(st + 2 * C::KBYTES + 2 * C::VBYTES);
    if (tid < 64) { ls[tid] = lr; ls[64 + tid] = dr; }
  };
  f32x4 dk[C::ET], dv[C::ET];
#pragma unroll
  for (int e = 0; e < C::ET; ++e) { dk[e] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[e] = dk[e]; }

  const int ntile = (L + 63) / 64;
  load(0);
  store(smem);
  __syncthreads();
  for (int t = 0; t < ntile; ++t) {
    char* st = smem + (t & 1) * STAGE;
    const bool more = t + 1 < ntile;
    if (more) load((t + 1) * 64);
    const float* ls = reinterpret_cast<const float*>(st + 2 * C::KBYTES + 2 * C::VBYTES);
    f32x4 s[4], dp[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      s[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int qrow = 16 * qt + li;
#pragma unroll
      for (int ks = 0; ks < C::KS; ++ks) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(st + k_off<DH>(qrow, 4 * ks + lg));
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(st + C::KBYTES + k_off<DH>(qrow, 4 * ks + lg));
        s[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[ks], s[qt], 0, 0, 0);
        dp[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, vf[ks], dp[qt], 0, 0, 0);
      }
    }
    bf16x8 pb[2], dsb[2];
    // dropout multipliers: the keys of a hash pair sit in lanes li, li ^ 1 with the same 16
    // queries, so each lane hashes half of them (r in {0,1} even lanes, {2,3} odd lanes) and
    // swaps with its neighbour (DPP quad_perm [1,0,3,2]); it then takes its key's 16-bit half
    float mkv[4][4];
    if (drop.thresh) {
      const bool odd = li & 1;
      // hash input of (query 64 t + 4 lg (+ 2 on odd lanes), this key's pair); (qt, rr) adds
      // (16 qt + rr) * C1
      const uint32_t drow = drop_row(dbase, (uint32_t)(t * 64 + 4 * lg + (odd ? 2 : 0)), (uint32_t)key >> 1);
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const uint32_t hm = drop_mix24(drow + (uint32_t)(16 * qt + rr) * DROP_C1);
          const uint32_t ho = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hm, 0xB1, 0xF, 0xF, false);
          const uint32_t h_lo = odd ? ho : hm, h_hi = odd ? hm : ho;       // hashes of r = rr, 2 + rr
          mkv[qt][rr] = (odd ? h_lo >> 16 : h_lo & 0xFFFFu) >= drop.thresh ? drop.scale : 0.f;
          mkv[qt][2 + rr] = (odd ? h_hi >> 16 : h_hi & 0xFFFFu) >= drop.thresh ? drop.scale : 0.f;
        }
    }
    // straight-line element math (raw v_exp_f32); only the ragged last query tile masks q >= L
    auto elem = [&](auto mask_tag) {
      constexpr bool MASK = decltype(mask_tag)::value;
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * qt + 4 * lg + r;
          float p = __builtin_amdgcn_exp2f(s[qt][r] * c_log2e - ls[ql]);
          if constexpr (MASK) p = t * 64 + ql < L ? p : 0.f;
          // dropout: dV uses the kept, rescaled probabilities; dP is masked the same way
          const float mk = drop.thresh ? mkv[qt][r] : 1.f;
          const float pm = p * mk;
          pb[qt >> 1][(qt & 1) * 4 + r] = (bf16)pm;
          dsb[qt >> 1][(qt & 1) * 4 + r] = (bf16)fmaf(pm, dp[qt][r], -p * ls[64 + ql]);
        }
    };
    if ((t + 1) * 64 <= L) elem(std::false_type{});
    else elem(std::true_type{});
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < C::ET; ++e) {
        dv[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t_frag<DH>(st + 2 * C::KBYTES + C::VBYTES, e, c, li, lg),
                                                        pb[c], dv[e], 0, 0, 0);
        dk[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t_frag<DH>(st + 2 * C::KBYTES, e, c, li, lg), dsb[c],
                                                        dk[e], 0, 0, 0);
      }
    if (more) store(smem + ((t + 1) & 1) * STAGE);
    __syncthreads();
  }
  if (key < L) {
    bf16* kp = dqkv + (row0 + key) * ldd + D + h * DH;
    bf16* vp = dqkv + (row0 + key) * ldd + 2 * D + h * DH;
#pragma unroll
    for (int e = 0; e < C::ET; ++e) {
      bf16x4 wk, wv;
#pragma unroll
      for (int r = 0; r < 4; ++r) { wk[r] = (bf16)(dk[e][r] * scale); wv[r] = (bf16)dv[e][r]; }
      *reinterpret_cast<bf16x4*>(kp + 16 * e + 4 * lg) = wk;
      *reinterpret_cast<bf16x4*>(vp + 16 * e + 4 * lg) = wv;
    }
  }
}

template <int DH>
static int launch_bwd(long nseq, long L, int H, const bf16* qkv, long ld, const bf16* O, long ldo, const bf16* dO,
                      long lddo, const float* lse, float* Dws, bf16* dqkv, long ldd, float scale, AttnDrop drop,
                      hipStream_t s) {
  const int nb = cdiv(L, 64);
  const long grid = (long)nb * H * nseq;
  SNV_CHECK_ARG(grid < (1L << 31), "grid too large");
  const float cl = scale * 1.4426950408889634f;
  evlog_begin(s);
  hipLaunchKernelGGL(attn_bwd_dq<DH>, dim3((unsigned)grid), dim3(256), 0, s, (int)L, H, qkv, ld, O, ldo, dO, lddo,
                     lse, Dws, dqkv, ldd, cl, scale, nb, drop);
  SNV_LAUNCH_CHECK();
  hipLaunchKernelGGL(attn_bwd_dkv<DH>, dim3((unsigned)grid), dim3(256), 0, s, (int)L, H, qkv, ld, dO, lddo, lse,
                     (const float*)Dws, dqkv, ldd, cl, scale, nb, drop);
  SNV_LAUNCH_CHECK();
  // QK^T and dO V^T in both kernels + the dQ, dK, dV products: 7 x 2 L^2 dh per head
  evlog_end(s, EV_ATTN_BWD, 14.0 * nseq * H * (double)L * L * DH);
  return 0;
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_attention_bwd(int64_t nseq, int64_t L, int heads, int dh, const void* qkv, int64_t ld_qkv,
                                    const void* out, int64_t ld_out, const void* dout, int64_t ld_dout,
                                    const float* lse, float* d_ws, void* dqkv, int64_t ld_dqkv, float scale,
                                    float dropout_p, uint64_t seed, void* stream) {
  SNV_CHECK_ARG(qkv && out && dout && lse && d_ws && dqkv, "null pointer");
  SNV_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout probability must be in [0, 1)");
  const AttnDrop drop = make_attn_drop(dropout_p, seed);
  SNV_CHECK_ARG(nseq >= 0 && L > 0 && heads > 0, "bad shape");
  SNV_CHECK_ARG(ld_qkv >= 3L * heads * dh && ld_dqkv >= 3L * heads * dh && ld_out >= (long)heads * dh &&
                    ld_dout >= (long)heads * dh, "leading dims too small");
  SNV_CHECK_ARG(ld_qkv % 8 == 0 && ld_out % 8 == 0 && ld_dout % 8 == 0 && ld_dqkv % 4 == 0, "bf16 alignment");
  if (nseq == 0) return 0;
  hipStream_t s = as_stream(stream);
  const bf16 *q = (const bf16*)qkv, *o = (const bf16*)out, *g = (const bf16*)dout;
  switch (dh) {
    case 32: return launch_bwd<32>(nseq, L, heads, q, ld_qkv, o, ld_out, g, ld_dout, lse, d_ws, (bf16*)dqkv, ld_dqkv,
                                   scale, drop, s);
    case 64: return launch_bwd<64>(nseq, L, heads, q, ld_qkv, o, ld_out, g, ld_dout, lse, d_ws, (bf16*)dqkv, ld_dqkv,
                                   scale, drop, s);
    default: return fail(__func__, "training attention supports head dims 32 and 64");
  }
}
