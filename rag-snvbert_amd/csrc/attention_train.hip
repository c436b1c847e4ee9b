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
#include <cstdlib>
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

// ------------------------------------------------- dh = 32: LDS-DMA ring, one image layout --
// attn_bwd_dq32 / attn_bwd_dkv32: the same FlashAttention-2 split and element math as the
// templates above, restructured for the VALU- and LDS-issue-bound dh = 32 case:
//  * Q / dO (dkv) and K / V (dq) tiles arrive by LDS-DMA (buffer_load ... lds, 1 KiB per wave
//    instruction, per-lane source offsets loop-invariant, the tile advance in soffset) through a
//    4-slot ring, 3 tiles in flight, one barrier per tile; lse and D (dkv) ride along in the slot;
//  * ONE image per tile (the inference kernel's V layout: 64-B rows, 32-B halves swapped on
//    (row >> 2) & 1), conflict-free both for the ds_read_b128 row reads (A operands over dh:
//    S, dP) and for the ds_read_b64_tr_b16 transposed reads (A operands over rows: dQ, dK, dV) —
//    the templates' transposed copies, written element by element with ds_write_b16, are gone;
//  * the ring loop is unrolled by its depth so every LDS address is an instruction immediate.
namespace b32 {
constexpr int NS = 4;
constexpr int TILE = 64 * 64;                           // 64 rows x 32 bf16
__device__ __forceinline__ int img(int row, int chunk) {
  return row * 64 + (((chunk >> 1) ^ ((row >> 2) & 1)) << 5) + ((chunk & 1) << 4);
}
// the source chunk that lands at 16-B position p of an image row
__device__ __forceinline__ int img_src(int row, int p) { return (((p >> 1) ^ ((row >> 2) & 1)) << 1) | (p & 1); }
__device__ __forceinline__ bf16x4 trr(const char* p) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  return __builtin_bit_cast(bf16x4, v);
}
// A fragment over 64 image rows (MFMA k = 8 lg + j: rows 32 c + 4 lg + {0..3}, 32 c + 16 + 4 lg + {0..3})
// at columns 16 e + li: the transposed tile, read transposed
__device__ __forceinline__ bf16x8 tfrag(const char* im, int e, int c, int li, int lg) {
  const int q = li >> 2, p = li & 3, r0 = 32 * c + 4 * lg + q, cb = 2 * e + (p >> 1), off = 8 * (p & 1);
  const bf16x4 lo = trr(im + img(r0, cb) + off), hi = trr(im + img(r0 + 16, cb) + off);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 rowfrag(const char* im, int row, int lg) {
  return *reinterpret_cast<const bf16x8*>(im + img(row, lg));
}
__device__ __forceinline__ i32x4 rsrc(const void* base, long bytes) { return dma_rsrc(base, bytes); }
// LDS-DMA by inline asm (common.h dma_x4): no compiler-inserted ring drains
__device__ __forceinline__ void dma(const i32x4& r, const char* lds, int voff, int soff) {
  dma_x4(r, lds_addr(lds), voff, soff);
}
}  // namespace b32

__global__ __launch_bounds__(256) void attn_bwd_dkv32(int L, int H, const bf16* __restrict__ qkv, long ld,
                                                      const bf16* __restrict__ dO, long lddo,
                                                      const float* __restrict__ lse, const float* __restrict__ Dq,
                                                      bf16* __restrict__ dqkv, long ldd, float c_log2e, float scale,
                                                      int nkb, AttnDrop drop, long total_rows) {
  using namespace b32;
  constexpr int SLOT = 2 * TILE + 512;                  // Q image, dO image, 4 x [lse 16, D 16] f32
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = wg % nkb, sh = wg / nkb, h = sh % H, seq = sh / H;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int D = H * 32;
  const long row0 = (long)seq * L;
  const long srow = ((long)seq * H + h) * L;
  const int key = kb * 64 + wave * 16 + li;
  const uint32_t dbase = drop_base(drop.seed, (uint32_t)sh);
  const bf16x8 kf = key < L ? *reinterpret_cast<const bf16x8*>(qkv + (row0 + key) * ld + D + h * 32 + 8 * lg) : bf16x8{};
  bf16x8 vf = key < L ? *reinterpret_cast<const bf16x8*>(qkv + (row0 + key) * ld + 2 * D + h * 32 + 8 * lg) : bf16x8{};
  bf16x8 kf_ = kf;
  asm volatile("" : "+v"(kf_), "+v"(vf));        // retire the loads before the DMA ring (dma_x4)

  // this wave's pieces of a tile: Q / dO rows 16 wave + lane / 4 (image position lane % 4), and
  // lanes 0..3: lse / D of queries 16 wave + 4 lane .. + 3 (rows past L: the buffer's zeros)
  const i32x4 rq = rsrc(qkv + row0 * ld, (total_rows - row0) * ld * 2);
  const i32x4 ro = rsrc(dO + row0 * lddo, (total_rows - row0) * lddo * 2);
  const i32x4 rl = rsrc(lse + srow, (long)L * 4), rd = rsrc(Dq + srow, (long)L * 4);
  const int prow = 16 * wave + (lane >> 2), pc = img_src(prow, lane & 3);
  const int vq = (int)(prow * ld * 2) + (h * 32 + 8 * pc) * 2;
  const int vo = (int)(prow * lddo * 2) + (h * 32 + 8 * pc) * 2;
  const int vl = (16 * wave + 4 * lane) * 4;
  const int tq = (int)(64 * ld * 2), to = (int)(64 * lddo * 2);
  auto issue = [&](int t, int slot) {
    char* sl = smem + slot * SLOT;
    dma(rq, sl + wave * 1024, vq, t * tq);
    dma(ro, sl + TILE + wave * 1024, vo, t * to);
    if (lane < 4) {
      dma(rl, sl + 2 * TILE + wave * 128, vl, t * 256);
      dma(rd, sl + 2 * TILE + wave * 128 + 64, vl, t * 256);
    }
  };
  auto wait = [&](int y) {                              // all but the y youngest tiles (4 per tile)
    if (y >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (y == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x4 dk[2], dv[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) dk[e] = dv[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntile = (L + 63) / 64;
  const bool odd = li & 1;
  auto body = [&](const char* st, int t, auto mask_tag) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const char* qi = st;
    const char* oi = st + TILE;
    const float* lf = reinterpret_cast<const float*>(st + 2 * TILE);
    f32x4 s[4], dp[4], l4[4], d4[4];
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      s[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag(qi, 16 * qt + li, lg), kf_, z, 0, 0, 0);
      dp[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag(oi, 16 * qt + li, lg), vf, z, 0, 0, 0);
      l4[qt] = *reinterpret_cast<const f32x4*>(lf + qt * 32 + 4 * lg);
      d4[qt] = *reinterpret_cast<const f32x4*>(lf + qt * 32 + 16 + 4 * lg);
    }
    // dropout multipliers: the keys of a hash pair sit in lanes li, li ^ 1 with the same 16
    // queries; each lane hashes half of them and swaps with its neighbour over DPP
    float mkv[4][4];
    if (drop.thresh) {
      const uint32_t drow = drop_row(dbase, (uint32_t)(t * 64 + 4 * lg + (odd ? 2 : 0)), (uint32_t)key >> 1);
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const uint32_t hm = drop_mix24(drow + (uint32_t)(16 * qt + rr) * DROP_C1);
          const uint32_t ho = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hm, 0xB1, 0xF, 0xF, false);
          const uint32_t h_lo = odd ? ho : hm, h_hi = odd ? hm : ho;
          mkv[qt][rr] = (odd ? h_lo >> 16 : h_lo & 0xFFFFu) >= drop.thresh ? drop.scale : 0.f;
          mkv[qt][2 + rr] = (odd ? h_hi >> 16 : h_hi & 0xFFFFu) >= drop.thresh ? drop.scale : 0.f;
        }
    }
    bf16x8 pb[2], dsb[2];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = __builtin_amdgcn_exp2f(fmaf(s[qt][r], c_log2e, -l4[qt][r]));
        if constexpr (MASK) p = t * 64 + 16 * qt + 4 * lg + r < L ? p : 0.f;
        const float pm = drop.thresh ? p * mkv[qt][r] : p;
        pb[qt >> 1][(qt & 1) * 4 + r] = (bf16)pm;
        dsb[qt >> 1][(qt & 1) * 4 + r] = (bf16)fmaf(pm, dp[qt][r], -p * d4[qt][r]);
      }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        dv[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tfrag(oi, e, c, li, lg), pb[c], dv[e], 0, 0, 0);
        dk[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tfrag(qi, e, c, li, lg), dsb[c], dk[e], 0, 0, 0);
      }
  };
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < ntile) issue(j, j);
  auto step = [&](auto s_tag, int t) __attribute__((always_inline)) {
    constexpr int S = decltype(s_tag)::value;
    wait(NS - 2);                       // unrolled loop (t + NS <= ntile): NS - 2 younger tiles in flight
    __builtin_amdgcn_s_barrier();
    issue(t + NS - 1, (S + NS - 1) % NS);
    if ((t + 1) * 64 <= L) body(smem + S * SLOT, t, std::false_type{});
    else body(smem + S * SLOT, t, std::true_type{});
  };
  int t = 0;
  for (; t + NS <= ntile; t += NS) {
    step(std::integral_constant<int, 0>{}, t);
    step(std::integral_constant<int, 1>{}, t + 1);
    step(std::integral_constant<int, 2>{}, t + 2);
    step(std::integral_constant<int, 3>{}, t + 3);
  }
  for (; t < ntile; ++t) {
    wait(min(NS - 2, ntile - 1 - t));
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < ntile) issue(t + NS - 1, (t + NS - 1) % NS);
    if ((t + 1) * 64 <= L) body(smem + (t % NS) * SLOT, t, std::false_type{});
    else body(smem + (t % NS) * SLOT, t, std::true_type{});
  }
  if (key < L) {
    bf16* kp = dqkv + (row0 + key) * ldd + D + h * 32;
    bf16* vp = dqkv + (row0 + key) * ldd + 2 * D + h * 32;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      bf16x4 wk, wv;
#pragma unroll
      for (int r = 0; r < 4; ++r) { wk[r] = (bf16)(dk[e][r] * scale); wv[r] = (bf16)dv[e][r]; }
      *reinterpret_cast<bf16x4*>(kp + 16 * e + 4 * lg) = wk;
      *reinterpret_cast<bf16x4*>(vp + 16 * e + 4 * lg) = wv;
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq32(int L, int H, const bf16* __restrict__ qkv, long ld,
                                                     const bf16* __restrict__ O, long ldo,
                                                     const bf16* __restrict__ dO, long lddo,
                                                     const float* __restrict__ lse, float* __restrict__ Dout,
                                                     bf16* __restrict__ dqkv, long ldd, float c_log2e, float scale,
                                                     int nqb, AttnDrop drop, long total_rows) {
  using namespace b32;
  constexpr int SLOT = 2 * TILE;                        // K image, V image
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = wg % nqb, sh = wg / nqb, h = sh % H, seq = sh / H;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int D = H * 32;
  const long row0 = (long)seq * L;
  const int q = qb * 64 + wave * 16 + li;
  const bool qv = q < L;
  const bf16x8 qf = qv ? *reinterpret_cast<const bf16x8*>(qkv + (row0 + q) * ld + h * 32 + 8 * lg) : bf16x8{};
  const bf16x8 df = qv ? *reinterpret_cast<const bf16x8*>(dO + (row0 + q) * lddo + h * 32 + 8 * lg) : bf16x8{};
  const bf16x8 of = qv ? *reinterpret_cast<const bf16x8*>(O + (row0 + q) * ldo + h * 32 + 8 * lg) : bf16x8{};
  float dq_ = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) dq_ += (float)df[j] * (float)of[j];
  dq_ += __shfl_xor(dq_, 16, 64);
  dq_ += __shfl_xor(dq_, 32, 64);
  const long srow = ((long)seq * H + h) * L;
  float lse_q = qv ? lse[srow + q] : 0.f;
  const uint32_t dbase = drop_base(drop.seed, (uint32_t)sh);
  if (qv && lg == 0) Dout[srow + q] = dq_;
  bf16x8 qf_ = qf, df_ = df;
  asm volatile("" : "+v"(qf_), "+v"(df_), "+v"(lse_q));   // retire the loads before the DMA ring (dma_x4)

  const i32x4 rk = rsrc(qkv + row0 * ld, (total_rows - row0) * ld * 2);
  const int prow = 16 * wave + (lane >> 2), pc = img_src(prow, lane & 3);
  const int vk = (int)(prow * ld * 2) + (D + h * 32 + 8 * pc) * 2;
  const int vv = (int)(prow * ld * 2) + (2 * D + h * 32 + 8 * pc) * 2;
  const int tb = (int)(64 * ld * 2);
  auto issue = [&](int t, int slot) {
    char* sl = smem + slot * SLOT;
    dma(rk, sl + wave * 1024, vk, t * tb);
    dma(rk, sl + TILE + wave * 1024, vv, t * tb);
  };
  auto wait = [&](int y) {                              // 2 per tile
    if (y >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (y == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const int ntile = (L + 63) / 64;
  auto body = [&](const char* st, int t, auto mask_tag) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const char* ki = st;
    const char* vi = st + TILE;
    f32x4 s[4], dp[4];
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag(ki, 16 * kt + li, lg), qf_, z, 0, 0, 0);
      dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag(vi, 16 * kt + li, lg), df_, z, 0, 0, 0);
    }
    const uint32_t drow = drop_row(dbase, (uint32_t)q, (uint32_t)(32 * t + 2 * lg));
    bf16x8 dsb[2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        float dm[2] = {1.f, 1.f};
        if (drop.thresh) drop_split(drop, drop_mix24(drow + (uint32_t)(8 * kt + (r >> 1)) * DROP_C2), dm[0], dm[1]);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          float p = __builtin_amdgcn_exp2f(fmaf(s[kt][r + e], c_log2e, -lse_q));
          if constexpr (MASK) p = t * 64 + 16 * kt + 4 * lg + r + e < L ? p : 0.f;
          dsb[kt >> 1][(kt & 1) * 4 + r + e] = (bf16)(p * fmaf(dp[kt][r + e], dm[e], -dq_));
        }
      }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 2; ++e)
        acc[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tfrag(ki, e, c, li, lg), dsb[c], acc[e], 0, 0, 0);
  };
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < ntile) issue(j, j);
  auto step = [&](auto s_tag, int t) __attribute__((always_inline)) {
    constexpr int S = decltype(s_tag)::value;
    wait(NS - 2);                       // unrolled loop (t + NS <= ntile): NS - 2 younger tiles in flight
    __builtin_amdgcn_s_barrier();
    issue(t + NS - 1, (S + NS - 1) % NS);
    if ((t + 1) * 64 <= L) body(smem + S * SLOT, t, std::false_type{});
    else body(smem + S * SLOT, t, std::true_type{});
  };
  int t = 0;
  for (; t + NS <= ntile; t += NS) {
    step(std::integral_constant<int, 0>{}, t);
    step(std::integral_constant<int, 1>{}, t + 1);
    step(std::integral_constant<int, 2>{}, t + 2);
    step(std::integral_constant<int, 3>{}, t + 3);
  }
  for (; t < ntile; ++t) {
    wait(min(NS - 2, ntile - 1 - t));
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < ntile) issue(t + NS - 1, (t + NS - 1) % NS);
    if ((t + 1) * 64 <= L) body(smem + (t % NS) * SLOT, t, std::false_type{});
    else body(smem + (t % NS) * SLOT, t, std::true_type{});
  }
  if (qv) {
    bf16* op = dqkv + (row0 + q) * ldd + h * 32;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(acc[e][r] * scale);
      *reinterpret_cast<bf16x4*>(op + 16 * e + 4 * lg) = w;
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
  if constexpr (DH == 32) {
    const long rows = nseq * L;
    hipLaunchKernelGGL(attn_bwd_dq32, dim3((unsigned)grid), dim3(256), 0, s, (int)L, H, qkv, ld, O, ldo, dO, lddo,
                       lse, Dws, dqkv, ldd, cl, scale, nb, drop, rows);
    SNV_LAUNCH_CHECK();
    hipLaunchKernelGGL(attn_bwd_dkv32, dim3((unsigned)grid), dim3(256), 0, s, (int)L, H, qkv, ld, dO, lddo, lse,
                       (const float*)Dws, dqkv, ldd, cl, scale, nb, drop, rows);
    SNV_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(attn_bwd_dq<DH>, dim3((unsigned)grid), dim3(256), 0, s, (int)L, H, qkv, ld, O, ldo, dO, lddo,
                       lse, Dws, dqkv, ldd, cl, scale, nb, drop);
    SNV_LAUNCH_CHECK();
    hipLaunchKernelGGL(attn_bwd_dkv<DH>, dim3((unsigned)grid), dim3(256), 0, s, (int)L, H, qkv, ld, dO, lddo, lse,
                       (const float*)Dws, dqkv, ldd, cl, scale, nb, drop);
    SNV_LAUNCH_CHECK();
  }
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
