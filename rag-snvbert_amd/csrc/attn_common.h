// Tile geometry shared by the bf16 attention kernels (inference forward in
// attention.hip, training forward/backward in attention_train.hip).
#pragma once
#include "common.h"

namespace snvrag {

constexpr int AQ = 64;     // queries per workgroup
constexpr int AK = 64;     // keys per tile

template <int DH>
struct AttnCfg {
  static constexpr int KS = (DH + 31) / 32;        // 32-wide MFMA k-steps over head dim
  static constexpr int DP = KS * 32;               // padded head dim in the K tile
  static constexpr int KROWB = DP * 2;             // bytes per K-tile row
  static constexpr int CPR = DP / 8;               // 16-B chunks per K row
  static constexpr int RPC = 256 / KROWB;          // rows per 256-B bank cycle
  static constexpr int ET = DH / 16;               // 16-wide output d tiles
  static constexpr int VT_LD = AK + 8;             // V^T row stride (bf16), padded
  static constexpr int KBYTES = AK * KROWB;
  static constexpr int VBYTES = DP * VT_LD * 2;
  static constexpr int STAGE = KBYTES + VBYTES;
};

template <int DH>
__device__ __forceinline__ int k_off(int key, int chunk) {
  using C = AttnCfg<DH>;
  return key * C::KROWB + ((chunk ^ ((key / C::RPC) % C::CPR)) << 4);
}

// Attention-probability dropout (model/attention/attention.py:28-29) with a counter-based
// RNG, so the forward and both backward kernels regenerate the same keep mask.  One hash
// serves a key PAIR (2j, 2j + 1), 16 bits each:
//   h(q, j) = mix24(base + q * 0x9E3779B1 + j * 0x85EBCA77),
//   base    = fmix32(lo(seed) ^ fmix32(hi(seed) + sh * 0xC2B2AE3D)),   sh = seq * heads + head
//   mix24(h): h ^= h >> 16; h = lo32((h & 0xFFFFFF) * 0xEB352D); h ^= h >> 15;
//             h = lo32((h & 0xFFFFFF) * 0x6CA68B); h ^= h >> 16
// keep (q, k) iff half (k & 1) of h(q, k >> 1) >= thresh (thresh = round(p * 2^16), so the
// drop probability is p to within 2^-17); kept probabilities are scaled by 1 / (1 - p).
// mix24 is the lowbias32 mixer with 24-bit multiplies (v_mul_u32_u24, full VALU rate) instead
// of the quarter-rate 32-bit ones of fmix32: the mask is hashed per probability pair inside the
// VALU-issue-bound attention loops (head dim 32), where fmix32's two v_mul_lo_u32 dominated the
// dropout cost.  Callers keep the hash input additive (drop_row + pair offset * C2) so the
// per-element work is one add plus the mixer.  thresh == 0: no dropout.
// (tests/attn_helpers.py restates it; tests/test_host_cpu.py checks the mask statistics.)
struct AttnDrop {
  uint32_t thresh;
  float scale;
  uint64_t seed;
};
constexpr uint32_t DROP_C1 = 0x9E3779B1u;     // query multiplier
constexpr uint32_t DROP_C2 = 0x85EBCA77u;     // key-pair multiplier
__host__ __device__ inline uint32_t drop_fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_mix24(uint32_t h) {
  h ^= h >> 16;
  h = __umul24(h, 0xEB352Du);
  h ^= h >> 15;
  h = __umul24(h, 0x6CA68Bu);
  h ^= h >> 16;
  return h;
}
__host__ __device__ inline uint32_t drop_base(uint64_t seed, uint32_t sh) {
  return drop_fmix32((uint32_t)seed ^ drop_fmix32((uint32_t)(seed >> 32) + sh * 0xC2B2AE3Du));
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t base, uint32_t q, uint32_t pair) {
  return drop_mix24(base + q * DROP_C1 + pair * DROP_C2);
}
// hash input of (q, pair0): add dpair * DROP_C2 for pair0 + dpair
__device__ __forceinline__ uint32_t drop_row(uint32_t base, uint32_t q, uint32_t pair0) {
  return base + q * DROP_C1 + pair0 * DROP_C2;
}
// multipliers of the two keys of a pair from its hash
__device__ __forceinline__ void drop_split(const AttnDrop& d, uint32_t h, float& m0, float& m1) {
  m0 = (h & 0xFFFFu) >= d.thresh ? d.scale : 0.f;
  m1 = (h >> 16) >= d.thresh ? d.scale : 0.f;
}
// probabilities of a key pair after dropout: w = the packed bf16 pair (key 2i low half, 2i + 1
// high half), h = the pair's hash.  A half is dropped iff its hash half < thresh, i.e. iff
// (hash half - thresh) is negative, whose bits 16..31 are then all ones: one byte permute
// gathers those bits of both differences into a drop mask and the kept halves pass unscaled
// (the 1 / (1 - p) scale is applied once to the output).  4 VALU ops per pair instead of two
// compares, two selects, two multiplies and a second conversion.
__device__ __forceinline__ uint32_t drop_pair_apply(uint32_t w, uint32_t h, uint32_t thresh) {
  const uint32_t xlo = (h & 0xFFFFu) - thresh, xhi = (h >> 16) - thresh;
  const uint32_t m = __builtin_amdgcn_perm(xhi, xlo, 0x07060302u);   // [xlo.b2, xlo.b3, xhi.b2, xhi.b3]
  return w & ~m;
}
// dropout multiplier of probability (q, k): 0 or 1 / (1 - p)
__device__ __forceinline__ float drop_mul(const AttnDrop& d, uint32_t base, uint32_t q, uint32_t k) {
  const uint32_t h = drop_hash(base, q, k >> 1);
  return ((k & 1u) ? h >> 16 : h & 0xFFFFu) >= d.thresh ? d.scale : 0.f;
}
// multipliers of (q, k) and (q, k + 1) for even k: one hash
__device__ __forceinline__ void drop_mul2(const AttnDrop& d, uint32_t base, uint32_t q, uint32_t k, float& m0,
                                          float& m1) {
  drop_split(d, drop_hash(base, q, k >> 1), m0, m1);
}
static inline AttnDrop make_attn_drop(float p, uint64_t seed) {
  AttnDrop d;
  const double t = (double)p * 65536.0 + 0.5;
  d.thresh = p > 0.f ? (t < 1.0 ? 1u : (uint32_t)t) : 0u;
  d.scale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  d.seed = seed;
  return d;
}

}  // namespace snvrag
