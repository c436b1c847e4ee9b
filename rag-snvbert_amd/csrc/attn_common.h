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
// serves a key PAIR (2j, 2j + 1), 16 bits each — the mask costs half the integer multiplies
// of a hash per probability in the kernels whose lanes hold consecutive keys:
//   h(q, j) = fmix32(base + q * 0x9E3779B1 + j * 0x85EBCA77),
//   base    = fmix32(lo(seed) ^ fmix32(hi(seed) + sh * 0xC2B2AE3D)),   sh = seq * heads + head
// keep (q, k) iff half (k & 1) of h(q, k >> 1) >= thresh (thresh = round(p * 2^16), so the
// drop probability is p to within 2^-17); kept probabilities are scaled by 1 / (1 - p).
// thresh == 0: no dropout.  (tests/attn_helpers.py restates it for the parity tests.)
struct AttnDrop {
  uint32_t thresh;
  float scale;
  uint64_t seed;
};
__host__ __device__ inline uint32_t drop_fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ inline uint32_t drop_base(uint64_t seed, uint32_t sh) {
  return drop_fmix32((uint32_t)seed ^ drop_fmix32((uint32_t)(seed >> 32) + sh * 0xC2B2AE3Du));
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t base, uint32_t q, uint32_t pair) {
  return drop_fmix32(base + q * 0x9E3779B1u + pair * 0x85EBCA77u);
}
// dropout multiplier of probability (q, k): 0 or 1 / (1 - p)
__device__ __forceinline__ float drop_mul(const AttnDrop& d, uint32_t base, uint32_t q, uint32_t k) {
  const uint32_t h = drop_hash(base, q, k >> 1);
  return ((k & 1u) ? h >> 16 : h & 0xFFFFu) >= d.thresh ? d.scale : 0.f;
}
// multipliers of (q, k) and (q, k + 1) for even k: one hash
__device__ __forceinline__ void drop_mul2(const AttnDrop& d, uint32_t base, uint32_t q, uint32_t k, float& m0,
                                          float& m1) {
  const uint32_t h = drop_hash(base, q, k >> 1);
  m0 = (h & 0xFFFFu) >= d.thresh ? d.scale : 0.f;
  m1 = (h >> 16) >= d.thresh ? d.scale : 0.f;
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
