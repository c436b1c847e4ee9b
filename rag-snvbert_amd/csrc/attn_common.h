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
// RNG, so the forward and both backward kernels regenerate the same keep mask:
//   h(q, k) = fmix32(base + q * 0x9E3779B1 + k * 0x85EBCA77),
//   base    = fmix32(lo(seed) ^ fmix32(hi(seed) + sh * 0xC2B2AE3D)),   sh = seq * heads + head
// keep iff h >= thresh (thresh = p * 2^32); kept probabilities are scaled by 1 / (1 - p).
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
// dropout multiplier of probability (q, k): 0 or 1 / (1 - p)
__device__ __forceinline__ float drop_mul(const AttnDrop& d, uint32_t base, uint32_t q, uint32_t k) {
  return drop_fmix32(base + q * 0x9E3779B1u + k * 0x85EBCA77u) >= d.thresh ? d.scale : 0.f;
}
static inline AttnDrop make_attn_drop(float p, uint64_t seed) {
  AttnDrop d;
  d.thresh = p > 0.f ? (uint32_t)((double)p * 4294967296.0) : 0u;
  d.scale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  d.seed = seed;
  return d;
}

}  // namespace snvrag
