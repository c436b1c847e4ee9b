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

}  // namespace snvrag
