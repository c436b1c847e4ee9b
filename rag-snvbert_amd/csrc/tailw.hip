// Block tail, wide-row form (option tail_wide), D = 384, eval — the same function as tail_kernel
// (csrc/tail.hip) on the same packed weight stream and vector tables:
//
//   x1  = LN1(x + att W_o^T + b_o)                     multi_head_attention.py:51, sublayer.py:15-16
//   x   = LN2(x1 + lrelu(LN_f(lrelu(x1 W1^T + b1)) W2^T + b2))   feed_forward.py:18-21
//
// tail_kernel gives each wave 32 token rows and ALL features, so every weight fragment is read
// from LDS by all four waves and the 2.65 MB stream enters each CU by LDS-DMA, whose issue cost
// (~60 cycles per 1 KiB piece, serialised with the wave's MFMAs at one wave per SIMD) caps it at
// ~41 % of the MFMA peak.  Here the roles are transposed, like the wide-row GEMM (gemm256.hip):
// a workgroup owns 128 rows (4 token groups of 32) and wave w owns FEATURES — output tiles
// 3w .. 3w+2 of the out-projection and of FFN2, and hidden chunks 4c + w of FFN1 — so every W
// fragment is loaded ONCE per workgroup straight into the registers of the one wave that uses it
// (buffer_load_dwordx4, three k16 steps ahead) and feeds four MFMAs (one per token group); the
// activations are the LDS-resident operands instead:
//   X [24 k16 steps][4 groups] x 1 KiB B-fragment images (96 KiB): att by LDS-DMA in the prologue,
//     then x1 (written by LN1, read by every FFN1 k-step and as the LN2 residual);
//   H [4 chunks][4 k16 steps][4 groups] x 1 KiB (64 KiB): the bf16 hidden of one round of four
//     64-unit chunks (one per wave), the B fragments of FFN2 — the packed W2' k order makes a
//     lane's 8 consecutive FFN1 accumulators exactly its 16-B slot of an FFN2 B fragment.
// Per round c (6 rounds): FFN1 of chunk 4c + w (24 k16 steps x 2 tiles x 4 groups = 192 MFMAs),
// barrier, the chunk epilogue (b1, LeakyReLU, LN_f sums, bf16 into H), barrier, FFN2 over the
// round's 4 chunks (16 k16 steps x 3 tiles x 4 groups = 192 MFMAs).  Row statistics (LN1, LN_f,
// LN2) are per-wave partials combined through LDS.
// The W fragment loads are inline asm with hand-counted s_waitcnt vmcnt (tw_younger): the
// compiler sees no loads, so it neither drains them at loop edges nor reorders around them; the
// MFMAs are inline asm too (fixed AGPR / VGPR accumulators), so every accumulator read waits for
// tw_drain() (the compiler's hazard recognizer does not know these are MFMAs).
#include "common.h"

#include <utility>

namespace snvrag {

constexpr int TW_D = 384, TW_NT = 12, TW_KS = 24;
constexpr int TW_FRAG = 1024;
constexpr int TW_FPRE = TW_NT * TW_KS;               // W_o' fragments (288)
constexpr int TW_FPC = 96;                           // fragments per 64-unit chunk: W1 48, W2' 48
constexpr int TW_NFRAG = TW_FPRE + 24 * TW_FPC;      // whole stream (2592)
constexpr int TW_X = 0;                              // LDS: X images (96 KiB)
constexpr int TW_H = 96 * 1024;                      // LDS: H images (64 KiB)
constexpr int TW_LDS = 160 * 1024;
constexpr int TW_L = 3;                              // k16 steps of W loads in flight ahead
constexpr int TW_R = TW_L + 1;                       // W register slots (divides 24 and 40)
constexpr int TW_QA = 24;                            // phase-A (out-projection) steps
constexpr int TW_RS = 40;                            // steps per FFN round: 24 FFN1 + 16 FFN2
constexpr int TW_IB = 20;                            // FFN1 step after which the chunk's b1 loads issue
constexpr int TW_NB1 = 8;                            // b1 loads per chunk
static_assert(TW_QA % TW_R == 0 && TW_RS % TW_R == 0, "W slots periodic over phase A and the rounds");

// W fragments loaded for global step q (phase A: 3 W_o' tiles; FFN1: 2 W1 tiles; FFN2: 3 W2' tiles)
__host__ __device__ constexpr int tw_nf(int q) { return q < TW_QA ? 3 : ((q - TW_QA) % TW_RS < 24 ? 2 : 3); }
// other vector-memory ops a wave issues during step q, after that step's W loads (the b1 loads)
__host__ __device__ constexpr int tw_extra(int q) { return q >= TW_QA && (q - TW_QA) % TW_RS == TW_IB ? TW_NB1 : 0; }
// vector-memory ops issued after step q's W loads up to the wait before step q's MFMAs: the loads
// of steps q+1 .. q+L-1 (issued during steps q-L+1 .. q-1) and the extras of steps q-L .. q-1
__host__ __device__ constexpr int tw_younger(int q) {
  int n = 0;
  for (int j = 1; j < TW_L; ++j) n += tw_nf(q + j);
  for (int j = q - TW_L; j < q; ++j)
    if (j >= 0) n += tw_extra(j);
  return n;
}
// ops issued after the b1 loads (during step IB) up to the chunk epilogue (after step 23)
__host__ __device__ constexpr int tw_b1_younger() {
  int n = 0;
  for (int i = TW_IB + 1; i < 24; ++i) n += tw_nf(TW_QA + i + TW_L);
  return n;
}
static_assert(tw_younger(TW_QA + TW_RS) == tw_younger(TW_QA) && tw_younger(TW_QA + TW_RS + 1) == tw_younger(TW_QA + 1) &&
                  tw_younger(TW_QA + TW_RS + 2) == tw_younger(TW_QA + 2),
              "round waits periodic");

template <typename Body, int... Is>
__device__ __forceinline__ void tw_unroll(Body&& body, std::integer_sequence<int, Is...>) {
  (body(std::integral_constant<int, Is>{}), ...);
}
template <bool AGPR>
__device__ __forceinline__ void tw_mfma(f32x16& c, const u32x4& a, const u32x4& b) {
  if constexpr (AGPR)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
// zero C operand: the accumulator's first k-step
template <bool AGPR>
__device__ __forceinline__ void tw_mfma0(f32x16& c, const u32x4& a, const u32x4& b) {
  if constexpr (AGPR)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
}
// a 32x32x16 result is readable 18 wait states after issue
__device__ __forceinline__ void tw_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
// the drain with the accumulators as operands: no read or register move of them (a compiler copy is
// not a memory access and crossed the plain drain) can be scheduled before it
__device__ __forceinline__ void tw_drain_o(f32x16 (&a)[3][4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+a"(a[0][0]), "+a"(a[0][1]), "+a"(a[0][2]), "+a"(a[0][3]), "+a"(a[1][0]), "+a"(a[1][1]),
                 "+a"(a[1][2]), "+a"(a[1][3]), "+a"(a[2][0]), "+a"(a[2][1]), "+a"(a[2][2]), "+a"(a[2][3])
               :: "memory");
}
__device__ __forceinline__ void tw_drain_h(f32x16 (&h)[2][4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+v"(h[0][0]), "+v"(h[1][0]), "+v"(h[0][1]), "+v"(h[1][1]), "+a"(h[0][2]), "+a"(h[1][2]),
                 "+a"(h[0][3]), "+a"(h[1][3])
               :: "memory");
}
__device__ __forceinline__ int tw_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ uint32_t tw_pack2(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}
__device__ __forceinline__ float tw_lrelu(float x) {
  float r;
  asm("v_mul_f32 %0, 0x3dcccccd, %1\n v_max_f32 %0, %1, %0" : "=&v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ float tw_bf(const u32x4& v, int j) {
  return (j & 1) ? __uint_as_float(v[j >> 1] & 0xffff0000u) : __uint_as_float(v[j >> 1] << 16);
}
__device__ __forceinline__ float tw_xsum32(float x) {
  return x + __int_as_float(__builtin_amdgcn_ds_bpermute((tw_lane() ^ 32) << 2, __float_as_int(x)));
}
// 16 consecutive floats of an LDS table (reads and their wait in one statement)
__device__ __forceinline__ void tw_ld16(uint32_t addr, float (&v)[16]) {
  u32x4 r[4];
  asm volatile(
      "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
      " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "v"(addr));
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = __uint_as_float(r[i >> 2][i & 3]);
}
// wait until at most Y younger vector-memory ops are in flight; w's uses are ordered after it
template <int Y> __device__ __forceinline__ void tw_waitw(u32x4 (&w)[3]) {
  static_assert(Y >= 0 && Y <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]) : "n"(Y) : "memory");
}
template <int OFF> __device__ __forceinline__ void tw_load_off(u32x4& r, int voff, const i32x4& rsrc, int so) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4" : "=v"(r) : "v"(voff), "s"(rsrc), "s"(so), "n"(OFF) : "memory");
}
__device__ __forceinline__ void tw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct TwArgs {
  int M;
  const bf16* att;          // [M, D]
  const bf16* resid;        // [M, D] (x; out may alias it)
  bf16* out;                // [M, D]
  const char* ws;           // snvrag_tail_pack stream
  const float* vec;         // [b1 4D | b2' | c1 | g2 | be2]
  const float* b_o; const float* g1; const float* be1;
  float eps;
  int desync;
  unsigned long long* stamps;   // VAR 1: [workgroup][wave][8] s_memtime stamps
};

template <int VAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void tailw_kernel(TwArgs p) {
  constexpr int D = TW_D, NT = TW_NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long row0 = (long)blockIdx.x * 128;
  unsigned long long st[8];
  auto stamp = [&](int i) {
    if constexpr (VAR == 1) st[i] = __builtin_amdgcn_s_memtime();
  };
  // first-round stagger (tail.hip): later rounds' prologue bursts overlap other CUs' MFMAs
  if (p.desync > 0 && blockIdx.x < 256) {
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }
  stamp(0);
  const uint32_t lds0 = lds_addr(smem);
  int lane16 = tw_lane() * 16;                        // (lane-derived values are re-made from a fresh
  asm volatile("" : "+v"(lane16));                    //  v_mbcnt where used: kept live across the FFN they spill)

  // ---- prologue: att -> X by LDS-DMA (wave w: token group w, k16 steps in order; lane (n, kh) of
  // piece s reads att[32 w + n][tail_in_feat(s, kh, 0 .. 7)]), the first W steps, the residual rows
  // (VGPRs, used by LN1), the LN1 tables -> H
  const i32x4 ars = dma_rsrc(p.att + row0 * D, ((long)p.M - row0) * D * 2);   // rows >= M read as 0
  const i32x4 wrs = dma_rsrc(p.ws, (long)TW_NFRAG * TW_FRAG);
  const i32x4 brs = dma_rsrc(p.vec, 4L * D * 4);                             // b1
  {
    const int l = tw_lane();
    const int voff = (32 * wave + (l & 31)) * (D * 2) + 32 * (l >> 5);
#pragma unroll
    for (int s = 0; s < TW_KS; ++s)
      dma_x4(ars, lds0 + TW_X + (s * 4 + wave) * TW_FRAG, voff, 64 * (s >> 1) + 16 * (s & 1));
  }
  u32x4 wr[TW_R][3];
  // W fragment F of the stream into register r (soffset: scalar)
  auto loadW = [&](u32x4& r, int F) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(r) : "v"(lane16), "s"(wrs), "s"(F * TW_FRAG) : "memory");
  };
  // the loads of global step q (compile-time position in the pattern; c = its round, runtime)
  auto issueW = [&](auto q_tag, int c) {
    constexpr int q = decltype(q_tag)::value;
    constexpr int slot = q % TW_R;
    if constexpr (q < TW_QA) {
#pragma unroll
      for (int t = 0; t < 3; ++t) loadW(wr[slot][t], q * NT + 3 * wave + t);
    } else {
      constexpr int i = (q - TW_QA) % TW_RS;
      const int cc = c < 5 ? c : 5;                  // overrun steps past the last round re-read it
      if constexpr (i < 24) {
#pragma unroll
        for (int t = 0; t < 2; ++t) loadW(wr[slot][t], TW_FPRE + (4 * cc + wave) * TW_FPC + 2 * i + t);
      } else {
        constexpr int u = i - 24, cl = u >> 2, s2 = u & 3;
#pragma unroll
        for (int t = 0; t < 3; ++t) loadW(wr[slot][t], TW_FPRE + (4 * cc + cl) * TW_FPC + 48 + s2 * NT + 3 * wave + t);
      }
    }
  };
  tw_unroll([&](auto qc) { issueW(qc, 0); }, std::make_integer_sequence<int, TW_L>{});
  u32x4 rr[3][4][2];                                 // residual x: tile t, group g, half h2
  {
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      long r = row0 + 32 * g + (l & 31);
      r = r < p.M ? r : (long)p.M - 1;
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          rr[t][g][h2] = *reinterpret_cast<const u32x4*>(p.resid + r * D + 32 * (3 * wave + t) + 16 * (l >> 5) + 8 * h2);
    }
  }
  float* tab = reinterpret_cast<float*>(smem + TW_H);                        // [b_o | g1 | be1]
  for (int i = threadIdx.x; i < D; i += 256) {
    tab[i] = p.b_o[i];
    tab[D + i] = p.g1[i];
    tab[2 * D + i] = p.be1[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the residual rows retired here (else the compiler's wait for them lands at LN1, behind the
  // in-flight W loads of the first FFN steps)
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) asm volatile("" : "+v"(rr[t][g][0]), "+v"(rr[t][g][1]));
  tw_barrier();
  stamp(1);

  // ---- phase A: ao = att W_o'^T (wave w: tiles 3w .. 3w+2 x 4 token groups, AGPRs)
  f32x16 acc[3][4];
  u32x4 bq[2][4];
  auto rdB = [&](uint32_t base, int blk) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(smem + base + blk * TW_FRAG + lane16);
  };
  auto waitW = [&](auto q_tag) {
    constexpr int q = decltype(q_tag)::value;
    tw_waitw<tw_younger(q)>(wr[q % TW_R]);
  };
#pragma unroll
  for (int g = 0; g < 4; ++g) bq[0][g] = rdB(TW_X, g);
  tw_unroll([&](auto qc) {
    constexpr int q = decltype(qc)::value, slot = q % TW_R;
    waitW(qc);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        if constexpr (q == 0) tw_mfma0<true>(acc[t][g], wr[slot][t], bq[q & 1][g]);
        else tw_mfma<true>(acc[t][g], wr[slot][t], bq[q & 1][g]);
      }
      if constexpr (q + 1 < TW_KS) bq[(q + 1) & 1][g] = rdB(TW_X, (q + 1) * 4 + g);
      if (g == 1) issueW(std::integral_constant<int, q + TW_L>{}, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }, std::make_integer_sequence<int, TW_QA>{});
  tw_drain_o(acc);
  stamp(2);

  // ---- LN1 over the 4 waves' features: v = ao + b_o + x; per-wave (sum, sumsq) -> LDS
  float2* s1 = reinterpret_cast<float2*>(smem + TW_H + 8 * 1024);          // [wave][128 rows]
  {
    const uint32_t tb = lds0 + TW_H + 64 * (tw_lane() >> 5);
    float sum[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float bo[16];
      tw_ld16(tb + 4 * 32 * (3 * wave + t), bo);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = acc[t][g][i] + bo[i] + tw_bf(rr[t][g][i >> 3], i & 7);
          acc[t][g][i] = v;
          sum[g] += v;
          sq[g] = fmaf(v, v, sq[g]);
        }
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) asm volatile("" : "+a"(acc[t][g]));   // v back in AGPRs
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      sum[g] = tw_xsum32(sum[g]);
      sq[g] = tw_xsum32(sq[g]);
      s1[wave * 128 + 32 * g + (l & 31)] = make_float2(sum[g], sq[g]);
    }
  }
  tw_barrier();                                       // every wave past phase A: X is free for x1
  {
    const int l = tw_lane();
    const uint32_t tb = lds0 + TW_H + 64 * (l >> 5);
    float mean[4], rstd[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) {
        const float2 v = s1[w2 * 128 + 32 * g + (l & 31)];
        a += v.x;
        b += v.y;
      }
      mean[g] = a * (1.0f / D);
      rstd[g] = 1.0f / sqrtf(fmaxf(b * (1.0f / D) - mean[g] * mean[g], 0.f) + p.eps);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float gg[16], bb[16];
      tw_ld16(tb + 4 * (D + 32 * (3 * wave + t)), gg);
      tw_ld16(tb + 4 * (2 * D + 32 * (3 * wave + t)), bb);
      const int T = 3 * wave + t;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float y[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = (acc[t][g][i] - mean[g]) * rstd[g] * gg[i] + bb[i];
        // x1 features 32T + 16hh + 8h2 + j = k16 step 2T + h2, lane slot (n, kh = hh)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          *reinterpret_cast<u32x4*>(smem + TW_X + ((2 * T + h2) * 4 + g) * TW_FRAG + lane16) =
              u32x4{tw_pack2(y[8 * h2], y[8 * h2 + 1]), tw_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                    tw_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tw_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
      }
    }
  }
  tw_barrier();                                       // x1 complete in X
  stamp(3);

  // ---- FFN rounds
#pragma unroll
  for (int g = 0; g < 4; ++g) bq[0][g] = rdB(TW_X, g);
  f32x16 hac[2][4];                                   // FFN1 accumulators: groups 0, 1 VGPRs, 2, 3 AGPRs
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[t][g] = f32x16{};
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) asm volatile("" : "+a"(acc[t][g]));
  float st1[4] = {0.f, 0.f, 0.f, 0.f}, st2[4] = {0.f, 0.f, 0.f, 0.f};
  u32x4 b1v[2][4];
#pragma unroll 1
  for (int c = 0; c < 6; ++c) {
    // FFN1: hac = x1 W1_{4c+w}^T (k16 step i: tiles t = 0, 1 of the chunk)
    tw_unroll([&](auto ic) {
      constexpr int i = decltype(ic)::value, q = TW_QA + i;
      constexpr int slot = q % TW_R;
      waitW(std::integral_constant<int, q>{});
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if constexpr (i == 0) {
            if (g < 2) tw_mfma0<false>(hac[t][g], wr[slot][t], bq[i & 1][g]);
            else tw_mfma0<true>(hac[t][g], wr[slot][t], bq[i & 1][g]);
          } else {
            if (g < 2) tw_mfma<false>(hac[t][g], wr[slot][t], bq[i & 1][g]);
            else tw_mfma<true>(hac[t][g], wr[slot][t], bq[i & 1][g]);
          }
        }
        if constexpr (i + 1 < 24) bq[(i + 1) & 1][g] = rdB(TW_X, (i + 1) * 4 + g);
        if (g == 1) issueW(std::integral_constant<int, q + TW_L>{}, c);
      }
      if constexpr (i == TW_IB) {
        // b1 of chunk 4c + w: bv[t][r] = b1[64 (4c + w) + 32 t + 8 r + 4 hh .. + 3]
        const int so = 4 * 64 * (4 * c + wave);
        tw_unroll([&](auto kc) {
          constexpr int k = decltype(kc)::value, t = k >> 2, r = k & 3;
          tw_load_off<4 * (32 * t + 8 * r)>(b1v[t][r], 16 * (tw_lane() >> 5), brs, so);
        }, std::make_integer_sequence<int, 8>{});
      }
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, 24>{});
    tw_drain_h(hac);
    asm volatile("s_barrier" ::: "memory");           // every wave done reading H (last round's FFN2)
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(b1v[0][0]), "+v"(b1v[0][1]), "+v"(b1v[0][2]), "+v"(b1v[0][3]), "+v"(b1v[1][0]),
                   "+v"(b1v[1][1]), "+v"(b1v[1][2]), "+v"(b1v[1][3])
                 : "n"(tw_b1_younger()) : "memory");
    // chunk epilogue: h = lrelu(acc + b1), LN_f sums, bf16 -> H block (w, 2t + h2, g), this lane's slot
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float h[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          h[i] = tw_lrelu(hac[t][g][i] + __uint_as_float(b1v[t][i >> 2][i & 3]));
          st1[g] += h[i];
          st2[g] = fmaf(h[i], h[i], st2[g]);
        }
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          *reinterpret_cast<u32x4*>(smem + TW_H + ((wave * 4 + 2 * t + h2) * 4 + g) * TW_FRAG + lane16) =
              u32x4{tw_pack2(h[8 * h2], h[8 * h2 + 1]), tw_pack2(h[8 * h2 + 2], h[8 * h2 + 3]),
                    tw_pack2(h[8 * h2 + 4], h[8 * h2 + 5]), tw_pack2(h[8 * h2 + 6], h[8 * h2 + 7])};
      }
    tw_barrier();                                     // the round's hidden complete in H
#pragma unroll
    for (int g = 0; g < 4; ++g) bq[0][g] = rdB(TW_H, g);
    // FFN2: acc += W2'_{4c+cl} h^T (k16 step u = 4 cl + s2: tiles 3w .. 3w+2)
    tw_unroll([&](auto uc) {
      constexpr int u = decltype(uc)::value, q = TW_QA + 24 + u;
      constexpr int slot = q % TW_R;
      waitW(std::integral_constant<int, q>{});
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int t = 0; t < 3; ++t) tw_mfma<true>(acc[t][g], wr[slot][t], bq[u & 1][g]);
        if constexpr (u + 1 < 16) bq[(u + 1) & 1][g] = rdB(TW_H, (u + 1) * 4 + g);
        else bq[(u + 1) & 1][g] = rdB(TW_X, g);       // the next round's first FFN1 step
        if (g == 1) issueW(std::integral_constant<int, q + TW_L>{}, c + (q + TW_L >= TW_QA + TW_RS ? 1 : 0));
      }
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, 16>{});
    tw_drain_o(acc);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the overrun loads have landed
  stamp(4);

  // ---- epilogue: out = LN2(x1 + lrelu(rstd_f (acc - mean_f c1) + b2'))
  float2* s2 = reinterpret_cast<float2*>(smem + TW_H + 8 * 1024);
  float2* s3 = reinterpret_cast<float2*>(smem + TW_H + 12 * 1024);
  float* et = reinterpret_cast<float*>(smem + TW_H);  // [b2' | c1 | g2 | be2]
  asm volatile("s_barrier" ::: "memory");             // every wave done reading H
  {
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      st1[g] = tw_xsum32(st1[g]);
      st2[g] = tw_xsum32(st2[g]);
      s2[wave * 128 + 32 * g + (l & 31)] = make_float2(st1[g], st2[g]);
    }
    for (int i = threadIdx.x; i < 4 * D; i += 256) et[i] = p.vec[4 * D + i];
  }
  tw_barrier();
  float hm[4], hr[4];
  {
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) {
        const float2 v = s2[w2 * 128 + 32 * g + (l & 31)];
        a += v.x;
        b += v.y;
      }
      hm[g] = a * (1.0f / (4 * D));
      hr[g] = 1.0f / sqrtf(fmaxf(b * (1.0f / (4 * D)) - hm[g] * hm[g], 0.f) + p.eps);
    }
  }
  const uint32_t eb = lds0 + TW_H + 64 * (tw_lane() >> 5);
  {
    float sum[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int T = 3 * wave + t;
      float b2[16], c1[16];
      tw_ld16(eb + 4 * (32 * T), b2);
      tw_ld16(eb + 4 * (D + 32 * T), c1);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u32x4 xa = rdB(TW_X, (2 * T) * 4 + g), xb = rdB(TW_X, (2 * T + 1) * 4 + g);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float u = hr[g] * fmaf(-hm[g], c1[i], acc[t][g][i]) + b2[i];
          u = tw_lrelu(u);
          const float v = u + tw_bf(i < 8 ? xa : xb, i & 7);
          acc[t][g][i] = v;
          sum[g] += v;
          sq[g] = fmaf(v, v, sq[g]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) asm volatile("" : "+a"(acc[t][g]));
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      sum[g] = tw_xsum32(sum[g]);
      sq[g] = tw_xsum32(sq[g]);
      s3[wave * 128 + 32 * g + (l & 31)] = make_float2(sum[g], sq[g]);
    }
  }
  tw_barrier();
  {
    const int l = tw_lane();
    float mean[4], rstd[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) {
        const float2 v = s3[w2 * 128 + 32 * g + (l & 31)];
        a += v.x;
        b += v.y;
      }
      mean[g] = a * (1.0f / D);
      rstd[g] = 1.0f / sqrtf(fmaxf(b * (1.0f / D) - mean[g] * mean[g], 0.f) + p.eps);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int T = 3 * wave + t;
      float g2[16], be2[16];
      tw_ld16(eb + 4 * (2 * D + 32 * T), g2);
      tw_ld16(eb + 4 * (3 * D + 32 * T), be2);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const long r = row0 + 32 * g + (l & 31);
        const float nmr = -mean[g] * rstd[g];
        float y[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = fmaf(fmaf(acc[t][g][i], rstd[g], nmr), g2[i], be2[i]);
        if (r < p.M) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
            *reinterpret_cast<u32x4*>(p.out + r * D + 32 * T + 16 * (l >> 5) + 8 * h2) =
                u32x4{tw_pack2(y[8 * h2], y[8 * h2 + 1]), tw_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                      tw_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tw_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
        }
      }
    }
  }
  if constexpr (VAR == 1) {
    stamp(5);
    if ((threadIdx.x & 63) == 0 && p.stamps) {
#pragma unroll
      for (int i = 0; i < 6; ++i) p.stamps[((long)blockIdx.x * 4 + wave) * 8 + i] = st[i];
    }
  }
}

int tailw_launch(int M, const void* att, const void* resid, void* out, const void* ws, const float* vec,
                 const float* b_o, const float* g1, const float* be1, float eps, int desync, int var,
                 hipStream_t s) {
  TwArgs a{M, (const bf16*)att, (const bf16*)resid, (bf16*)out, (const char*)ws, vec, b_o, g1, be1, eps, desync,
           diag_stamps()};
  auto kern = (var == 1 && a.stamps) ? tailw_kernel<1> : tailw_kernel<0>;
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, TW_LDS));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(M, 128)), dim3(256), TW_LDS, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

}  // namespace snvrag
