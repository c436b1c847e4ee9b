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

#ifndef TW_PACKED_LN
#define TW_PACKED_LN 1                               // LayerNorm epilogues in packed f32 (v_pk_*) math
#endif

constexpr int TW_D = 384, TW_NT = 12, TW_KS = 24;
constexpr int TW_FRAG = 1024;
constexpr int TW_FPRE = TW_NT * TW_KS;               // W_o' fragments (288)
constexpr int TW_FPC = 96;                           // fragments per 64-unit chunk: W1 48, W2' 48
constexpr int TW_NFRAG = TW_FPRE + 24 * TW_FPC;      // whole stream (2592)
constexpr int TW_X = 0;                              // LDS: X images (96 KiB)
constexpr int TW_H = 96 * 1024;                      // LDS: H images (64 KiB)
constexpr int TW_LDS = 160 * 1024;
// W fragments: one stream per wave in consumption order, TW_AH fragments in flight ahead of the
// step being consumed, in a ring of TW_RING registers (fragment n in register n % 12)
constexpr int TW_AH = 9;
constexpr int TW_RING = 12;
// k16 steps: q in [0, 24) phase A (3 W_o' fragments each); [24, 48) FFN1 of half-round 0 (1 W1
// fragment); half-round h = 1 .. 11: 32 steps at 48 + 32 (h - 1): FFN1(h) x 24 (1), FFN2(h - 1) x 8
// (3 W2' fragments); [400, 408) FFN2(11)
constexpr int TW_QA = 24;
constexpr int TW_Q0 = 48;
constexpr int TW_HS = 32;
constexpr int TW_QF = TW_Q0 + 11 * TW_HS;
constexpr int TW_QEND = TW_QF + 8;
constexpr int TW_QREP = TW_Q0 + TW_HS;               // half-round 2: the loop's representative steps
constexpr int TW_NB1 = 4;                            // b1 loads of one half-round's tile

__host__ __device__ constexpr int tw_nf(int q) {
  return q < 0 ? 0 : q < TW_QA ? 3 : q < TW_Q0 ? 1 : q < TW_QF ? ((q - TW_Q0) % TW_HS < 24 ? 1 : 3) : q < TW_QEND ? 3 : 0;
}
__host__ __device__ constexpr int tw_f0(int q) {     // first fragment of step q
  if (q <= TW_QA) return 3 * q;
  if (q <= TW_Q0) return 72 + (q - TW_QA);
  if (q <= TW_QF) {
    const int k = (q - TW_Q0) / TW_HS, r = (q - TW_Q0) % TW_HS;
    return 96 + 48 * k + (r <= 24 ? r : 24 + 3 * (r - 24));
  }
  return q <= TW_QEND ? 624 + 3 * (q - TW_QF) : 648;
}
__host__ __device__ constexpr int tw_step_of(int m) {  // the step that consumes fragment m
  if (m < 72) return m / 3;
  if (m < 96) return TW_QA + (m - 72);
  if (m < 624) {
    const int k = (m - 96) / 48, r = (m - 96) % 48;
    return TW_Q0 + TW_HS * k + (r < 24 ? r : 24 + (r - 24) / 3);
  }
  return TW_QF + (m - 624) / 3;
}
constexpr int TW_NFRAGW = 648;                       // fragments per wave
// the b1 loads (after the step's W loads): half-round 0's at its FFN1 step 16, half-round h's
// (h >= 1) at the first FFN2 step of its iteration
__host__ __device__ constexpr int tw_extra(int q) {
  return (q == TW_QA + 16 || (q >= TW_Q0 && q < TW_QF && (q - TW_Q0) % TW_HS == 24)) ? TW_NB1 : 0;
}
// the step during which fragment n is issued (-1: the prologue); step q issues [f0(q) + AH, + nf(q))
__host__ __device__ constexpr int tw_issuer(int n) { return n < TW_AH ? -1 : tw_step_of(n - TW_AH); }
__host__ __device__ constexpr int tw_min(int a, int b) { return a < b ? a : b; }
// vector-memory ops issued after step q's last fragment up to the wait before step q's MFMAs
__host__ __device__ constexpr int tw_younger(int q) {
  const int nl = tw_f0(q) + tw_nf(q) - 1;
  int n = tw_min(tw_f0(q) + TW_AH, TW_NFRAGW) - 1 - nl;
  const int qi = tw_issuer(nl);
  for (int j = qi < 0 ? 0 : qi; j < q; ++j) n += tw_extra(j);
  return n;
}
// ops issued during steps qa+1 .. qb
__host__ __device__ constexpr int tw_ops_between(int qa, int qb) {
  int n = 0;
  for (int q = qa + 1; q <= qb; ++q) n += (tw_f0(q) + TW_AH < TW_NFRAGW ? tw_nf(q) : 0) + tw_extra(q);
  return n;
}
// b1 of half-round h - 1 waited for at FFN1 step 2 of half-round h (h = 1: loaded at step 40; h >= 2:
// at the previous iteration's first FFN2 step): the smaller count is safe for every h
constexpr int TW_B1_WAIT = tw_min(tw_ops_between(TW_QA + 16, TW_Q0 + 2), tw_ops_between(TW_Q0 + 24, TW_QREP + 2));
// b1 of half-round 11 (loaded at step 392), waited for after step 399
constexpr int TW_B1_WAIT_END = tw_ops_between(TW_Q0 + 10 * TW_HS + 24, TW_QF - 1);
// the loop body serves half-rounds 1 .. 11: its wait at step i of an iteration is the smallest
// count over them (h = 1 sees half-round 0's b1 loads in its first windows) — a smaller count only
// waits for more
__host__ __device__ constexpr int tw_younger_it(int i) {
  int m = 63;
  for (int h = 1; h <= 11; ++h) m = tw_min(m, tw_younger(TW_Q0 + (h - 1) * TW_HS + i));
  return m;
}
// step q's wait: in the loop (the representative half-round's steps) the iteration minimum
__host__ __device__ constexpr int tw_wait_of(int q) {
  return (q >= TW_QREP && q < TW_QREP + TW_HS) ? tw_younger_it(q - TW_QREP) : tw_younger(q);
}
__host__ __device__ constexpr bool tw_ring_periodic() {
  return tw_f0(TW_QEND) == TW_NFRAGW && tw_f0(TW_QA) % TW_RING == 0 && tw_f0(TW_Q0) % TW_RING == 0 &&
         tw_f0(TW_QREP) % TW_RING == 0 && (tw_f0(TW_QREP + TW_HS) - tw_f0(TW_QREP)) % TW_RING == 0 &&
         tw_f0(TW_QF) % TW_RING == 0;
}
static_assert(tw_ring_periodic(), "fragment ring registers periodic over the sections");
static_assert(TW_B1_WAIT_END <= 63 && tw_younger(0) <= 63, "vmcnt range");

template <typename Body, int... Is>
__device__ __forceinline__ void tw_unroll(Body&& body, std::integer_sequence<int, Is...>) {
  (body(std::integral_constant<int, Is>{}), ...);
}
// NOP: s_nop 1 ahead of the MFMA — hipcc pads nothing inside an asm string, and outside the FFN
// loop (phase A, half-round 0, the last half-rounds) it stashes W fragments in AGPRs and reads one
// back right before its MFMA (a VALU write of an operand: 2 wait states); the loop body has no such
// write (tests/test_asm_hazards.py scans for it)
// TW_NOPMASK: which MFMA segments outside the FFN loop carry the s_nop (bit 0 phase A, bit 1 FFN1(0),
// bit 2 the last FFN1 / FFN2 of the loop's tail, bit 3 FFN2(11)); the 32-row (G = 1) body always.
// r6: only FFN1(0) gets a VALU write of an MFMA operand within 2 wait states without it (a scan of
// each segment with its s_nop removed: tests/test_asm_hazards.py keeps checking the build)
#ifndef TW_NOPMASK
#define TW_NOPMASK 2
#endif
template <bool AGPR, bool NOP = true>
__device__ __forceinline__ void tw_mfma(f32x16& c, const u32x4& a, const u32x4& b) {
  if constexpr (AGPR && NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else if constexpr (AGPR)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
// zero C operand: the accumulator's first k-step
template <bool AGPR, bool NOP = true>
__device__ __forceinline__ void tw_mfma0(f32x16& c, const u32x4& a, const u32x4& b) {
  if constexpr (AGPR && NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  else if constexpr (AGPR)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  else if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
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
template <bool AGPR> __device__ __forceinline__ void tw_drain_h4(f32x16 (&h)[4]) {
  if constexpr (AGPR)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(h[0]), "+a"(h[1]), "+a"(h[2]), "+a"(h[3]) :: "memory");
  else
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]) :: "memory");
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
typedef float tw_f2 __attribute__((ext_vector_type(2)));
// the two bf16 of a packed word as floats (low half first)
__device__ __forceinline__ tw_f2 tw_bf2(uint32_t w) { return tw_f2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; }
__device__ __forceinline__ tw_f2 tw_lrelu2(tw_f2 x) {
  const tw_f2 m = x * 0.1f;                           // one v_pk_mul_f32
  float a, b;
  asm("v_max_f32 %0, %1, %2" : "=v"(a) : "v"(x.x), "v"(m.x));
  asm("v_max_f32 %0, %1, %2" : "=v"(b) : "v"(x.y), "v"(m.y));
  return tw_f2{a, b};
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
// the same by plain LDS reads (LN phases: no LDS-DMA is in flight there, so the compiler's waits
// count only these reads and it may issue the next tile's reads under this tile's math)
__device__ __forceinline__ void tw_ld16p(const char* p, float (&v)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(p + 16 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * i + j] = q[j];
  }
}
// wait until at most Y younger vector-memory ops are in flight; the fragments' uses are ordered after it
#ifndef TW_ASM_WAITS
#define TW_ASM_WAITS 0                                 // 1: hand-counted waits on asm loads (diagnostics)
#endif
template <int Y> __device__ __forceinline__ void tw_wait1(u32x4& a) {
  static_assert(Y >= 0 && Y <= 63, "vmcnt range");
  if constexpr (TW_ASM_WAITS) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(a) : "n"(Y) : "memory");
}
template <int Y> __device__ __forceinline__ void tw_wait3(u32x4& a, u32x4& b, u32x4& c) {
  static_assert(Y >= 0 && Y <= 63, "vmcnt range");
  if constexpr (TW_ASM_WAITS) asm volatile("s_waitcnt vmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(Y) : "memory");
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
  int n_full;                   // workgroups of 128 rows (the rest: 32 rows)
};

// G token groups of 32 rows (G = 4: a 128-row tile; G = 1: the 32-row tiles that spread the last
// partial round of 128-row tiles over more CUs, tailw_kernel below).  GI: the group after whose
// MFMAs a step issues its W loads
template <int VAR, int G>
__device__ __forceinline__ void tailw_body(const TwArgs& p, const long row0) {
  constexpr int D = TW_D, NT = TW_NT, GI = G > 1 ? 1 : 0;
  // VAR bit 3: the FFN epilogue in FFN2's MFMA gaps instead of FFN1's (A/B)
  constexpr bool EPI_FFN2 = (VAR & 8) != 0;
  // the residual rows loaded during phase A (after step TW_RES_STEP's W loads: the prologue's HBM
  // burst halves, -2 k cycles per wave net, r6 tools/tailw_diag.py); VAR bit 4: in the prologue (A/B)
  constexpr bool LATE_RES = (VAR & 16) == 0;
  constexpr int TW_RES_STEP = 21;
  // s_nop ahead of the inline-asm MFMAs of a segment (TW_NOPMASK bit b, or the 32-row body)
  constexpr bool NOPA = G == 1 || (TW_NOPMASK & 1), NOP0 = G == 1 || (TW_NOPMASK & 2);
  constexpr bool NOPT = G == 1 || (TW_NOPMASK & 4), NOPF = G == 1 || (TW_NOPMASK & 8);
  using TNA = std::integral_constant<bool, NOP0>;
  using TNT = std::integral_constant<bool, NOPT>;
  using TNF = std::integral_constant<bool, NOPF>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned long long st[8] = {};
  auto stamp = [&](int i) {
    if constexpr (VAR & 1) st[i] = __builtin_amdgcn_s_memtime();
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
    if (wave < G) {
#pragma unroll
      for (int s = 0; s < TW_KS; ++s)
        dma_x4(ars, lds0 + TW_X + (s * 4 + wave) * TW_FRAG, voff, 64 * (s >> 1) + 16 * (s & 1));
    }
  }
  u32x4 wf[TW_RING];                                 // W fragment ring
  // W fragment F of the stream into register r (soffset: scalar)
  // (compiler-visible loads: its waitcnt pass places the waits before every read of the register —
  // hand-counted asm loads were seen copied into AGPRs by the register allocator before they landed)
  const __amdgpu_buffer_rsrc_t wrb = __builtin_amdgcn_make_buffer_rsrc((void*)p.ws, (short)0, TW_NFRAG * TW_FRAG, 0x00020000);
  // (diagnostic VAR bit 1: every load reads fragment F % 12 — a cache-resident 12 KiB, results wrong)
  auto loadW = [&](u32x4& r, int F) {
    r = __builtin_amdgcn_raw_buffer_load_b128(wrb, lane16, ((VAR & 2) ? F % 12 : F) * TW_FRAG, 0);
  };
  // stream offsets: FFN1(h) step i = wave w's tile of chunk 4 (h >> 1) + w, half h & 1;
  // FFN2(h) step u, tile t = chunk 4 (h >> 1) + u / 2, k16 step 2 (h & 1) + u % 2, tile 3w + t
  auto f_ffn1 = [&](int h, int i) { return TW_FPRE + (4 * (h >> 1) + wave) * TW_FPC + 2 * i + (h & 1); };
  auto f_ffn2 = [&](int h, int u, int t) {
    return TW_FPRE + (4 * (h >> 1) + (u >> 1)) * TW_FPC + 48 + (2 * (h & 1) + (u & 1)) * NT + 3 * wave + t;
  };
  // fragment n of the prologue / phase A / half-round 0 (n < 120: W_o' k16 step n / 3 tile n % 3,
  // FFN1(0), FFN1(1))
  auto issue_a = [&](auto n_tag) {
    constexpr int n = decltype(n_tag)::value;
    if constexpr (n < 72) loadW(wf[n % TW_RING], (n / 3) * NT + 3 * wave + n % 3);
    else if constexpr (n < 96) loadW(wf[n % TW_RING], f_ffn1(0, n - 72));
    else loadW(wf[n % TW_RING], f_ffn1(1, n - 96));
  };
  tw_unroll([&](auto nc) { issue_a(nc); }, std::make_integer_sequence<int, TW_AH>{});
  u32x4 rr[3][4][2];                                 // residual x: tile t, group g, half h2
  // (LATE_RES: issued after phase A step TW_RES_STEP's W loads instead of here — the prologue's HBM
  // burst halves; the W waits after it then also wait for these rows, in-order vmcnt)
  auto load_res = [&]() {
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      long r = row0 + 32 * g + (l & 31);
      r = r < p.M ? r : (long)p.M - 1;
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          rr[t][g][h2] = *reinterpret_cast<const u32x4*>(p.resid + r * D + 32 * (3 * wave + t) + 16 * (l >> 5) + 8 * h2);
    }
  };
  if constexpr (!LATE_RES) load_res();
  float* tab = reinterpret_cast<float*>(smem + TW_H);                        // [b_o | g1 | be1]
  for (int i = threadIdx.x; i < D; i += 256) {
    tab[i] = p.b_o[i];
    tab[D + i] = p.g1[i];
    tab[2 * D + i] = p.be1[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the residual rows retired here (else the compiler's wait for them lands at LN1, behind the
  // in-flight W loads of the first FFN steps)
  if constexpr (!LATE_RES) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int g = 0; g < G; ++g) asm volatile("" : "+v"(rr[t][g][0]), "+v"(rr[t][g][1]));
  }
  tw_barrier();
  stamp(1);

  // ---- phase A: ao = att W_o'^T (wave w: tiles 3w .. 3w+2 x 4 token groups, AGPRs)
  f32x16 acc[3][4];
  u32x4 bq[3][4];                                     // B fragments, read two k16 steps ahead
  auto rdB = [&](uint32_t base, int blk) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(smem + base + blk * TW_FRAG + lane16);
  };
  // (B fragments one step ahead in two buffers here: 12 MFMAs per step cover the LDS latency, and
  // a third buffer beside the residual rows pushed the W fragments into AGPR copies taken before
  // their loads had landed)
#pragma unroll
  for (int g = 0; g < G; ++g) bq[0][g] = rdB(TW_X, g);
  tw_unroll([&](auto qc) {
    constexpr int q = decltype(qc)::value, n0 = 3 * q;
    tw_wait3<tw_younger(q)>(wf[n0 % TW_RING], wf[(n0 + 1) % TW_RING], wf[(n0 + 2) % TW_RING]);
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        if constexpr (q == 0) tw_mfma0<true, NOPA>(acc[t][g], wf[(n0 + t) % TW_RING], bq[q & 1][g]);
        else tw_mfma<true, NOPA>(acc[t][g], wf[(n0 + t) % TW_RING], bq[q & 1][g]);
      }
      if constexpr (q + 1 < TW_KS) bq[(q + 1) & 1][g] = rdB(TW_X, (q + 1) * 4 + g);
      if (g == GI)
        tw_unroll([&](auto tc) { issue_a(std::integral_constant<int, n0 + TW_AH + decltype(tc)::value>{}); },
                  std::make_integer_sequence<int, 3>{});
    }
    if constexpr (LATE_RES && q == TW_RES_STEP) load_res();
    __builtin_amdgcn_sched_barrier(0);
  }, std::make_integer_sequence<int, TW_QA>{});
  tw_drain_o(acc);
  stamp(2);

  // ---- LN1 over the 4 waves' features: v = ao + b_o + x; per-wave (sum, sumsq) -> LDS
  float2* s1 = reinterpret_cast<float2*>(smem + TW_H + 8 * 1024);          // [wave][128 rows]
  {
    const uint32_t tb = lds0 + TW_H + 64 * (tw_lane() >> 5);
#if TW_PACKED_LN
    // (packed f32 math: pairs of features per v_pk_* instruction)
    tw_f2 s2v[4], q2v[4];
#pragma unroll
    for (int g = 0; g < G; ++g) s2v[g] = q2v[g] = tw_f2{0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float bo[16];
      tw_ld16p(smem + (tb - lds0) + 4 * 32 * (3 * wave + t), bo);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const tw_f2 v = tw_f2{acc[t][g][2 * e], acc[t][g][2 * e + 1]} + tw_f2{bo[2 * e], bo[2 * e + 1]} +
                          tw_bf2(rr[t][g][e >> 2][e & 3]);
          acc[t][g][2 * e] = v.x;
          acc[t][g][2 * e + 1] = v.y;
          s2v[g] += v;
          q2v[g] = v * v + q2v[g];
        }
    }
    float sum[4], sq[4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      sum[g] = s2v[g].x + s2v[g].y;
      sq[g] = q2v[g].x + q2v[g].y;
    }
#else
    float sum[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float bo[16];
      tw_ld16p(smem + (tb - lds0) + 4 * 32 * (3 * wave + t), bo);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = acc[t][g][i] + bo[i] + tw_bf(rr[t][g][i >> 3], i & 7);
          acc[t][g][i] = v;
          sum[g] += v;
          sq[g] = fmaf(v, v, sq[g]);
        }
    }
#endif
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int g = 0; g < G; ++g) {}   // v back in AGPRs
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < G; ++g) {
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
    for (int g = 0; g < G; ++g) {
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
      tw_ld16p(smem + (tb - lds0) + 4 * (D + 32 * (3 * wave + t)), gg);
      tw_ld16p(smem + (tb - lds0) + 4 * (2 * D + 32 * (3 * wave + t)), bb);
      const int T = 3 * wave + t;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float y[16];
#if TW_PACKED_LN
        const float nmr = -mean[g] * rstd[g];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const tw_f2 z = (tw_f2{acc[t][g][2 * e], acc[t][g][2 * e + 1]} * rstd[g] + nmr) * tw_f2{gg[2 * e], gg[2 * e + 1]} +
                          tw_f2{bb[2 * e], bb[2 * e + 1]};
          y[2 * e] = z.x;
          y[2 * e + 1] = z.y;
        }
#else
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = (acc[t][g][i] - mean[g]) * rstd[g] * gg[i] + bb[i];
#endif
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

  // ---- FFN in 12 half-rounds.  Half-round h: wave w's FFN1 tile (32 hidden units: chunk
  // 4 (h >> 1) + w, half h & 1) over all 128 rows into hv / ha (even / odd h: VGPRs / AGPRs), while
  // the chunk epilogue of half-round h - 1 (b1, LeakyReLU, LN_f sums, bf16) is interleaved between
  // its MFMAs and writes that hidden into H half (h - 1) & 1; one barrier; then FFN2 of half-round
  // h - 1 (the 4 waves' tiles = 8 k16 steps) from that H half.  H is double-buffered, so the next
  // half-round's epilogue writes the other half while this FFN2 reads.
  // B fragments: FFN2 step u uses bq[u % 3], FFN1 step i bq[(i + 2) % 3] (so that FFN2's
  // last two steps prefetch the next FFN1's first two), each read two steps ahead.
  f32x16 hv[4], ha[4];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g) acc[t][g] = f32x16{};
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g) asm volatile("" : "+a"(acc[t][g]));
  typedef float f2 __attribute__((ext_vector_type(2)));
  float sa1[4], sa2[4];                               // LN_f partial sums of this lane's hidden units
#pragma unroll
  for (int g = 0; g < G; ++g) sa1[g] = sa2[g] = 0.f;
  u32x4 b1v[4];                                       // b1 of the tile whose epilogue runs next
  const __amdgpu_buffer_rsrc_t b1b = __builtin_amdgcn_make_buffer_rsrc((void*)p.vec, (short)0, 4 * D * 4, 0x00020000);
  auto b1_load = [&](int h) {                         // b1[64 c' + 32 (h & 1) + 8 r + 4 hh .. + 3]
    const int so = 4 * (64 * (4 * (h >> 1) + wave) + 32 * (h & 1));
    const int vo = 16 * (tw_lane() >> 5);
#pragma unroll
    for (int r = 0; r < 4; ++r) b1v[r] = __builtin_amdgcn_raw_buffer_load_b128(b1b, vo + 32 * r, so, 0);
  };
  // epilogue unit k (0 .. 7: group k / 2, k16 step j = k % 2 of the tile) of the half-round with
  // parity Q: 8 hidden units of this lane's token -> its 16-B slot of an FFN2 B fragment in H half Q.
  // A unit runs as TW_EP pieces spread over the MFMA gaps of three FFN1 steps (piece p after MFMA
  // g of step 3k + p / G): values v at piece v (TW_EP - 2) / 8 (b1, LeakyReLU, the LN_f sums: five
  // scalar VALU each), the four bf16 packs at piece TW_EP - 2, the LDS write at TW_EP - 1 — at most
  // ~5 VALU per 32x32x16 gap, which the MFMA hides; one ~40-instruction block per unit (packed f32)
  // stalled the matrix pipe for ~130 cycles after every third step.
  constexpr int TW_EP = 3 * G;
  float ex[8];                                        // the unit's values between its pieces
  uint32_t epk[4];
  auto epi_piece = [&](auto k_tag, auto q_tag, auto p_tag) {
    constexpr int k = decltype(k_tag)::value, Q = decltype(q_tag)::value, pc = decltype(p_tag)::value;
    constexpr int g = k >> 1, j = k & 1;
    if constexpr (g < G) {
      const f32x16& a = Q ? ha[g] : hv[g];
      tw_unroll([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        if constexpr (v * (TW_EP - 2) / 8 == pc) {
          // (LeakyReLU as plain code: the inline-asm form made hipcc pad an s_nop after every one)
          const float u = a[8 * j + v] + __uint_as_float(b1v[(8 * j + v) >> 2][(8 * j + v) & 3]);
          const float x = fmaxf(u, 0.1f * u);
          ex[v] = x;
          sa1[g] += x;
          sa2[g] = fmaf(x, x, sa2[g]);
        }
      }, std::make_integer_sequence<int, 8>{});
      if constexpr (pc == TW_EP - 2) {
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) epk[e2] = tw_pack2(ex[2 * e2], ex[2 * e2 + 1]);
      }
      if constexpr (pc == TW_EP - 1)
        *reinterpret_cast<u32x4*>(smem + TW_H + Q * 32768 + ((wave * 2 + j) * 4 + g) * TW_FRAG + lane16) =
            u32x4{epk[0], epk[1], epk[2], epk[3]};
    }
  };
  // fragment r of an iteration (r relative to its first fragment; h = the iteration's half-round):
  // [0, 24) FFN1(h), [24, 48) FFN2(h - 1), then the next iteration's FFN1(h + 1) (LAST: FFN2(11))
  auto issue_it = [&](auto r_tag, int h, auto last_tag) {
    constexpr int r = decltype(r_tag)::value, n = r;  // iteration starts are multiples of the ring
    if constexpr (r < 24) loadW(wf[n % TW_RING], f_ffn1(h, r));
    else if constexpr (r < 48) loadW(wf[n % TW_RING], f_ffn2(h - 1, (r - 24) / 3, (r - 24) % 3));
    else if constexpr (decltype(last_tag)::value) loadW(wf[n % TW_RING], f_ffn2(h, (r - 48) / 3, (r - 48) % 3));
    else loadW(wf[n % TW_RING], f_ffn1(h + 1, r - 48));
  };
  // FFN1(h), parity P; Q0 = its first global step (the representative half-round for h >= 1);
  // EPI: with the epilogue of half-round h - 1 (unit k over steps 3k .. 3k + 2, one piece per MFMA gap)
  auto seg1 = [&](int h, auto p_tag, auto q0_tag, auto epi_tag, auto nop_tag, auto b1_tag) {
    constexpr int P = decltype(p_tag)::value, Q0 = decltype(q0_tag)::value;
    constexpr bool EPI = decltype(epi_tag)::value, NOP = decltype(nop_tag)::value, B1 = decltype(b1_tag)::value;
    constexpr int F0 = tw_f0(Q0);
    tw_unroll([&](auto ic) {
      constexpr int i = decltype(ic)::value, q = Q0 + i, n = F0 + i;
      tw_wait1<tw_wait_of(q)>(wf[n % TW_RING]);
      tw_unroll([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        if constexpr (P == 0) {
          if constexpr (i == 0) tw_mfma0<false, NOP>(hv[g], wf[n % TW_RING], bq[(i + 2) % 3][g]);
          else tw_mfma<false, NOP>(hv[g], wf[n % TW_RING], bq[(i + 2) % 3][g]);
        } else {
          if constexpr (i == 0) tw_mfma0<true, NOP>(ha[g], wf[n % TW_RING], bq[(i + 2) % 3][g]);
          else tw_mfma<true, NOP>(ha[g], wf[n % TW_RING], bq[(i + 2) % 3][g]);
        }
        // (diagnostic VAR bit 2: FFN1 reads no B fragments — stale operands, no LDS traffic)
        if constexpr (i + 2 < 24 && !(VAR & 4)) bq[(i + 4) % 3][g] = rdB(TW_X, (i + 2) * 4 + g);
        if constexpr (g == GI) {
          if constexpr (Q0 == TW_QA) issue_a(std::integral_constant<int, n + TW_AH>{});
          else issue_it(std::integral_constant<int, i + TW_AH>{}, h, std::false_type{});
        }
        if constexpr (EPI) {                          // piece (i % 3) G + g of unit i / 3, in this gap
          epi_piece(std::integral_constant<int, i / 3>{}, std::integral_constant<int, 1 - P>{},
                    std::integral_constant<int, (i % 3) * G + g>{});
          __builtin_amdgcn_sched_barrier(0);
        }
      }, std::make_integer_sequence<int, G>{});
      if constexpr (Q0 == TW_QA && i == 16) b1_load(0);
      if constexpr (B1 && i == 8) b1_load(h);        // for this half-round's epilogue in the next FFN2
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, 24>{});
    if constexpr (P == 0) tw_drain_h4<false>(hv);
    else tw_drain_h4<true>(ha);
  };
  // FFN2(h) from H half h & 1 (P = h & 1); in the loop (Q0 = representative) its iteration is h + 1;
  // LAST: the iteration of h = 10, whose lookahead loads FFN2(11); FINAL: FFN2(11) itself
  // EPI: with the epilogue of half-round h + 1 (whose FFN1 ran just before; parity 1 - P), one piece
  // after each of the 24 G MFMAs (unit k over gaps 3 G k .. 3 G k + 3 G - 1)
  // (FFN1-gap schedule: b1 of half-round h + 1 loaded at step 0, for its epilogue in FFN1(h + 2))
  auto seg2 = [&](int h, auto p_tag, auto q0_tag, auto last_tag, auto final_tag, auto nop_tag, auto epi_tag) {
    constexpr int P = decltype(p_tag)::value, Q0 = decltype(q0_tag)::value;
    constexpr bool LAST = decltype(last_tag)::value, FINAL = decltype(final_tag)::value;
    constexpr bool NOP = decltype(nop_tag)::value, EPI = decltype(epi_tag)::value;
    constexpr bool B1N = !EPI && !FINAL && !EPI_FFN2;
    constexpr uint32_t HB = TW_H + P * 32768;
    constexpr int F0 = tw_f0(Q0);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      bq[0][g] = rdB(HB, g);
      bq[1][g] = rdB(HB, 4 + g);
    }
    tw_unroll([&](auto uc) {
      constexpr int u = decltype(uc)::value, q = Q0 + u, n0 = F0 + 3 * u;
      tw_wait3<tw_wait_of(q)>(wf[n0 % TW_RING], wf[(n0 + 1) % TW_RING], wf[(n0 + 2) % TW_RING]);
      tw_unroll([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        tw_unroll([&](auto tc) {
          constexpr int t = decltype(tc)::value, x = 3 * G * u + 3 * g + t;
          tw_mfma<true, NOP>(acc[t][g], wf[(n0 + t) % TW_RING], bq[u % 3][g]);
          if constexpr (EPI) {
            epi_piece(std::integral_constant<int, x / (3 * G)>{}, std::integral_constant<int, 1 - P>{},
                      std::integral_constant<int, x % (3 * G)>{});
            __builtin_amdgcn_sched_barrier(0);
          }
        }, std::make_integer_sequence<int, 3>{});
        if constexpr (u + 2 < 8) bq[(u + 2) % 3][g] = rdB(HB, (u + 2) * 4 + g);
        else if constexpr (!FINAL && !LAST) bq[(u + 2) % 3][g] = rdB(TW_X, (u - 6) * 4 + g);   // next FFN1 steps 0, 1
        if constexpr (g == GI) {
          if constexpr (FINAL) {
            if constexpr (n0 + TW_AH < TW_NFRAGW)
              tw_unroll([&](auto tc) {
                constexpr int m = n0 + TW_AH + decltype(tc)::value;
                if constexpr (m < TW_NFRAGW) loadW(wf[m % TW_RING], f_ffn2(h, (m - F0) / 3, (m - F0) % 3));
              }, std::make_integer_sequence<int, 3>{});
          } else {
            tw_unroll([&](auto tc) {
              issue_it(std::integral_constant<int, 24 + 3 * u + TW_AH + decltype(tc)::value>{}, h + 1, last_tag);
            }, std::make_integer_sequence<int, 3>{});
          }
        }
      }, std::make_integer_sequence<int, G>{});
      if constexpr (B1N && u == 0) b1_load(h + 1);
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, 8>{});
    tw_drain_o(acc);
  };
#pragma unroll
  for (int g = 0; g < G; ++g) {
    bq[2][g] = rdB(TW_X, g);
    bq[0][g] = rdB(TW_X, 4 + g);
  }
  seg1(0, std::integral_constant<int, 0>{}, std::integral_constant<int, TW_QA>{}, std::false_type{}, TNA{},
       std::false_type{});
#pragma unroll
  for (int g = 0; g < G; ++g) {
    bq[2][g] = rdB(TW_X, g);
    bq[0][g] = rdB(TW_X, 4 + g);
  }
  using T0 = std::false_type;
  using T1 = std::true_type;
  using IQR = std::integral_constant<int, TW_QREP>;
  using IQ2 = std::integral_constant<int, TW_QREP + 24>;
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  // a barrier of the FFN (stamped variants: cycles parked in the FFN's barriers into stamp slot 6)
  auto ffn_barrier = [&]() {
    if constexpr (VAR & 1) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      tw_barrier();
      st[6] += __builtin_amdgcn_s_memtime() - t0;
    } else {
      tw_barrier();
    }
  };
  if constexpr (!EPI_FFN2) {
    // FFN1(h) with the epilogue of half-round h - 1 in its MFMA gaps (b1(h - 1) loaded at FFN2(h - 2)
    // step 0), barrier, FFN2(h - 1)
#pragma unroll 1
    for (int h = 1; h < 11; h += 2) {
      seg1(h, P1{}, IQR{}, T1{}, T0{}, T0{});
      ffn_barrier();                                  // H half (h - 1) & 1 complete
      seg2(h - 1, P0{}, IQ2{}, T0{}, T0{}, T0{}, T0{});
      seg1(h + 1, P0{}, IQR{}, T1{}, T0{}, T0{});
      ffn_barrier();
      seg2(h, P1{}, IQ2{}, T0{}, T0{}, T0{}, T0{});
    }
    seg1(11, P1{}, IQR{}, T1{}, TNT{}, T0{});
    ffn_barrier();
    seg2(10, P0{}, IQ2{}, T1{}, T0{}, TNT{}, T0{});
    // the epilogue of half-round 11, then its FFN2
    tw_unroll([&](auto kc) {                          // (unit by unit: a unit's pieces share ex / epk)
      tw_unroll([&](auto pc) { epi_piece(kc, P1{}, pc); }, std::make_integer_sequence<int, TW_EP>{});
    }, std::make_integer_sequence<int, 8>{});
    ffn_barrier();
  } else {
    // FFN1(1) with the epilogue of half-round 0 in its MFMA gaps (no FFN2 to carry it yet); then b1
    // of half-round 1 (after the epilogue's last read of b1v)
    seg1(1, P1{}, std::integral_constant<int, TW_Q0>{}, T1{}, TNT{}, T0{});
    b1_load(1);
    ffn_barrier();                                    // H half 0 complete
    // FFN2(h - 1) with the epilogue of half-round h in its MFMA gaps, FFN1(h + 1) (pure MFMA +
    // B-fragment reads), one barrier (H half h & 1 complete): the same W consumption order
#pragma unroll 1
    for (int h = 1; h < 11; h += 2) {
      seg2(h - 1, P0{}, IQ2{}, T0{}, T0{}, T0{}, T1{});
      seg1(h + 1, P0{}, IQR{}, T0{}, T0{}, T1{});
      ffn_barrier();
      seg2(h, P1{}, IQ2{}, T0{}, T0{}, T0{}, T1{});
      seg1(h + 2, P1{}, IQR{}, T0{}, T0{}, T1{});
      ffn_barrier();
    }
    // FFN2(10) with the epilogue of half-round 11, then FFN2(11)
    seg2(10, P0{}, IQ2{}, T1{}, T0{}, TNT{}, T1{});
    ffn_barrier();
  }
  // H half 0 is free from here (its last reader, FFN2(10), is behind this barrier): the LN epilogue's
  // tables [b2' | c1 | g2 | be2] (6 KiB) arrive there by LDS-DMA during FFN2(11) (retired by the
  // vmcnt(0) after it, visible after the epilogue's first barrier)
  {
    const i32x4 vrs = dma_rsrc(p.vec + 4 * D, 4L * D * 4);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = wave + 4 * j;
      if (pc < 6) dma_x4(vrs, lds0 + TW_H + pc * TW_FRAG, lane16, pc * TW_FRAG);
    }
  }
  seg2(11, std::integral_constant<int, 1>{}, std::integral_constant<int, TW_QF>{}, std::false_type{},
       std::true_type{}, TNF{}, std::false_type{});
  float st1[4], st2[4];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    st1[g] = sa1[g];
    st2[g] = sa2[g];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the overrun loads have landed
  stamp(4);

  // ---- epilogue: out = LN2(x1 + lrelu(rstd_f (acc - mean_f c1) + b2'))
  float2* s2 = reinterpret_cast<float2*>(smem + TW_H + 8 * 1024);
  float2* s3 = reinterpret_cast<float2*>(smem + TW_H + 12 * 1024);
  // (H half 0 holds the tables, DMA'd during FFN2(11), and the statistics; FFN2(11) reads half 1)
  {
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      st1[g] = tw_xsum32(st1[g]);
      st2[g] = tw_xsum32(st2[g]);
      s2[wave * 128 + 32 * g + (l & 31)] = make_float2(st1[g], st2[g]);
    }
  }
  tw_barrier();
  float hm[4], hr[4];
  {
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < G; ++g) {
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
#if TW_PACKED_LN
    // u = hr (acc - hm c1) + b2' = acc hr + (b2' - hm hr c1), in pairs (v_pk_fma_f32)
    tw_f2 s2v[4], q2v[4];
#pragma unroll
    for (int g = 0; g < G; ++g) s2v[g] = q2v[g] = tw_f2{0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int T = 3 * wave + t;
      float b2[16], c1[16];
      tw_ld16p(smem + (eb - lds0) + 4 * (32 * T), b2);
      tw_ld16p(smem + (eb - lds0) + 4 * (D + 32 * T), c1);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const u32x4 xa = rdB(TW_X, (2 * T) * 4 + g), xb = rdB(TW_X, (2 * T + 1) * 4 + g);
        const float nhh = -hm[g] * hr[g];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const tw_f2 k = tw_f2{c1[2 * e], c1[2 * e + 1]} * nhh + tw_f2{b2[2 * e], b2[2 * e + 1]};
          const tw_f2 u = tw_lrelu2(tw_f2{acc[t][g][2 * e], acc[t][g][2 * e + 1]} * hr[g] + k);
          const tw_f2 v = u + tw_bf2((e < 4 ? xa : xb)[e & 3]);
          acc[t][g][2 * e] = v.x;
          acc[t][g][2 * e + 1] = v.y;
          s2v[g] += v;
          q2v[g] = v * v + q2v[g];
        }
      }
    }
    float sum[4], sq[4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      sum[g] = s2v[g].x + s2v[g].y;
      sq[g] = q2v[g].x + q2v[g].y;
    }
#else
    float sum[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int T = 3 * wave + t;
      float b2[16], c1[16];
      tw_ld16p(smem + (eb - lds0) + 4 * (32 * T), b2);
      tw_ld16p(smem + (eb - lds0) + 4 * (D + 32 * T), c1);
#pragma unroll
      for (int g = 0; g < G; ++g) {
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
#endif
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int g = 0; g < G; ++g) {}
    const int l = tw_lane();
#pragma unroll
    for (int g = 0; g < G; ++g) {
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
    for (int g = 0; g < G; ++g) {
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
      tw_ld16p(smem + (eb - lds0) + 4 * (2 * D + 32 * T), g2);
      tw_ld16p(smem + (eb - lds0) + 4 * (3 * D + 32 * T), be2);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const long r = row0 + 32 * g + (l & 31);
        const float nmr = -mean[g] * rstd[g];
        float y[16];
#pragma unroll
#if TW_PACKED_LN
        for (int e = 0; e < 8; ++e) {
          const tw_f2 z = (tw_f2{acc[t][g][2 * e], acc[t][g][2 * e + 1]} * rstd[g] + nmr) * tw_f2{g2[2 * e], g2[2 * e + 1]} +
                          tw_f2{be2[2 * e], be2[2 * e + 1]};
          y[2 * e] = z.x;
          y[2 * e + 1] = z.y;
        }
#else
        for (int i = 0; i < 16; ++i) y[i] = fmaf(fmaf(acc[t][g][i], rstd[g], nmr), g2[i], be2[i]);
#endif
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
  if constexpr (VAR & 1) {
    stamp(5);
    if ((threadIdx.x & 63) == 0 && p.stamps) {
#pragma unroll
      for (int i = 0; i < 7; ++i) p.stamps[((long)blockIdx.x * 4 + wave) * 8 + i] = st[i];
    }
  }
}

// workgroups [0, n_full): 128-row tiles; the rest: 32-row tiles after row 128 n_full (the launch's
// last partial round of 128-row tiles spread over 4x the CUs, dispatched last)
template <int VAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void tailw_kernel(TwArgs p) {
  if ((int)blockIdx.x < p.n_full) tailw_body<VAR, 4>(p, (long)blockIdx.x * 128);
  else tailw_body<VAR, 1>(p, (long)p.n_full * 128 + (long)(blockIdx.x - p.n_full) * 32);
}

int tailw_launch(int M, const void* att, const void* resid, void* out, const void* ws, const float* vec,
                 const float* b_o, const float* g1, const float* be1, float eps, int desync, int var,
                 hipStream_t s) {
  // the last partial round of 128-row tiles (rem of 256 CUs) as 4 rem workgroups of 32 rows, when
  // they fit one round of 32-row tiles (option tail_split = the largest rem split; 0: off)
  const long T = cdiv(M, 128), rem = T % 256;
  const long split = options().tail_split;
  const long n_full = (T > 256 && rem > 0 && rem <= split) ? T - rem : T;
  const long nwg = n_full < T ? n_full + cdiv((long)M - n_full * 128, 32) : T;
  TwArgs a{M, (const bf16*)att, (const bf16*)resid, (bf16*)out, (const char*)ws, vec, b_o, g1, be1, eps, desync,
           diag_stamps(), (int)n_full};
  // var (option tail_wide - 1): bit 0 phase stamps, bit 1 / bit 2 the W-latency / FFN1-LDS
  // diagnostics (wrong results: tools/tailw_diag.py timing only; r6: W-cached no faster, no-FFN1-LDS
  // 2 %), bit 3 the FFN epilogue in FFN2's gaps (A/B)
  if ((var & 1) && !a.stamps) var &= ~1;
  auto kern = var == 1 ? tailw_kernel<1> : var == 2 ? tailw_kernel<2> : var == 4 ? tailw_kernel<4>
              : var == 8 ? tailw_kernel<8> : var == 9 ? tailw_kernel<9> : var == 16 ? tailw_kernel<16>
              : var == 17 ? tailw_kernel<17> : tailw_kernel<0>;
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, TW_LDS));
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(256), TW_LDS, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}


// ---------------------------------------------------------------------------------------------
// Wide-row projection (option proj_wide; the encoder's QKV: out[M, NC D] = x W^T + b, D = 384,
// multi_head_attention.py:44-51): the tail's phase A per output chunk of D features.  A
// workgroup owns 128 rows (x by LDS-DMA into X once), wave w owns tiles 3w .. 3w+2 of each chunk;
// per chunk 24 k16 steps x 12 MFMAs into 192 AGPR accumulators, then + bias -> bf16 -> two 16-B
// stores per (tile, token group).  W fragments (snvrag_proj_pack: chunk c, k16 step s, tile T at
// fragment c 288 + 12 s + T) through the 12-register ring 9 ahead, compiler-visible loads.
struct PwArgs {
  int M, NC;
  const bf16* x;            // [M, D]
  const char* ws;           // snvrag_proj_pack stream
  const float* bias;        // [NC D]
  bf16* out;                // [M, NC D]
  int desync;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void projw_kernel(PwArgs p) {
  constexpr int D = TW_D, NT = TW_NT, KS = TW_KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long row0 = (long)blockIdx.x * 128;
  if (p.desync > 0 && blockIdx.x < 256) {
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }
  const uint32_t lds0 = lds_addr(smem);
  int lane16 = tw_lane() * 16;
  asm volatile("" : "+v"(lane16));
  const i32x4 xrs = dma_rsrc(p.x + row0 * D, ((long)p.M - row0) * D * 2);     // rows >= M read as 0
  {
    const int l = tw_lane();
    const int voff = (32 * wave + (l & 31)) * (D * 2) + 32 * (l >> 5);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      dma_x4(xrs, lds0 + TW_X + (s * 4 + wave) * TW_FRAG, voff, 64 * (s >> 1) + 16 * (s & 1));
  }
  const int nfr = p.NC * TW_FPRE;
  const __amdgpu_buffer_rsrc_t wrb = __builtin_amdgcn_make_buffer_rsrc((void*)p.ws, (short)0, nfr * TW_FRAG, 0x00020000);
  u32x4 wf[TW_RING];
  // fragment n of this wave's stream: chunk n / 72, k16 step (n % 72) / 3, tile 3w + n % 3 (past the
  // last chunk: the last chunk again, never consumed)
  auto loadW = [&](u32x4& r, int c, int n72) {
    const int cc = c < p.NC ? c : p.NC - 1;
    r = __builtin_amdgcn_raw_buffer_load_b128(wrb, lane16, (cc * TW_FPRE + (n72 / 3) * NT + 3 * wave + n72 % 3) * TW_FRAG, 0);
  };
#pragma unroll
  for (int n = 0; n < TW_AH; ++n) loadW(wf[n], 0, n);
  float* bs = reinterpret_cast<float*>(smem + TW_H);
  for (int i = threadIdx.x; i < p.NC * D; i += 256) bs[i] = p.bias[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the x image (LDS-DMA) landed
  tw_barrier();
  auto rdB = [&](int blk) -> u32x4 { return *reinterpret_cast<const u32x4*>(smem + TW_X + blk * TW_FRAG + lane16); };
  const long o_bytes = ((long)p.M - row0) * p.NC * D * 2;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.out + row0 * p.NC * D), (short)0, (int)(o_bytes < 0x7fffffffL ? o_bytes : 0x7fffffffL), 0x00020000);
  f32x16 acc[3][4];
  u32x4 bq[2][4];
#pragma unroll 1
  for (int c = 0; c < p.NC; ++c) {
#pragma unroll
    for (int g = 0; g < 4; ++g) bq[0][g] = rdB(g);
    tw_unroll([&](auto sc) {
      constexpr int s = decltype(sc)::value, n0 = 3 * s;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          if constexpr (s == 0) tw_mfma0<true, false>(acc[t][g], wf[(n0 + t) % TW_RING], bq[s & 1][g]);
          else tw_mfma<true, false>(acc[t][g], wf[(n0 + t) % TW_RING], bq[s & 1][g]);
        }
        if constexpr (s + 1 < KS) bq[(s + 1) & 1][g] = rdB((s + 1) * 4 + g);
        if (g == 1) {
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            constexpr int dummy = 0;
            const int m = n0 + TW_AH + t;              // within [0, 72 + 9): this chunk or the next
            if (m < 72) loadW(wf[(n0 + TW_AH + t) % TW_RING], c, m);
            else loadW(wf[(n0 + TW_AH + t) % TW_RING], c + 1, m - 72);
            (void)dummy;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, KS>{});
    tw_drain_o(acc);
    // + bias -> bf16 -> out[row][c D + 32 T + 16 hh .. + 15]
    const int l = tw_lane();
    const uint32_t bb = lds0 + TW_H + 4 * (c * D + 16 * (l >> 5));
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int T = 3 * wave + t;
      float bv[16];
      tw_ld16(bb + 4 * 32 * T, bv);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ro = ((32 * g + (l & 31)) * p.NC * D + c * D + 32 * T + 16 * (l >> 5)) * 2;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          float y[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] = acc[t][g][8 * h2 + j] + bv[8 * h2 + j];
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{tw_pack2(y[0], y[1]), tw_pack2(y[2], y[3]), tw_pack2(y[4], y[5]),
                                                       tw_pack2(y[6], y[7])},
                                                 ors, ro + 16 * h2, 0, 0);
        }
      }
    }
  }
}

int projw_launch(int M, int NC, const void* x, const void* ws, const float* bias, void* out, int desync, hipStream_t s) {
  PwArgs a{M, NC, (const bf16*)x, (const char*)ws, bias, (bf16*)out, desync};
  SNV_HIP(hipFuncSetAttribute((const void*)projw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, TW_LDS));
  hipLaunchKernelGGL(projw_kernel, dim3((unsigned)cdiv(M, 128)), dim3(256), TW_LDS, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

}  // namespace snvrag
