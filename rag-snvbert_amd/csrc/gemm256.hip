// Wide-row GEMM for the large-K projections onto N = 32 NT features (384 at d384), bf16:
//
//   out[M, N] = A[M, K] W[N, K]^T (+ bias[N]) (+ resid[M, N])          K % 64 == 0
//
// the shapes of FeedForward's w_2 forward (K = 4D, feed_forward.py:20) and of the large-K dX GEMMs
// of the training backward (q/k/v: K = 3D, w_1: K = 4D, pretrain_with_val_optimized.py:235) at
// M = 2 B L rows (49 440 at B = 24).  The row-panel GEMM (128-row tiles) runs those as 387
// workgroups = 1.5 rounds of the 256 CUs; here a workgroup owns 256 rows x all N features (194
// workgroups: one round), so every weight byte streamed into a CU feeds twice the rows.
//
// 4 waves (one per SIMD, 512 registers), wave w: rows 64 w .. 64 w + 63 as two 32-token groups.
// Every MFMA (v_mfma_f32_32x32x16_bf16) computes a TRANSPOSED tile — 32 weight rows (A operand, a
// 1 KiB fragment read from LDS) x 32 tokens (B operand) — so a lane ends up holding 16 consecutive
// output features of one token (the weight rows are permuted at pack time, g2_out_feat), stored as
// two 16-B pieces.  Per K-step of 64 the LDS ring streams 2 + NT / 4 slabs of 16 KiB by LDS-DMA:
// A0, A1 (the 256 rows x 128 B of A: 8 whole 128-B lines per DMA instruction, 16-B chunks XOR-
// swizzled by row & 7 so the B-fragment reads are conflict-free), then the K-step's W fragments in
// consumption order (k16 step s, feature tile T).  One barrier per slab, counted vmcnt (inline-asm
// DMA: the compiler sees no LDS stores), 7 slabs in flight.
#include "common.h"

#include <utility>

namespace snvrag {

constexpr int G2_FRAG = 1024;
constexpr int G2_SLAB = 16 * G2_FRAG;
constexpr int G2_NSLOT = 9;
constexpr int G2_ROWS = 256;
constexpr int G2_PF = 4;
constexpr int G2_NACC = 16;                          // accumulator tiles in AGPRs

// weight row held by MFMA row m of feature tile T: lane (token, hh) then holds features
// 32 T + 16 hh + i in accumulator element i
__host__ __device__ constexpr int g2_out_feat(int T, int m) {
  return 32 * T + 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3);
}

template <typename Body, int... Is>
__device__ __forceinline__ void g2_unroll(Body&& body, std::integer_sequence<int, Is...>) {
  (body(std::integral_constant<int, Is>{}), ...);
}

// 384 accumulator registers per lane: the first G2_NACC tiles live in AGPRs, the rest in VGPRs.
// The MFMA is inline asm so that the register class of every accumulator is fixed (the builtin's
// single AGPR-or-VGPR form for the whole kernel spills half of them); the compiler then does not
// know these are MFMAs, so nothing may read an accumulator within 18 wait states of its last MFMA
// unless g2_drain runs in between — including the compiler's own register moves (see g3_kernel).
template <bool AGPR>
__device__ __forceinline__ void g2_mfma(f32x16& c, const u32x4& a, const u32x4& b) {
  if constexpr (AGPR)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
// 32x32 MFMA (16 passes): a result is readable 18 wait states after issue
__device__ __forceinline__ void g2_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }

// lane id produced afresh at each use (not kept live across the K loop)
__device__ __forceinline__ int g2_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ int g2_opq(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ uint32_t g2_pack2(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

struct G2Args {
  int M, K;
  const bf16* A;
  long lda;
  const char* ws;            // snvrag_gemm256_pack stream of W
  const float* bias;         // [N] or null
  const bf16* resid;         // [M, N] (ld_resid) or null
  long ld_resid;
  bf16* out;                 // [M, N] (ldo)
  long ldo;
  unsigned long long* stamps;  // VAR 3 (diagnostics): [workgroup][wave][8] s_memtime stamps
  // EPI 1 (g3 only): row LayerNorm over the N outputs, then out = base + post_scale * LN(y) * w(af):
  // fusion.py:152-162 (the rag fusion's Linear(4D, D) -> LayerNorm, MAF weighting, residual)
  const float* ln_g;
  const float* ln_b;
  float ln_eps;
  const bf16* base;          // [M, N] (ld_base) or null
  long ld_base;
  float post_scale;
  const float* post_af;      // [period] or null: w = min(log1p(1 / (min(af, 1 - af) + 1e-6)), 3)
  long post_af_period;
  int desync;                // g3: > 0, first-round stagger step in cycles (multi-round launches)
};

__device__ __forceinline__ float g2_maf_w(float af) {   // fusion.py:155-160
  const float maf = fminf(af, 1.0f - af);
  return fminf(log1pf(1.0f / (maf + 1e-6f)), 3.0f);
}

template <int NT, int VAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void g2_kernel(G2Args p) {
  constexpr int N = 32 * NT;
  constexpr int FPK = 4 * NT;                         // W fragments per K-step of 64
  static_assert(FPK % 16 == 0, "whole W slabs per K-step");
  constexpr int WS = FPK / 16;                        // W slabs per K-step
  constexpr int SPK = 2 + WS;                         // slabs per K-step: A0, A1, W ...
  constexpr int RING = G2_NSLOT * G2_SLAB;
  constexpr int AHEAD = G2_NSLOT - 2;                 // sync(g) issues slab g + AHEAD
  constexpr int VM = 4 * (G2_NSLOT - 3);
  static_assert(VM <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* sb = reinterpret_cast<float*>(smem + RING);  // bias [N]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x;
  const int M = p.M, nk = p.K / 64;
  // VAR 3: [0] start, [1] realtime at start, [2] first slab landed, [3] K loop done, [4] end,
  // [5] realtime at end, [6] cycles in the K loop's slab waits (vmcnt + barrier), [7] cycles from
  // the A1 wait to the B fragments in registers
  unsigned long long st_wait = 0, st_b = 0, st_t = 0;
  auto stamp = [&](int i, unsigned long long v) {
    if constexpr (VAR == 3)
      if ((threadIdx.x & 63) == 0) p.stamps[((long)blockIdx.x * 4 + wave) * 8 + i] = v;
  };
  stamp(0, __builtin_amdgcn_s_memtime());
  stamp(1, __builtin_amdgcn_s_memrealtime());
  const long row0 = (long)blockIdx.x * G2_ROWS;

  for (int i = tid; i < N; i += 256) sb[i] = p.bias ? p.bias[i] : 0.f;

  // ---- issue side: slab (K-step kt, position r) into ring slot is_slot
  const long a_bytes = ((long)M - row0) * p.lda * 2;
  const i32x4 ars = dma_rsrc(p.A + row0 * p.lda, a_bytes);      // rows >= M read as zeros
  const i32x4 wrs = dma_rsrc(p.ws, (long)nk * WS * G2_SLAB);
  const uint32_t ring_lds = lds_addr(ring) + wave * 4 * G2_FRAG;
  int is_slot = 0;
  // per-lane offsets kept in two VGPRs for the whole kernel: the lane's 16 B of a fragment, and the
  // lane's piece of an A slab (row 32 w + l / 8 of the slab, swizzled chunk)
  int lane16 = g2_lane() * 16;
  int voffA;
  {
    const int l = g2_lane(), row = 32 * wave + (l >> 3);
    voffA = (int)(row * p.lda * 2) + 16 * ((l & 7) ^ ((l >> 3) & 7));
  }
  asm volatile("" : "+v"(lane16), "+v"(voffA));
  // A slab r: wave w loads pieces 4 w + j = rows 128 r + 8 (4 w + j) + l / 8, chunk (l % 8) ^ (row % 8)
  auto put = [&](int r, int kt) {                     // r, kt wave-uniform; r compile-time at every call
    const int lds = (int)g2_opq((int)ring_lds) + is_slot;
    if constexpr (VAR == 1) {                         // diagnostic: no loads
      is_slot = is_slot + G2_SLAB == RING ? 0 : is_slot + G2_SLAB;
      return;
    }
    if (r < 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        dma_x4(ars, lds + j * G2_FRAG, voffA + (int)((128 * r + 8 * j) * p.lda * 2), 128 * kt);
    } else {
      const int so = ((kt * WS + r - 2) * 16 + 4 * g2_opq(wave)) * G2_FRAG;
#pragma unroll
      for (int j = 0; j < 4; ++j) dma_x4(wrs, lds + j * G2_FRAG, lane16, so + j * G2_FRAG);
    }
    is_slot = is_slot + G2_SLAB == RING ? 0 : is_slot + G2_SLAB;
  };
  // the target of a sync at K-step k, position R (compile-time): slab (k, R) + AHEAD
  auto issue = [&](auto r_tag, int k) {
    constexpr int R = decltype(r_tag)::value;
    constexpr int RT = (R + AHEAD) % SPK, DK = (R + AHEAD) / SPK;
    int kt = k + DK;
    kt = kt < nk ? kt : nk - 1;                       // past the end: re-read the last K-step
    put(RT, kt);
  };
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // bias table loads retired
  __syncthreads();
  g2_unroll([&](auto qc) {
    constexpr int q = decltype(qc)::value;
    put(q % SPK, q / SPK < nk ? q / SPK : nk - 1);
  }, std::make_integer_sequence<int, AHEAD>{});
  auto sync = [&](auto r_tag, int k) {
    if constexpr (VAR == 3) st_t = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (VAR == 3) st_wait += __builtin_amdgcn_s_memtime() - st_t;
    issue(r_tag, k);
  };

  // ---- read side
  int rd_slot = 0;
  auto adv = [&](int n) {
    rd_slot += n * G2_SLAB;
    rd_slot = rd_slot >= RING ? rd_slot - RING : rd_slot;
  };
  auto rdA = [&](auto j_tag, auto fi_tag) -> u32x4 {  // W fragment fi of slab j of the current part
    constexpr int j = decltype(j_tag)::value, fi = decltype(fi_tag)::value;
    int so = rd_slot + j * G2_SLAB;
    so = so >= RING ? so - RING : so;
    return *reinterpret_cast<const u32x4*>(ring + so + lane16 + fi * G2_FRAG);
  };
  // B fragment (token group g, k16 step s) of this wave's rows from the K-step's A slabs (A0 at
  // the current rd_slot): row 64 w + 32 g + n lies in slab w / 2
  auto rdB = [&](int g, int s) -> u32x4 {
    const int l = g2_lane();
    const int rs = (64 * g2_opq(wave) + 32 * g + (l & 31)) & 127;
    int so = rd_slot + (g2_opq(wave) >> 1) * G2_SLAB;
    so = so >= RING ? so - RING : so;
    const int c = 2 * s + (l >> 5);
    return *reinterpret_cast<const u32x4*>(ring + so + rs * 128 + 16 * (c ^ (rs & 7)));
  };

  f32x16 acc[2][NT];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int T = 0; T < NT; ++T) acc[g][T] = f32x16{};
  u32x4 a[G2_PF];
  using R0 = std::integral_constant<int, 0>;
  using R1 = std::integral_constant<int, 1>;
  using R2 = std::integral_constant<int, 2>;

  sync(R0{}, 0);                                       // slab (0, A0)
  stamp(2, __builtin_amdgcn_s_memtime());
  st_wait = 0;
#pragma unroll 1
  for (int k = 0; k < nk; ++k) {
    // A1 landed, the B fragments of the K-step into registers (before A0's slot recycles)
    sync(R1{}, k);
    unsigned long long tb0 = 0;
    if constexpr (VAR == 3) tb0 = __builtin_amdgcn_s_memtime();
    u32x4 bf[2][4];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int s = 0; s < 4; ++s) bf[g][s] = rdB(g, s);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (VAR == 3) st_b += __builtin_amdgcn_s_memtime() - tb0;
    adv(2);
    sync(R2{}, k);                                     // the first W slab
    g2_unroll([&](auto ic) { a[decltype(ic)::value] = rdA(R0{}, ic); }, std::make_integer_sequence<int, G2_PF>{});
    // FPK fragments: fragment f = s NT + T feeds both token groups; one sync per slab, PF ahead
    g2_unroll([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      const u32x4 cur = a[f % G2_PF];
      if constexpr ((f & 15) == 16 - G2_PF) {
        __builtin_amdgcn_sched_barrier(0);
        // slab (f >> 4) + 1 of the W part: W slab, or the next K-step's A0 after the last
        sync(std::integral_constant<int, 2 + (f >> 4) + 1>{}, k);
      }
      constexpr int s = f / NT, T = f % NT;
      if constexpr (VAR != 2) {
        g2_mfma<true>(acc[0][T], cur, bf[0][s]);
        g2_mfma<(NT + T < G2_NACC)>(acc[1][T], cur, bf[1][s]);
      } else {
        asm volatile("" ::"v"(cur), "v"(bf[0][s]), "v"(bf[1][s]));
      }
      constexpr int qn = f + G2_PF;
      if constexpr (qn < FPK)
        a[f % G2_PF] = rdA(std::integral_constant<int, (qn >> 4)>{}, std::integral_constant<int, (qn & 15)>{});
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }, std::make_integer_sequence<int, FPK>{});
    adv(WS);
    if (k == nk - 1) g2_drain();                      // (inside the loop: see g3_kernel)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the ring overrun has landed
  stamp(3, __builtin_amdgcn_s_memtime());
  stamp(6, st_wait);
  stamp(7, st_b);

  // ---- epilogue: + bias (+ resid) -> bf16, two 16-B stores per (token group, feature tile)
  const long rows_left = (long)M - row0;
  const long o_bytes = rows_left * p.ldo * 2;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.out + row0 * p.ldo), (short)0, (int)(o_bytes < 0x7fffffffL ? o_bytes : 0x7fffffffL), 0x00020000);
  const long r_bytes = p.resid ? rows_left * p.ld_resid * 2 : 0;
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.resid ? p.resid + row0 * p.ld_resid : p.out), (short)0,
      (int)(r_bytes < 0x7fffffffL ? r_bytes : 0x7fffffffL), 0x00020000);
  const bool has_res = p.resid != nullptr;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int l = g2_lane();
    const int rl = 64 * wave + 32 * g + (l & 31);     // row within the workgroup's tile
    const int hh = l >> 5;
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      const int f0 = 32 * T + 16 * hh;
      u32x4 bv[4];
      const uint32_t ba = lds_addr(sb) + 4 * f0;
      asm volatile(
          "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
          " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
          : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
          : "v"(ba));
      float y[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) y[i] = acc[g][T][i] + __uint_as_float(bv[i >> 2][i & 3]);
      if (has_res) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rrs, (int)(rl * p.ld_resid + f0 + 8 * h2) * 2, 0, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y[8 * h2 + 2 * e] += __uint_as_float(r[e] << 16);
            y[8 * h2 + 2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
          }
        }
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{g2_pack2(y[8 * h2], y[8 * h2 + 1]), g2_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                  g2_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), g2_pack2(y[8 * h2 + 6], y[8 * h2 + 7])},
            ors, (int)(rl * p.ldo + f0 + 8 * h2) * 2, 0, 0);
    }
  }
  stamp(4, __builtin_amdgcn_s_memtime());
  stamp(5, __builtin_amdgcn_s_memrealtime());
}

// ---- v2 (default): the W fragments in registers, A alone through LDS
//
// Wave w owns output features 96 w .. 96 w + 95 (feature tiles 3 w .. 3 w + 2) for all 256 rows of
// the workgroup (8 token groups): 24 accumulator tiles (16 in AGPRs, 8 in VGPRs).  Per K-step of 64
// a wave needs 12 W fragments (k16 step s, its 3 tiles): loaded straight into registers by
// buffer_load_dwordx4 one K-step ahead (the register of fragment (s, t) is reloaded for the next
// K-step right after its last MFMA), so W never passes through LDS; only the 256 x 128 B image of
// A is staged (LDS-DMA, 8 whole-line pieces per wave per K-step, G3_AH images ahead, one barrier per
// K-step), and each B-fragment read from it feeds 3 MFMAs.  Per wave and K-step: 96 MFMA, 32
// ds_read_b128, 12 register loads, 8 DMA pieces.
//
// Memory-op order per K-step phase s (8 token groups): DMA piece at groups 1 and 5, the three W
// loads after group 7 — 5 vector-memory ops per phase, so the W fragments of phase s issued one
// K-step earlier have exactly 15 younger ops at the next phase s: s_waitcnt vmcnt(15).
//
// G token groups per workgroup (32 G rows, G = 4 .. 8): chosen per launch so that the workgroups
// fit one round of the CUs (M = 49 440: G = 7, 221 workgroups) — a wave's G DMA pieces per K-step
// go to phases j % 4 (d_s of them in phase s), so phase s waits with vmcnt(G + 9 - d_s).
constexpr int G3_AH = 3;                              // A images in flight ahead of the one read
constexpr int G3_NS = G3_AH + 1;                      // A image slots
constexpr int G3_PF = 3;                              // B-fragment reads ahead
__host__ __device__ constexpr int g3_img(int G) { return 32 * G * 128; }   // one A image: 32 G rows x 128 B
__host__ __device__ constexpr int g3_pieces_in_phase(int G, int s) { return G / 4 + (s < G % 4 ? 1 : 0); }

template <int G, int VAR, int EPI = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void g3_kernel(G2Args p) {
  constexpr int N = 384, TW = 3, G3_IMG = g3_img(G);
  static_assert(G >= 4 && G <= 8, "4 .. 8 token groups");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sb = reinterpret_cast<float*>(smem + G3_NS * G3_IMG);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int M = p.M, nk = p.K / 64;
  unsigned long long st_wait = 0, st_t = 0;
  auto stamp = [&](int i, unsigned long long v) {
    if constexpr (VAR == 3)
      if ((threadIdx.x & 63) == 0) p.stamps[((long)blockIdx.x * 4 + wave) * 8 + i] = v;
  };
  if (p.desync > 0 && blockIdx.x < 256) {             // first-round stagger (sg_kernel's)
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }
  stamp(0, __builtin_amdgcn_s_memtime());
  stamp(1, __builtin_amdgcn_s_memrealtime());
  const long row0 = (long)blockIdx.x * (32 * G);
  for (int i = threadIdx.x; i < N; i += 256) sb[i] = p.bias ? p.bias[i] : 0.f;
  if constexpr (EPI == 1)
    for (int i = threadIdx.x; i < N; i += 256) {
      sb[N + i] = p.ln_g[i];
      sb[2 * N + i] = p.ln_b[i];
    }

  const i32x4 ars = dma_rsrc(p.A + row0 * p.lda, ((long)M - row0) * p.lda * 2);   // rows >= M read as 0
  const i32x4 wrs = dma_rsrc(p.ws, (long)nk * 4 * 12 * G2_FRAG);
  const uint32_t img_lds = lds_addr(smem);
  // per-lane offsets (VGPRs for the whole kernel): the lane's 16 B of a fragment; its piece of an A
  // image (row l / 8 of the piece, swizzled chunk); its B-fragment bytes per k16 step s (row n,
  // chunk 2 s + kh stored at (2 s + kh) ^ (n % 8))
  int lane16, voffA, boff[4];
  {
    const int l = g2_lane(), n = l & 31, kh = l >> 5;
    lane16 = l * 16;
    voffA = (int)((l >> 3) * p.lda * 2) + 16 * ((l & 7) ^ ((l >> 3) & 7));
#pragma unroll
    for (int s = 0; s < 4; ++s) boff[s] = n * 128 + 16 * ((2 * s + kh) ^ (n & 7));
  }
  asm volatile("" : "+v"(lane16), "+v"(voffA), "+v"(boff[0]), "+v"(boff[1]), "+v"(boff[2]), "+v"(boff[3]));

  // piece j (0 .. G - 1) of A image kt into the slot at byte offset slot: rows 8 (G w + j) .. + 7
  auto putA = [&](int slot, int j, int kt) {
    if constexpr (VAR == 1) return;                   // diagnostic: no A loads
    const int pc = G * g2_opq(wave) + j;
    dma_x4(ars, img_lds + slot + pc * G2_FRAG, voffA + (int)(8 * pc * p.lda * 2), 128 * kt);
  };
  auto loadW = [&](u32x4& w, int kt, int s, int t) {
    const int so = ((4 * kt + s) * 12 + 3 * g2_opq(wave) + t) * G2_FRAG;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(w) : "v"(lane16), "s"(wrs), "s"(so) : "memory");
  };

  f32x16 acc[G][TW];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < TW; ++t) acc[g][t] = f32x16{};
  u32x4 w[4][TW];
  // prologue: the first K-step's W fragments, A images 0 .. AH - 1; wait for the W fragments and
  // image 0 only
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < TW; ++t) loadW(w[s][t], 0, s, t);
#pragma unroll
  for (int q = 0; q < G3_AH; ++q)
#pragma unroll
    for (int j = 0; j < G; ++j) putA(q * G3_IMG, j, q < nk ? q : nk - 1);
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((G3_AH - 1) * G) : "memory");
  __builtin_amdgcn_s_barrier();
  stamp(2, __builtin_amdgcn_s_memtime());

  int slot_rd = 0, slot_wr = G3_AH * G3_IMG;
#pragma unroll 1
  for (int k = 0; k < nk; ++k) {
    int ka = k + G3_AH, kw = k + 1;
    ka = ka < nk ? ka : nk - 1;                       // past the end: re-read the last K-step
    kw = kw < nk ? kw : nk - 1;
    u32x4 bq[G3_PF];
    auto rdB = [&](int i) -> u32x4 {                  // B fragment i = G s + g of this K-step
      return *reinterpret_cast<const u32x4*>(smem + slot_rd + boff[i / G] + (i % G) * 4096);
    };
    g2_unroll([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      if constexpr (VAR == 3) st_t = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(w[s][2])
                   : "n"(G + 9 - g3_pieces_in_phase(G, s)) : "memory");
      if constexpr (s == 0) {
        __builtin_amdgcn_s_barrier();                 // A(k) landed for every wave; A(k - 1)'s slot free
#pragma unroll
        for (int i = 0; i < G3_PF; ++i) bq[i] = rdB(i);
      }
      if constexpr (VAR == 3) st_wait += __builtin_amdgcn_s_memtime() - st_t;
      g2_unroll([&](auto gc) {
        constexpr int g = decltype(gc)::value, i = G * s + g;
        const u32x4 b = bq[i % G3_PF];
        if constexpr (i + G3_PF < 4 * G) bq[i % G3_PF] = rdB(i + G3_PF);
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          if constexpr (VAR != 2) {
            if (g * TW + t < G2_NACC) g2_mfma<true>(acc[g][t], w[s][t], b);
            else g2_mfma<false>(acc[g][t], w[s][t], b);
          } else {
            asm volatile("" ::"v"(w[s][t]), "v"(b));
          }
        }
        // pieces s and s + 4 of the phase at groups 1 and min(5, G - 1)
        if constexpr (g == 1) putA(slot_wr, s, ka);
        if constexpr (g == (G - 1 < 5 ? G - 1 : 5) && s + 4 < G) putA(slot_wr, s + 4, ka);
        if constexpr (g == G - 1) {
#pragma unroll
          for (int t = 0; t < TW; ++t) loadW(w[s][t], kw, s, t);
        }
        __builtin_amdgcn_sched_barrier(0);
      }, std::make_integer_sequence<int, G>{});
    }, std::make_integer_sequence<int, 4>{});
    slot_rd = slot_rd + G3_IMG == G3_NS * G3_IMG ? 0 : slot_rd + G3_IMG;
    slot_wr = slot_wr + G3_IMG == G3_NS * G3_IMG ? 0 : slot_wr + G3_IMG;
    // the last K-step's MFMA results: the drain sits INSIDE the loop body, so that the register
    // moves the compiler places on the loop exit (re-homing accumulators for the epilogue) come
    // after it — after the loop they were seen reading an AGPR before its last MFMA had written it.
    // Likewise the last K-step's overrun W loads (asm: the compiler takes their registers as written
    // at issue and dead after the loop): they must land before the loop exit, whose moves were seen
    // reusing a W register (v_accvgpr_read into v[120:121] while its buffer_load was in flight —
    // a rare wrong accumulator, tests/test_gpu_kernels.py in-place check)
    if (k == nk - 1) {
      asm volatile("s_waitcnt vmcnt(0)"
                   : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[0][2]), "+v"(w[1][0]), "+v"(w[1][1]), "+v"(w[1][2]),
                     "+v"(w[2][0]), "+v"(w[2][1]), "+v"(w[2][2]), "+v"(w[3][0]), "+v"(w[3][1]), "+v"(w[3][2])
                   :: "memory");
      g2_drain();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the A overrun DMA has landed
  stamp(3, __builtin_amdgcn_s_memtime());
  stamp(6, st_wait);

  const long rows_left = (long)M - row0;
  const long o_bytes = rows_left * p.ldo * 2;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.out + row0 * p.ldo), (short)0, (int)(o_bytes < 0x7fffffffL ? o_bytes : 0x7fffffffL), 0x00020000);
  if constexpr (EPI == 1) {
    // ---- epilogue: y = acc + bias; two-pass row LayerNorm over the 384 outputs (a row's features
    // are spread over the 4 waves: per-wave partial sums through LDS, summed in wave order); then
    // out = base + post_scale * (LN(y) g + be) * w(af[row % period]) -> bf16
    float* red = sb + 3 * N;                          // [4 waves][G][32]
    const int n = g2_lane() & 31, hh = g2_lane() >> 5;
    auto tile_vec = [&](const float* tab, int t, u32x4 (&v)[4]) {
      const uint32_t ba = lds_addr(tab) + 4 * (96 * wave + 32 * t + 16 * hh);
      asm volatile(
          "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
          " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
          : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
          : "v"(ba));
    };
    // sum over the workgroup's 4 waves of the per-(wave, group, row) partials s[g]
    auto row_sum = [&](float (&s)[G]) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        s[g] += __shfl_xor(s[g], 32, 64);
        if (hh == 0) red[(wave * G + g) * 32 + n] = s[g];
      }
      __syncthreads();
#pragma unroll
      for (int g = 0; g < G; ++g)
        s[g] = ((red[g * 32 + n] + red[(G + g) * 32 + n]) + red[(2 * G + g) * 32 + n]) + red[(3 * G + g) * 32 + n];
      __syncthreads();                                // red is rewritten by the next pass
    };
    float mean[G], rstd[G];
#pragma unroll
    for (int g = 0; g < G; ++g) mean[g] = 0.f;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      u32x4 bv[4];
      tile_vec(sb, t, bv);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 16; ++i) mean[g] += acc[g][t][i] + __uint_as_float(bv[i >> 2][i & 3]);
    }
    row_sum(mean);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      mean[g] *= 1.0f / N;
      rstd[g] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      u32x4 bv[4];
      tile_vec(sb, t, bv);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float d = acc[g][t][i] + __uint_as_float(bv[i >> 2][i & 3]) - mean[g];
          rstd[g] = fmaf(d, d, rstd[g]);
        }
    }
    row_sum(rstd);
    float w[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      rstd[g] = 1.0f / sqrtf(rstd[g] * (1.0f / N) + p.ln_eps);
      long m = row0 + 32 * g + n;
      m = m < M ? m : M - 1;
      w[g] = p.post_af ? g2_maf_w(p.post_af[p.post_af_period > 0 ? m % p.post_af_period : m]) : 1.0f;
    }
    const long b_bytes = p.base ? rows_left * p.ld_base * 2 : 0;
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.base ? p.base + row0 * p.ld_base : p.out), (short)0,
        (int)(b_bytes < 0x7fffffffL ? b_bytes : 0x7fffffffL), 0x00020000);
    // (by halves of 8 features: the b / g / be of one half, 24 registers, beside the accumulators)
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int f0 = 96 * wave + 32 * t + 16 * hh + 8 * h2;
        u32x4 bv[2], gv[2], ev[2];
        asm volatile(
            "ds_read_b128 %0, %6 offset:0\n ds_read_b128 %1, %6 offset:16\n ds_read_b128 %2, %7 offset:0\n"
            " ds_read_b128 %3, %7 offset:16\n ds_read_b128 %4, %8 offset:0\n ds_read_b128 %5, %8 offset:16\n"
            " s_waitcnt lgkmcnt(0)"
            : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(gv[0]), "=&v"(gv[1]), "=&v"(ev[0]), "=&v"(ev[1])
            : "v"(lds_addr(sb) + 4 * f0), "v"(lds_addr(sb + N) + 4 * f0), "v"(lds_addr(sb + 2 * N) + 4 * f0));
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int rl = 32 * g + n;
          float y[8];
#pragma unroll
          for (int i = 0; i < 8; ++i)
            y[i] = fmaf((acc[g][t][8 * h2 + i] + __uint_as_float(bv[i >> 2][i & 3]) - mean[g]) * rstd[g],
                        __uint_as_float(gv[i >> 2][i & 3]), __uint_as_float(ev[i >> 2][i & 3]));
          if (p.base) {
            const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(brs, (int)(rl * p.ld_base + f0) * 2, 0, 0);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              y[2 * e] = __uint_as_float(r[e] << 16) + p.post_scale * (y[2 * e] * w[g]);
              y[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u) + p.post_scale * (y[2 * e + 1] * w[g]);
            }
          }
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{g2_pack2(y[0], y[1]), g2_pack2(y[2], y[3]), g2_pack2(y[4], y[5]), g2_pack2(y[6], y[7])},
              ors, (int)(rl * p.ldo + f0) * 2, 0, 0);
        }
      }
    stamp(4, __builtin_amdgcn_s_memtime());
    stamp(5, __builtin_amdgcn_s_memrealtime());
    return;
  }
  // ---- epilogue: + bias (+ resid) -> bf16, two 16-B stores per (token group, feature tile)
  const long r_bytes = p.resid ? rows_left * p.ld_resid * 2 : 0;
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.resid ? p.resid + row0 * p.ld_resid : p.out), (short)0,
      (int)(r_bytes < 0x7fffffffL ? r_bytes : 0x7fffffffL), 0x00020000);
  const bool has_res = p.resid != nullptr;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int l = g2_lane();
    const int f0 = 96 * wave + 32 * t + 16 * (l >> 5);
    u32x4 bv[4];
    asm volatile(
        "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
        " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
        : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
        : "v"(lds_addr(sb) + 4 * f0));
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int rl = 32 * g + (g2_lane() & 31);
      float y[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) y[i] = acc[g][t][i] + __uint_as_float(bv[i >> 2][i & 3]);
      if (has_res) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rrs, (int)(rl * p.ld_resid + f0 + 8 * h2) * 2, 0, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y[8 * h2 + 2 * e] += __uint_as_float(r[e] << 16);
            y[8 * h2 + 2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
          }
        }
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{g2_pack2(y[8 * h2], y[8 * h2 + 1]), g2_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                  g2_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), g2_pack2(y[8 * h2 + 6], y[8 * h2 + 7])},
            ors, (int)(rl * p.ldo + f0 + 8 * h2) * 2, 0, 0);
    }
  }
  stamp(4, __builtin_amdgcn_s_memtime());
  stamp(5, __builtin_amdgcn_s_memrealtime());
}

template <int G, int VAR, int EPI = 0>
static int g3_launch(G2Args a, hipStream_t s) {
  auto kern = g3_kernel<G, VAR, EPI>;
  // first-round stagger for multi-round launches (r6, tools/g3_desync_sweep.py, the rag fusion's
  // K = 4D projection at M = 527 360: 10 k cycles 0.929 vs 0.961 ms; training's one-round launches none)
  const int64_t dz = options().g2_desync;
  a.desync = cdiv(a.M, 32 * G) >= 4 * 256 ? (dz >= 0 ? (int)dz : 10000) : 0;
  // + bias table (+ EPI 1: LN g, be tables and the [4][G][32] row-sum exchange)
  constexpr size_t lds = (size_t)G3_NS * g3_img(G) + 384 * 4 + (EPI == 1 ? 2 * 384 * 4 + 4 * G * 32 * 4 : 0);
  static_assert(lds <= 160 * 1024, "LDS budget");
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(a.M, 32 * G)), dim3(256), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

template <int VAR, int EPI = 0>
static int g3_dispatch(int G, const G2Args& a, hipStream_t s) {
  switch (G) {
    case 4: return g3_launch<4, VAR, EPI>(a, s);
    case 5: return g3_launch<5, VAR, EPI>(a, s);
    case 6: return g3_launch<6, VAR, EPI>(a, s);
    case 7: return g3_launch<7, VAR, EPI>(a, s);
    default: return g3_launch<8, VAR, EPI>(a, s);
  }
}

// token groups per workgroup: the fewest rows that still fit one round of the CUs (4 .. 8 groups
// of 32); past one round of 8-group workgroups, the G whose rounds x (G + 1) (a workgroup's time
// ~ G plus a fixed prologue / epilogue share) is least; option g2_groups overrides
static int g3_groups(long M) {
  static int n_cu = 0;
  if (n_cu <= 0) {
    int dev = 0, v = 0;
    n_cu = hipGetDevice(&dev) == hipSuccess &&
                   hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0
               ? v : 256;
  }
  int G = (int)std::min<long>(8, std::max<long>(4, (M + 32L * n_cu - 1) / (32L * n_cu)));
  if (M > 8L * 32 * n_cu) {
    long best = -1;
    for (int g = 8; g >= 4; --g) {
      const long rounds = (cdiv(M, 32L * g) + n_cu - 1) / n_cu, cost = rounds * (g + 1);
      if (best < 0 || cost < best) best = cost, G = g;
    }
  }
  if (options().g2_groups >= 4 && options().g2_groups <= 8) G = (int)options().g2_groups;
  return G;
}

// One thread per 16-byte piece: fragment F = k16 NT + T, lane l = (m = l % 32, kh = l / 32) holds
// W[g2_out_feat(T, m)][16 k16 + 8 kh + j], j < 8 (W bf16 [N, K] row-major, leading dim ldw)
__global__ void g2_pack_kernel(int NT, long n_pieces, const bf16* __restrict__ w, long ldw, bf16* __restrict__ out) {
  const long pc = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pc >= n_pieces) return;
  const long F = pc / 64;
  const int l = (int)(pc % 64), m = l & 31, kh = l >> 5;
  const long k16 = F / NT;
  const int T = (int)(F % NT);
  const long n = g2_out_feat(T, m);
  for (int j = 0; j < 8; ++j) out[pc * 8 + j] = w[n * ldw + 16 * k16 + 8 * kh + j];
}

template <int NT, int VAR>
static int g2_launch(const G2Args& a, hipStream_t s) {
  auto kern = g2_kernel<NT, VAR>;
  constexpr size_t lds = (size_t)G2_NSLOT * G2_SLAB + 32 * NT * 4;
  static_assert(lds <= 160 * 1024, "LDS budget");
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(a.M, G2_ROWS)), dim3(256), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

}  // namespace snvrag

using namespace snvrag;

extern "C" size_t snvrag_gemm256_pack_bytes(int N, int K) {
  if (N <= 0 || K <= 0 || N % 128 != 0 || K % 64 != 0) return 0;
  return (size_t)N * K * 2;
}

extern "C" int snvrag_gemm256_pack(int N, int K, const void* w, int64_t ldw, void* out, void* stream) {
  SNV_CHECK_ARG(snvrag_gemm256_pack_bytes(N, K) > 0, "gemm256 pack: N % 128 == 0 and K % 64 == 0");
  SNV_CHECK_ARG(w && out && ldw >= K, "bad arguments");
  const long pieces = (long)N * K / 8;
  hipLaunchKernelGGL(g2_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), N / 32,
                     pieces, (const bf16*)w, (long)ldw, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_gemm256_forward(int64_t M, int N, int K, const void* A, int64_t lda, const void* wpacked,
                                      const float* bias, const void* resid, int64_t ld_resid, void* out, int64_t ldo,
                                      void* stream) {
  SNV_CHECK_ARG(N == 384, "gemm256: N = 384");
  SNV_CHECK_ARG(K >= 64 && K % 64 == 0, "gemm256: K % 64 == 0");
  SNV_CHECK_ARG(A && wpacked && out, "null pointer");
  SNV_CHECK_ARG(M >= 0 && lda >= K && ldo >= N && (!resid || ld_resid >= N), "bad shape / leading dims");
  SNV_CHECK_ARG(lda % 8 == 0 && ldo % 8 == 0 && (!resid || ld_resid % 8 == 0), "16-byte rows");
  SNV_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)wpacked % 16) == 0 &&
                    ((uintptr_t)resid % 16) == 0,
                "16-byte aligned operands");
  SNV_CHECK_ARG(257L * lda * 2 < (1L << 31) && 257L * ldo * 2 < (1L << 31) &&
                    (!resid || 257L * ld_resid * 2 < (1L << 31)),
                "row offsets must fit 31 bits");
  if (M == 0) return 0;
  const G2Args a{(int)M, K, (const bf16*)A, (long)lda, (const char*)wpacked, bias, (const bf16*)resid,
                 (long)ld_resid, (bf16*)out, (long)ldo, nullptr};
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  const int64_t var = options().g2_variant;
  G2Args b = a;
  b.stamps = diag_stamps();
  const int G = g3_groups(M);
  // g2_variant: 0 v2 (default); 1 / 2 / 3: v2 without A loads / without MFMA / with stamps;
  // 4: v1 (W through LDS); 5 / 6 / 7: v1 without loads / without MFMA / with stamps
  int rc;
  switch (var) {
    case 1: rc = g3_dispatch<1>(G, a, s); break;
    case 2: rc = g3_dispatch<2>(G, a, s); break;
    case 3: rc = b.stamps ? g3_dispatch<3>(G, b, s) : g3_dispatch<0>(G, a, s); break;
    case 4: rc = g2_launch<12, 0>(a, s); break;
    case 5: rc = g2_launch<12, 1>(a, s); break;
    case 6: rc = g2_launch<12, 2>(a, s); break;
    case 7: rc = b.stamps ? g2_launch<12, 3>(b, s) : g2_launch<12, 0>(a, s); break;
    default: rc = g3_dispatch<0>(G, a, s);
  }
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)N * K);
  return 0;
}

extern "C" int snvrag_gemm256_ln_forward(int64_t M, int N, int K, const void* A, int64_t lda, const void* wpacked,
                                         const float* bias, const float* ln_g, const float* ln_b, float eps,
                                         const void* base, int64_t ld_base, float post_scale, const float* post_af,
                                         int64_t post_af_period, void* out, int64_t ldo, void* stream) {
  SNV_CHECK_ARG(N == 384, "gemm256: N = 384");
  SNV_CHECK_ARG(K >= 64 && K % 64 == 0, "gemm256: K % 64 == 0");
  SNV_CHECK_ARG(A && wpacked && out && ln_g && ln_b, "null pointer");
  SNV_CHECK_ARG(M >= 0 && lda >= K && ldo >= N && (!base || ld_base >= N), "bad shape / leading dims");
  SNV_CHECK_ARG(post_af_period >= 0, "bad af period");
  SNV_CHECK_ARG(lda % 8 == 0 && ldo % 8 == 0 && (!base || ld_base % 8 == 0), "16-byte rows");
  SNV_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)wpacked % 16) == 0 &&
                    ((uintptr_t)base % 16) == 0,
                "16-byte aligned operands");
  SNV_CHECK_ARG(257L * lda * 2 < (1L << 31) && 257L * ldo * 2 < (1L << 31) &&
                    (!base || 257L * ld_base * 2 < (1L << 31)),
                "row offsets must fit 31 bits");
  if (M == 0) return 0;
  G2Args a{(int)M, K, (const bf16*)A, (long)lda, (const char*)wpacked, bias, nullptr, 0, (bf16*)out, (long)ldo,
           nullptr};
  a.ln_g = ln_g;
  a.ln_b = ln_b;
  a.ln_eps = eps;
  a.base = (const bf16*)base;
  a.ld_base = (long)ld_base;
  a.post_scale = post_scale;
  a.post_af = post_af;
  a.post_af_period = (long)post_af_period;
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  // (at most 7 token groups unless option g2_groups asks for 8: the 8-group LN epilogue spills 36 B)
  const int G = options().g2_groups == 8 ? 8 : std::min(7, g3_groups(M));
  const int rc = g3_dispatch<0, 1>(G, a, s);
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)N * K);
  return 0;
}
