// Stream GEMM on 32x32x16 bf16 MFMAs (gfx950) for the K = D projections around the encoder:
//
//   ACT   out[M, N] = act(x W^T + b + r1[m] c1 + r2[m] c2)      (bf16)
//   HEAD2 probs[M, 2] = softmax(act(x W^T + b) w_out^T + b_out)  (the 4D hidden never leaves
//         the registers)
//   LN    out[M, D] = LN(act(x W^T + b + r1 c1 + r2 c2) + x)     (N = D)
//
// with x [M, D], W [N, D], D in {128, 256, 384} (768: ACT + GELU only), N a multiple of 64.  Reference call sites:
// fusion.py:355-360 (EmbeddingFusionModule: cat(emb, pos, af) -> Linear -> LeakyReLU + emb ->
// LayerNorm; the pos / af columns as the rank-2 term), fusion.py:131-141 (af_adapter[0] + GELU),
// foundation_model.py:64-80 (af_fusion[0] over cat(x, af, af_p) + GELU; net[0] + GELU + net[2]
// + softmax).
//
// The block tail's machinery (tail.hip) with the output tiles OUTERMOST: a workgroup owns 128
// token rows (4 waves x 32, one wave per SIMD), x stays in VGPRs as B fragments for the whole
// launch, W streams once per workgroup through an 8-slot ring of 16 KiB LDS slabs by LDS-DMA
// (buffer_load ... lds, counted vmcnt, one barrier per slab).  The stream is ordered by pairs
// of 32-feature output tiles and, inside a tile, by k-step, so each tile's accumulator is
// complete after D / 16 MFMAs: the epilogue of pair P - 1 (bias, rank terms, activation, bf16
// packing and the stores, or the head's 2-logit dot products) is spread between the MFMAs of
// pair P (ping-pong accumulators), instead of a VALU block after all tiles.  Only 4 live
// accumulators (64 registers) instead of N / 32 x 16.  Workgroups start at rotated pairs
// (blockIdx % pairs) so concurrent workgroups read different stream offsets.
#include "common.h"

#include <utility>

namespace snvrag {

constexpr int SG_FRAG = 1024;              // one A fragment: 32 W rows x 16 k (bf16)
constexpr int SG_SLAB = 16 * SG_FRAG;
constexpr int SG_NSLOT = 8;                // ring slots (128 KiB)
constexpr int SG_PF = 4;                   // A fragments read ahead
constexpr int SG_VEC_BYTES = 24 * 1024;    // f32 vector table in LDS
enum { SG_ACT = 0, SG_HEAD2 = 1, SG_LN = 2 };

// feature permutations shared with tail.hip: MFMA row m of an output tile is feature
// 16((m/4)%2) + 4(m/8) + m%4, so lane (n, hh) holds features 16hh + i (i < 16) of its tile; the
// k order of x's B fragments and W's columns: k-step s, lane half kh, element j
__host__ __device__ constexpr int sg_out_feat(int m) { return 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3); }
__host__ __device__ constexpr int sg_in_feat(int s, int kh, int j) { return 32 * (s >> 1) + 16 * kh + 8 * (s & 1) + j; }

__device__ __forceinline__ f32x16 sg_mfma(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
typedef __bf16 sg_bf16x2 __attribute__((ext_vector_type(2)));
typedef float sg_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t sg_pack2(float a, float b) {          // one v_cvt_pk_bf16_f32
  const sg_f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, sg_bf16x2));
}
__device__ __forceinline__ uint32_t sg_lds(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// LDS reads of the vector table: the reads and their wait in ONE asm statement (a compiler LDS
// read here would wait for the whole in-flight weight stream).
// the 8 x 4 floats of one tile PAIR this lane needs from a table at LDS byte address `a` (its
// tile-0 features): tile t, quad q at a + 128 t + 16 q; ONE wait for the 8 reads
__device__ __forceinline__ void sg_vec8(uint32_t a, u32x4 (&v)[8]) {
  asm volatile(
      "ds_read_b128 %0, %8 offset:0\n ds_read_b128 %1, %8 offset:16\n ds_read_b128 %2, %8 offset:32\n"
      " ds_read_b128 %3, %8 offset:48\n ds_read_b128 %4, %8 offset:128\n ds_read_b128 %5, %8 offset:144\n"
      " ds_read_b128 %6, %8 offset:160\n ds_read_b128 %7, %8 offset:176\n s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(a));
}
template <typename Body, int... Is>
__device__ __forceinline__ void sg_unroll(Body&& body, std::integer_sequence<int, Is...>) {
  (body(std::integral_constant<int, Is>{}), ...);
}
template <int ACT> __device__ __forceinline__ float sg_act(float x, float slope) {
  if constexpr (ACT == SNVRAG_ACT_GELU) return gelu_bf16(x);
  else if constexpr (ACT == SNVRAG_ACT_LRELU) return x >= 0.f ? x : x * slope;
  else if constexpr (ACT == SNVRAG_ACT_SIGMOID) return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
  else return x;
}

struct SgArgs {
  int M, N;
  const bf16* x;            // [M, D]
  bf16* out;                // [M, N] (ACT, LN)
  const char* ws;           // stream (snvrag_sgemm_pack)
  const float* vec;         // [bias N | RANK: c1 N, c2 N | LN: g N, be N | HEAD2: w_out 2N, b_out 2]
  const float* r1; const float* r2; int period;    // rank terms: row scalars r[m % period]
  float* probs; float* logits;                     // HEAD2 [M, 2] (logits optional)
  float slope, eps;
  // CAT: x = [q | bf16(x2 * g2[m % period2])], q = `x` and x2 [M, D/2], g2 [period2, D/2] (fusion.py:157:
  // cat(h, aw * h_rag) built in registers)
  const bf16* x2; const bf16* g2; int period2;
  int desync;               // > 0: first-round phase step in cycles (tail.hip's de-synchronised rounds)
};

template <int EPI, bool RANK> __host__ __device__ constexpr int sg_nvec(int N) {
  return N * (1 + (RANK ? 2 : 0) + (EPI == SG_LN ? 2 : 0) + (EPI == SG_HEAD2 ? 2 : 0)) + (EPI == SG_HEAD2 ? 2 : 0);
}

// WAVES = 4: 128 rows per workgroup, one wave per SIMD (512 registers); WAVES = 8: 256 rows, two
// waves per SIMD (256 registers each) — every streamed weight byte feeds twice the rows.
template <int D, int EPI, int ACT, bool RANK, int WAVES = 4, bool CAT = false>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4, WAVES / 4)))
void sg_kernel(SgArgs p) {
  constexpr int KS = D / 16, NT = D / 32, FPP = 2 * KS;           // fragments per tile pair
  static_assert(FPP % 16 == 0, "pairs are whole slabs");
  constexpr int SPP = FPP / 16;                                    // slabs per pair
  constexpr int RING = SG_NSLOT * SG_SLAB;
  constexpr int NTH = 64 * WAVES, ROWS = 32 * WAVES, PPW = 16 / WAVES;   // pieces per wave per slab
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* sv = reinterpret_cast<float*>(smem + RING);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x, lane = tid & 63;
  const int ln = lane & 31, hh = lane >> 5;
  const int N = p.N, NP = N / 64;                                  // tile pairs
  const long row = (long)blockIdx.x * ROWS + wave * 32 + ln;
  const long rc = row < p.M ? row : (long)p.M - 1;
  // first-round workgroups start at 8 phase offsets (see tail.hip): later rounds' activation
  // loads and output stores then stop hitting HBM as one chip-wide burst
  if (p.desync > 0 && blockIdx.x < 256) {
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }

  // ---- vector table -> LDS, x -> B fragments, rank scalars: all plain loads retire before the
  // DMA ring starts (its waits are counted)
  const int nvec = sg_nvec<EPI, RANK>(N);
  for (int i = tid; i < nvec; i += NTH) sv[i] = p.vec[i];
  u32x4 xa[KS];
  if constexpr (CAT) {
    constexpr int DH = D / 2;
    const long rg = rc % p.period2;
#pragma unroll
    for (int s = 0; s < KS / 2; ++s) xa[s] = *reinterpret_cast<const u32x4*>(p.x + rc * DH + sg_in_feat(s, hh, 0));
#pragma unroll
    for (int s = KS / 2; s < KS; ++s) {
      const int f = sg_in_feat(s, hh, 0) - DH;
      const u32x4 r = *reinterpret_cast<const u32x4*>(p.x2 + rc * DH + f);
      const u32x4 g = *reinterpret_cast<const u32x4*>(p.g2 + rg * DH + f);
#pragma unroll
      for (int w = 0; w < 4; ++w)           // bf16(r * g) per element, as rag_concat rounds it
        xa[s][w] = sg_pack2(__uint_as_float(r[w] << 16) * __uint_as_float(g[w] << 16),
                            __uint_as_float(r[w] & 0xffff0000u) * __uint_as_float(g[w] & 0xffff0000u));
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) xa[s] = *reinterpret_cast<const u32x4*>(p.x + rc * D + sg_in_feat(s, hh, 0));
  }
  float r1v = 0.f, r2v = 0.f;
  if constexpr (RANK) {
    const long ri = rc % p.period;
    r1v = p.r1[ri];
    r2v = p.r2[ri];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- weight stream: slab i of the launch = slab i % SPP of pair (rot + i / SPP) % NP
  // (LN keeps every tile in a compile-time indexed register array: stream order, no rotation)
  const int rot = EPI == SG_LN ? 0 : (int)(blockIdx.x % NP);
  const int nslab = NP * SPP;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.ws, (short)0, nslab * SG_SLAB, 0x00020000);
  const int voff = lane * 16;
  int is_slot = 0, is_i = 0;
  auto issue_next = [&]() {
    auto* dst = (__attribute__((address_space(3))) char*)(ring + is_slot + wave * PPW * SG_FRAG);
    const int pi = is_i / SPP, j = is_i - pi * SPP;
    int pr = rot + pi;
    pr = pr % NP;                                   // issues run past the end: the stream wraps
    const int src = (pr * SPP + j) * SG_SLAB;
    ++is_i;
    sg_unroll([&](auto jc) {
      constexpr int q = decltype(jc)::value;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, dst + q * SG_FRAG, 16, voff, src + (wave * PPW + q) * SG_FRAG, 0, 0);
    }, std::make_integer_sequence<int, PPW>{});
    is_slot = is_slot + SG_SLAB == RING ? 0 : is_slot + SG_SLAB;
  };
#pragma unroll
  for (int g = 0; g < SG_NSLOT - 1; ++g) issue_next();
  static_assert(PPW * (SG_NSLOT - 2) <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (SG_NSLOT - 2)) : "memory");
  __syncthreads();                                   // slab 0 and the vector table visible

  int rd_slot = 0;
  auto rdA = [&](auto j_tag, auto fi_tag) -> u32x4 {
    constexpr int j = decltype(j_tag)::value, fi = decltype(fi_tag)::value;
    int so = rd_slot + j * SG_SLAB;
    so = so >= RING ? so - RING : so;
    return *reinterpret_cast<const u32x4*>(ring + so + lane * 16 + fi * SG_FRAG);
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (SG_NSLOT - 3)) : "memory");
    __builtin_amdgcn_s_barrier();
    issue_next();                                    // into the slot of the slab two behind
  };
  u32x4 a[SG_PF];
  sg_unroll([&](auto ic) { a[decltype(ic)::value] = rdA(std::integral_constant<int, 0>{}, ic); },
            std::make_integer_sequence<int, SG_PF>{});
  // consume one tile pair (FPP fragments, whole slabs): mma(f, A) per fragment, LDS reads PF ahead
  auto run = [&](auto&& mma) {
    sg_unroll([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      const u32x4 cur = a[f % SG_PF];
      if constexpr ((f & 15) == 16 - SG_PF) {
        __builtin_amdgcn_sched_barrier(0);
        sync();
      }
      mma(fc, cur);
      constexpr int qn = f + SG_PF;
      a[f % SG_PF] = rdA(std::integral_constant<int, (qn >> 4)>{}, std::integral_constant<int, (qn & 15)>{});
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }, std::make_integer_sequence<int, FPP>{});
    rd_slot += SPP * SG_SLAB;
    rd_slot = rd_slot >= RING ? rd_slot - RING : rd_slot;
  };
  const uint32_t sv_lane = sg_lds(sv) + 64 * hh;    // &sv[16 hh]
  // the pair's epilogue vectors (bias, rank columns, head weights) for this lane's features,
  // read in blocks of 8 with one wait each — NOT one wait per 4 features in the MFMA stream
  // b = bias + r1 c1 + r2 c2 (r1, r2: this lane's row scalars, so the rank terms fold into the
  // pair's bias once); c1 / c2 keep the head's w_out rows (HEAD2) or the LN g / be (LN, at the end)
  struct PairVec {
    u32x4 b[8], c1[EPI == SG_ACT ? 1 : 8], c2[EPI == SG_ACT ? 1 : 8];
  };
  auto load_vec = [&](int pp, PairVec& v) {
    const uint32_t a = sv_lane + 4 * 64 * pp;
    sg_vec8(a, v.b);
    if constexpr (RANK) {
      u32x4 c[8];
      sg_vec8(a + 4 * N, c);
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) v.b[k][e] = __float_as_uint(fmaf(r1v, __uint_as_float(c[k][e]), __uint_as_float(v.b[k][e])));
      sg_vec8(a + 8 * N, c);
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) v.b[k][e] = __float_as_uint(fmaf(r2v, __uint_as_float(c[k][e]), __uint_as_float(v.b[k][e])));
    }
    if constexpr (EPI == SG_HEAD2) {                 // the head's w_out rows
      sg_vec8(a + 4 * N, v.c1);
      sg_vec8(a + 8 * N, v.c2);
    }
  };
  // y = act(acc + bias (+ rank)) of features 4q .. 4q + 3 (+16 hh) of tile t of the pair
  auto pre = [&](const f32x16& acc, const PairVec& v, int t, int q, float (&y)[4]) {
    const int k = 4 * t + q;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = sg_act<ACT>(acc[4 * q + e] + __uint_as_float(v.b[k][e]), p.slope);
  };

  if constexpr (EPI == SG_LN) {
    // ---- N = D: every tile kept (v = act(.) + x), then the row LayerNorm
    f32x16 acc[NT];
    float sum = 0.f, sq = 0.f;
    sg_unroll([&](auto pc) {
      constexpr int P = decltype(pc)::value;
      run([&](auto fc, const u32x4& A) {
        constexpr int f = decltype(fc)::value, T = 2 * P + f / KS, s = f % KS;
        if constexpr (s == 0) acc[T] = sg_mfma(A, xa[0], f32x16{});
        else acc[T] = sg_mfma(A, xa[s], acc[T]);
      });
    }, std::make_integer_sequence<int, NT / 2>{});
    PairVec pv;
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if ((T & 1) == 0 && q == 0) load_vec(T >> 1, pv);
        float y[4];
        pre(acc[T], pv, T & 1, q, y);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * q + e;                   // feature 32T + 16hh + i = x's k-step 2T + i/8, j = i%8
          const uint32_t w = xa[2 * T + (i >> 3)][(i & 7) >> 1];
          const float v = y[e] + ((i & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16));
          acc[T][i] = v;
          sum += v;
          sq = fmaf(v, v, sq);
        }
      }
    sum += __shfl_xor(sum, 32, 64);
    sq += __shfl_xor(sq, 32, 64);
    const float mean = sum * (1.0f / D);
    const float rstd = 1.0f / sqrtf(fmaxf(sq * (1.0f / D) - mean * mean, 0.f) + p.eps);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the stream overrun has landed
    if (row < p.M) {
#pragma unroll
      for (int T = 0; T < NT; ++T) {
        float y[16];
        if ((T & 1) == 0) {                          // g, be of the pair's two tiles
          const uint32_t a = sv_lane + 4 * (32 * T + (RANK ? 3 : 1) * N);
          sg_vec8(a, pv.b);
          sg_vec8(a + 4 * N, pv.c1);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = 4 * (T & 1) + q;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            y[4 * q + e] = fmaf((acc[T][4 * q + e] - mean) * rstd, __uint_as_float(pv.b[k][e]), __uint_as_float(pv.c1[k][e]));
        }
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          *reinterpret_cast<u32x4*>(p.out + row * D + 32 * T + 16 * hh + 8 * h2) =
              u32x4{sg_pack2(y[8 * h2], y[8 * h2 + 1]), sg_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                    sg_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), sg_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
      }
    }
    return;
  } else {
    // ---- ACT / HEAD2: pairs of tiles with ping-pong accumulators; the epilogue of the previous
    // pair in 8 steps of 4 features (step k: tile k / 4, quad k % 4) between this pair's MFMAs
    const long out_bytes = EPI == SG_ACT ? (long)p.M * N * 2 : 16;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.out, (short)0, (int)(out_bytes < 0x7fffffffL ? out_bytes : 0x7fffffffL), 0x00020000);
    const int row_off = EPI == SG_ACT ? (int)(row * N + 16 * hh) * 2 : 0;   // bytes (row < 2^31 / 2N)
    float l0 = 0.f, l1 = 0.f;                        // HEAD2 partial logits
    u32x4 yo;
    PairVec pv;
    auto epi_step = [&](const f32x16 (&acc)[2], int pp, int k) {
      const int t = k >> 2, q = k & 3;
      const int fb = 32 * (2 * pp + t) + 4 * q;     // this lane's features fb .. fb + 3 (+16 hh)
      float y[4];
      pre(acc[t], pv, t, q, y);
      if constexpr (EPI == SG_ACT) {
        yo[2 * (q & 1)] = sg_pack2(y[0], y[1]);
        yo[2 * (q & 1) + 1] = sg_pack2(y[2], y[3]);
        if (q & 1) __builtin_amdgcn_raw_buffer_store_b128(yo, ors, row_off + 2 * (fb - 4), 0, 0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          l0 = fmaf(y[e], __uint_as_float(pv.c1[k][e]), l0);
          l1 = fmaf(y[e], __uint_as_float(pv.c2[k][e]), l1);
        }
      }
    };
    constexpr int EVERY = FPP / 8;                   // one epilogue step per EVERY MFMAs
    auto pair = [&](int P, f32x16 (&an)[2], const f32x16 (&ap)[2], auto prev_tag) {
      constexpr bool PREV = decltype(prev_tag)::value;
      const int pp_prev = (rot + P - 1 + NP) % NP;
      if constexpr (PREV) load_vec(pp_prev, pv);
      run([&](auto fc, const u32x4& A) {
        constexpr int f = decltype(fc)::value, t = f / KS, s = f % KS;
        if constexpr (s == 0) an[t] = sg_mfma(A, xa[0], f32x16{});
        else an[t] = sg_mfma(A, xa[s], an[t]);
        if constexpr (PREV && f % EVERY == 0) epi_step(ap, pp_prev, f / EVERY);
      });
    };
    f32x16 e0[2], e1[2];
    pair(0, e0, e1, std::false_type{});
    int P = 1;
#pragma unroll 1
    for (; P + 1 < NP; P += 2) {
      pair(P, e1, e0, std::true_type{});
      pair(P + 1, e0, e1, std::true_type{});
    }
    const int pl = (rot + NP - 1) % NP;               // stream index of the last pair
    if (P < NP) {
      pair(P, e1, e0, std::true_type{});
      load_vec(pl, pv);
#pragma unroll
      for (int k = 0; k < 8; ++k) epi_step(e1, pl, k);
    } else {
      load_vec(pl, pv);
#pragma unroll
      for (int k = 0; k < 8; ++k) epi_step(e0, pl, k);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stores + the stream overrun retired
    if constexpr (EPI == SG_HEAD2) {
      l0 += __shfl_xor(l0, 32, 64);
      l1 += __shfl_xor(l1, 32, 64);
      if (hh == 0 && row < p.M) {
        const float2 bo = *reinterpret_cast<const float2*>(p.vec + (RANK ? 5 : 3) * N);
        l0 += bo.x;
        l1 += bo.y;
        const float mx = fmaxf(l0, l1);
        const float e0v = __expf(l0 - mx), e1v = __expf(l1 - mx), inv = 1.0f / (e0v + e1v);
        reinterpret_cast<float2*>(p.probs)[row] = make_float2(e0v * inv, e1v * inv);
        if (p.logits) reinterpret_cast<float2*>(p.logits)[row] = make_float2(l0, l1);
      }
    }
  }
}

// ------------------------------------------------------------------------- MLP --
// Two projections in one launch, the 4D hidden kept on chip (fusion.py:131-141 af_adapter:
// Linear(D, 4D) -> GELU -> Linear(4D, D) -> Sigmoid; foundation_model.py:25-33 af_fusion:
// Linear(D + 2, 4D) over cat(x, af, af_p) -> GELU -> Linear(4D, D) -> LayerNorm):
//   out[M, D] = EPI2(GELU(x W1^T + b1 [+ r1 c1 + r2 c2]) W2^T + b2),  EPI2 = sigmoid | LN.
// The stream GEMM above for W1 (hidden tile pairs, 64 units), whose pair epilogue (bias, rank,
// GELU, bf16 packing) now produces the B fragments of W2's k-steps over those 64 units (the k
// order baked into W2's columns at pack time), so phase 2 accumulates all D outputs (12 f32
// tiles, 192 registers) pair by pair.  Per pair: 48 W1 fragments (the previous pair's epilogue
// spread between them), then the previous pair's 48 W2 fragments.  4 waves x 32 rows.
// AFG: the input x = CrossAFInteraction(af, af_p) (fusion.py:82-86, the af_gate kernel's function)
// computed in the prologue straight into the B fragments instead of read from memory — the gate
// GEMV (32 hidden -> D) on MFMAs (split bf16: hi x hi + hi x lo + lo x hi, f32-level products),
// the joint encoder's LayerNorm from closed-form moments of its 2-input affine map (see
// af_gate_kernel), so the af_adapter chain is one launch (fusion.py:135-138).
constexpr int AFG_TAB = 6 * 384 + 64 + 32 + 9;      // [g2_b | j0 | j1 | jb | ln_w | ln_b] D, g1_w, g1_b, moments
template <int D, bool RANK, int EPI2, bool AFG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void mlp_kernel(SgArgs p) {
  constexpr int KS = D / 16, NT = D / 32, F1 = 2 * KS, F2 = 4 * NT, FPP = F1 + F2;
  static_assert(F1 % 16 == 0 && F2 % 16 == 0, "parts are whole slabs");
  constexpr int SPP = FPP / 16;
  constexpr int RING = SG_NSLOT * SG_SLAB;
  constexpr int H = 4 * D, NP = H / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* sv = reinterpret_cast<float*>(smem + RING);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x, lane = tid & 63;
  const int ln = lane & 31, hh = lane >> 5;
  const long row = (long)blockIdx.x * 128 + wave * 32 + ln;
  const long rc = row < p.M ? row : (long)p.M - 1;
  // first-round stagger (sg_kernel's): later rounds' activation loads and stores spread out
  if (p.desync > 0 && blockIdx.x < 256) {
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }
  // vector table [b1 H | RANK: c1 H, c2 H | b2 D | LN: g D, be D]
  constexpr int OB2 = H * (RANK ? 3 : 1);
  const int nvec = OB2 + D * (EPI2 == 1 ? 3 : 1) + (AFG ? AFG_TAB : 0);
  for (int i = tid; i < nvec; i += 256) sv[i] = p.vec[i];
  u32x4 xa[KS];
  if constexpr (AFG) {
    static_assert(D == 384 && !RANK, "AF-gate prologue: D = 384, no rank terms");
    __syncthreads();                                 // the vector table (no LDS-DMA in flight yet)
    const float* tg = sv + OB2 + D * (EPI2 == 1 ? 3 : 1);
    const float* g1w = tg + 6 * D;
    const float* g1b = g1w + 64;
    const float* mo = g1b + 32;                      // m0 m1 mb S00 S11 S01 S0b S1b Sbb
    const float a0 = p.r1[rc], a1 = p.r2[rc];
    const float mean = mo[0] * a0 + mo[1] * a1 + mo[2];
    const float var = a0 * a0 * mo[3] + a1 * a1 * mo[4] + 2.f * (a0 * a1 * mo[5] + a0 * mo[6] + a1 * mo[7]) + mo[8];
    const float rstd = 1.0f / sqrtf(fmaxf(var, 0.f) + 1e-5f);
    // gate hidden units 16 hh + 8 s + j of this lane's row (the B fragments of the gate GEMV, k16
    // step s), split into bf16 hi + lo
    u32x4 hb[2], hl[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float h[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int u = 16 * hh + 8 * s + 2 * e + t;
          h[t] = gelu_erf(g1w[u * 2] * a0 + g1w[u * 2 + 1] * a1 + g1b[u]);
        }
        const uint32_t w = sg_pack2(h[0], h[1]);
        hb[s][e] = w;
        hl[s][e] = sg_pack2(h[0] - __uint_as_float(w << 16), h[1] - __uint_as_float(w & 0xffff0000u));
      }
    // W2 fragments (tile T, step s, hi / lo) of the gate GEMV: afgate pack order, 1 KiB each
    const u32x4* gw = reinterpret_cast<const u32x4*>(p.g2) + lane;
    const float rs = p.slope;
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      u32x4 w[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) w[s][pt] = gw[((T * 2 + s) * 2 + pt) * 64];
      f32x16 g = sg_mfma(w[0][0], hb[0], f32x16{});
      g = sg_mfma(w[0][0], hl[0], g);
      g = sg_mfma(w[0][1], hb[0], g);
      g = sg_mfma(w[1][0], hb[1], g);
      g = sg_mfma(w[1][0], hl[1], g);
      g = sg_mfma(w[1][1], hb[1], g);
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {                 // feature 32 T + 16 hh + i
        const int f = 32 * T + 16 * hh + i;
        const float gt = 1.0f / (1.0f + __expf(-(g[i] + tg[f])));
        const float enc = tg[D + f] * a0 + tg[2 * D + f] * a1 + tg[3 * D + f];
        const float e = gelu_erf((enc - mean) * rstd * tg[4 * D + f] + tg[5 * D + f]);
        v[i] = a0 + rs * (gt * e);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xa[2 * T][k] = sg_pack2(v[2 * k], v[2 * k + 1]);
        xa[2 * T + 1][k] = sg_pack2(v[8 + 2 * k], v[9 + 2 * k]);
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) xa[s] = *reinterpret_cast<const u32x4*>(p.x + rc * D + sg_in_feat(s, hh, 0));
  }
  float r1v = 0.f, r2v = 0.f;
  if constexpr (RANK) {
    const long ri = rc % p.period;
    r1v = p.r1[ri];
    r2v = p.r2[ri];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int rot = (int)(blockIdx.x % NP);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.ws, (short)0, NP * SPP * SG_SLAB, 0x00020000);
  const int voff = lane * 16;
  int is_slot = 0, is_i = 0;
  // consumption order of the stream's blocks B(2P) = W1(P), B(2P + 1) = W2(P) (HS slabs each):
  // W1(r), W1(r+1), W2(r), W1(r+2), W2(r+1), ..., W1(r+NP-1), W2(r+NP-2), W2(r+NP-1) (mod NP) —
  // launch block b: 0 -> B(2r); odd b < 2NP-1 -> B(2r+b+1); even b >= 2 -> B(2r+b-1); 2NP-1 -> B(2r+b)
  constexpr int HS = F1 / 16;
  static_assert(F1 == F2, "equal W1 / W2 blocks per pair");
  auto issue_next = [&]() {
    auto* dst = (__attribute__((address_space(3))) char*)(ring + is_slot + wave * 4 * SG_FRAG);
    const int b = is_i / HS, j = is_i - b * HS;
    int m = 2 * rot + b + ((b == 0 || b == 2 * NP - 1) ? 0 : (b & 1) ? 1 : -1);
    m %= 2 * NP;                                     // (issues past the end wrap: addresses stay valid)
    const int src = (m * HS + j) * SG_SLAB;
    ++is_i;
    sg_unroll([&](auto jc) {
      constexpr int q = decltype(jc)::value;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, dst + q * SG_FRAG, 16, voff, src + (wave * 4 + q) * SG_FRAG, 0, 0);
    }, std::make_integer_sequence<int, 4>{});
    is_slot = is_slot + SG_SLAB == RING ? 0 : is_slot + SG_SLAB;
  };
#pragma unroll
  for (int g = 0; g < SG_NSLOT - 1; ++g) issue_next();
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SG_NSLOT - 2)) : "memory");
  __syncthreads();

  int rd_slot = 0;
  auto rdA = [&](auto j_tag, auto fi_tag) -> u32x4 {
    constexpr int j = decltype(j_tag)::value, fi = decltype(fi_tag)::value;
    int so = rd_slot + j * SG_SLAB;
    so = so >= RING ? so - RING : so;
    return *reinterpret_cast<const u32x4*>(ring + so + lane * 16 + fi * SG_FRAG);
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SG_NSLOT - 3)) : "memory");
    __builtin_amdgcn_s_barrier();
    issue_next();
  };
  u32x4 a[SG_PF];
  sg_unroll([&](auto ic) { a[decltype(ic)::value] = rdA(std::integral_constant<int, 0>{}, ic); },
            std::make_integer_sequence<int, SG_PF>{});
  auto run = [&](auto nf_tag, auto&& mma) {
    constexpr int NF = decltype(nf_tag)::value;
    sg_unroll([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      const u32x4 cur = a[f % SG_PF];
      if constexpr ((f & 15) == 16 - SG_PF) {
        __builtin_amdgcn_sched_barrier(0);
        sync();
      }
      mma(fc, cur);
      constexpr int qn = f + SG_PF;
      a[f % SG_PF] = rdA(std::integral_constant<int, (qn >> 4)>{}, std::integral_constant<int, (qn & 15)>{});
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }, std::make_integer_sequence<int, NF>{});
    rd_slot += (NF / 16) * SG_SLAB;
    rd_slot = rd_slot >= RING ? rd_slot - RING : rd_slot;
  };
  const uint32_t sv_lane = sg_lds(sv) + 64 * hh;
  u32x4 pb[8];                                       // the pair's b1 (+ rank) for this lane's 32 units
  auto load_b1 = [&](int pp) {
    const uint32_t ad = sv_lane + 4 * 64 * pp;
    sg_vec8(ad, pb);
    if constexpr (RANK) {
      u32x4 c[8];
      sg_vec8(ad + 4 * H, c);
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) pb[k][e] = __float_as_uint(fmaf(r1v, __uint_as_float(c[k][e]), __uint_as_float(pb[k][e])));
      sg_vec8(ad + 8 * H, c);
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) pb[k][e] = __float_as_uint(fmaf(r2v, __uint_as_float(c[k][e]), __uint_as_float(pb[k][e])));
    }
  };
  u32x4 hf[4];                                       // phase-2 B fragments of the epilogued pair
  // step k (0..7): units 4(k%4) .. +3 of tile k/4 -> GELU -> bf16 into hf[2(k/4) + (k%4)/2]
  auto epi_step = [&](const f32x16 (&e)[2], int k) {
    const int t = k >> 2, q = k & 3;
    float y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = gelu_bf16(e[t][4 * q + j] + __uint_as_float(pb[k][j]));
    hf[2 * t + (q >> 1)][2 * (q & 1)] = sg_pack2(y[0], y[1]);
    hf[2 * t + (q >> 1)][2 * (q & 1) + 1] = sg_pack2(y[2], y[3]);
  };
  constexpr int EVERY = F1 / 8;
  auto phase1 = [&](f32x16 (&en)[2], const f32x16 (&ep)[2], auto prev_tag) {
    constexpr bool PREV = decltype(prev_tag)::value;
    run(std::integral_constant<int, F1>{}, [&](auto fc, const u32x4& A) {
      constexpr int f = decltype(fc)::value, t = f / KS, s = f % KS;
      if constexpr (s == 0) en[t] = sg_mfma(A, xa[0], f32x16{});
      else en[t] = sg_mfma(A, xa[s], en[t]);
      if constexpr (PREV && f % EVERY == 0) epi_step(ep, f / EVERY);
    });
  };
  f32x16 acc[NT];
  auto phase2 = [&](auto first_tag) {                // fragment f: k-step f / NT, output tile f % NT
    constexpr bool FIRST = decltype(first_tag)::value;
    run(std::integral_constant<int, F2>{}, [&](auto fc, const u32x4& A) {
      constexpr int f = decltype(fc)::value;
      if constexpr (FIRST && f < NT) acc[f] = sg_mfma(A, hf[0], f32x16{});
      else acc[f % NT] = sg_mfma(A, hf[f / NT], acc[f % NT]);
    });
  };
  f32x16 e0[2], e1[2];
  phase1(e0, e1, std::false_type{});
  load_b1(rot);
  phase1(e1, e0, std::true_type{});
  phase2(std::true_type{});
  int P = 2;
#pragma unroll 1
  for (; P + 1 < NP; P += 2) {
    load_b1((rot + P - 1) % NP);
    phase1(e0, e1, std::true_type{});
    phase2(std::false_type{});
    load_b1((rot + P) % NP);
    phase1(e1, e0, std::true_type{});
    phase2(std::false_type{});
  }
  static_assert(NP % 2 == 0, "pairs of hidden tile pairs");
  load_b1((rot + NP - 1) % NP);                      // the last pair (in e1)
#pragma unroll
  for (int k = 0; k < 8; ++k) epi_step(e1, k);
  phase2(std::false_type{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the stream overrun has landed

  // ---- out = EPI2(acc + b2): sigmoid, or LayerNorm over the D outputs of the row
  float sum = 0.f, sq = 0.f;
#pragma unroll
  for (int T = 0; T < NT; T += 2) {
    u32x4 vb[8];
    sg_vec8(sv_lane + 4 * (OB2 + 32 * T), vb);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int tt = i >> 4, ii = i & 15;
      float v = acc[T + tt][ii] + __uint_as_float(vb[4 * tt + (ii >> 2)][ii & 3]);
      if constexpr (EPI2 == 0) v = __builtin_amdgcn_rcpf(1.0f + __expf(-v));
      acc[T + tt][ii] = v;
      sum += v;
      sq = fmaf(v, v, sq);
    }
  }
  float mean = 0.f, rstd = 1.f;
  if constexpr (EPI2 == 1) {
    sum += __shfl_xor(sum, 32, 64);
    sq += __shfl_xor(sq, 32, 64);
    mean = sum * (1.0f / D);
    rstd = 1.0f / sqrtf(fmaxf(sq * (1.0f / D) - mean * mean, 0.f) + p.eps);
  }
  if (row < p.M) {
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      float y[16];
      if constexpr (EPI2 == 1) {
        u32x4 g[8], be[8];
        sg_vec8(sv_lane + 4 * (OB2 + D + 32 * (T & ~1)), g);
        sg_vec8(sv_lane + 4 * (OB2 + 2 * D + 32 * (T & ~1)), be);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int k = 4 * (T & 1) + (i >> 2);
          y[i] = fmaf((acc[T][i] - mean) * rstd, __uint_as_float(g[k][i & 3]), __uint_as_float(be[k][i & 3]));
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = acc[T][i];
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        *reinterpret_cast<u32x4*>(p.out + row * D + 32 * T + 16 * hh + 8 * h2) =
            u32x4{sg_pack2(y[8 * h2], y[8 * h2 + 1]), sg_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                  sg_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), sg_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
    }
  }
}

// MLP stream: per hidden pair P: W1 rows 64P .. 64P + 63 as in sg_pack (F = t KS + s), then
// W2's 64 columns of the pair: fragment F2 = q NT + T, lane (m, kh) holds
// W2[32T + sg_out_feat(m)][64P + sg_in_feat(q, kh, 0 .. 7)].
__global__ void mlp_pack_kernel(int D, long n_pieces, const bf16* __restrict__ w1, const bf16* __restrict__ w2,
                                bf16* __restrict__ out) {
  const long pc = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pc >= n_pieces) return;
  const int KS = D / 16, NT = D / 32, F1 = 2 * KS, FPP = F1 + 4 * NT;
  const long F = pc / 64;
  const int l = (int)(pc % 64), m = l & 31, kh = l >> 5;
  const long P = F / FPP;
  const int f = (int)(F % FPP);
  if (f < F1) {
    const int t = f / KS, s = f % KS;
    const long n = 64 * P + 32 * t + sg_out_feat(m);
    for (int j = 0; j < 8; ++j) out[pc * 8 + j] = w1[n * D + sg_in_feat(s, kh, j)];
  } else {
    const int f2 = f - F1, q = f2 / NT, T = f2 % NT;
    const long n = 32 * T + sg_out_feat(m);
    for (int j = 0; j < 8; ++j) out[pc * 8 + j] = w2[n * 4 * D + 64 * P + sg_in_feat(q, kh, j)];
  }
}

template <int D, bool RANK, int EPI2, bool AFG = false>
static int mlp_launch(SgArgs a, hipStream_t s) {
  auto kern = mlp_kernel<D, RANK, EPI2, AFG>;
  // first-round stagger (r6, tools/sg4_desync_sweep.py OPT=mlp_desync at the bench shapes): the
  // AF-gate form, whose prologue computes its input, 25 k cycles (0.83 vs 0.89 ms); the others 5 k
  // (af_fusion: 1.465 vs 1.489 ms)
  const int64_t dz = options().mlp_desync;
  a.desync = cdiv(a.M, 128) >= 4 * 256 ? (dz >= 0 ? (int)dz : (AFG ? 25000 : 5000)) : 0;
  const size_t lds = (size_t)SG_NSLOT * SG_SLAB + SG_VEC_BYTES;
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(a.M, 128)), dim3(256), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

// One thread per 16-byte piece (8 bf16) of the stream: fragment F = T KS + s (output tile T, k-step
// s), lane l = (m = l % 32, kh = l / 32) holds W[32T + sg_out_feat(m)][sg_in_feat(s, kh, 0 .. 7)].
__global__ void sg_pack_kernel(int D, long n_pieces, const bf16* __restrict__ w, bf16* __restrict__ out) {
  const long pc = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pc >= n_pieces) return;
  const int KS = D / 16;
  const long F = pc / 64;
  const int l = (int)(pc % 64), m = l & 31, kh = l >> 5;
  const long T = F / KS;
  const int s = (int)(F % KS);
  const long n = 32 * T + sg_out_feat(m);
  for (int j = 0; j < 8; ++j) out[pc * 8 + j] = w[n * D + sg_in_feat(s, kh, j)];
}

// snvrag_derive (see the header): one thread per 8 output elements; its job by binary search
// over the jobs' first pieces
__global__ __launch_bounds__(256) void derive_kernel(const snvrag_derive_job_t* __restrict__ jobs, int njobs,
                                                     long total) {
  const long pc = (long)blockIdx.x * 256 + threadIdx.x;
  if (pc >= total) return;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].piece0 <= pc) lo = mid;
    else hi = mid - 1;
  }
  const snvrag_derive_job_t& J = jobs[lo];
  const long p = pc - J.piece0;
  auto src = [&](long r, long c) -> float {
    int i = 0;
    while (i < J.nparts - 1 && r >= J.part_rows[i]) { r -= J.part_rows[i]; ++i; }
    return J.src[i][r * J.rs[i] + c * J.cs[i]];
  };
  if (J.kind == 2) {                                  // stream-GEMM pack (sg_pack_kernel's order)
    const int D = (int)J.cols, KS = D / 16;
    const long F = p / 64;
    const int l = (int)(p % 64), m = l & 31, kh = l >> 5;
    const long T = F / KS;
    const int sidx = (int)(F % KS);
    const long n = 32 * T + sg_out_feat(m);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)src(n, sg_in_feat(sidx, kh, j));
    *reinterpret_cast<bf16x8*>((bf16*)J.dst + p * 8) = o;
    return;
  }
  if (J.kind == 3) {                                  // wide-row GEMM pack (gemm256.hip g2_pack_kernel's order)
    const int NT = (int)(J.rows / 32);
    const long F = p / 64;
    const int l = (int)(p % 64), m = l & 31, kh = l >> 5;
    const long k16 = F / NT;
    const long n = 32 * (F % NT) + sg_out_feat(m);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)src(n, 16 * k16 + 8 * kh + j);
    *reinterpret_cast<bf16x8*>((bf16*)J.dst + p * 8) = o;
    return;
  }
  const long nel = J.rows * J.cols;
  for (int j = 0; j < 8; ++j) {
    const long e = p * 8 + j;
    if (e >= nel) break;
    const long r = e / J.cols, c = e % J.cols;
    const float v = src(r, c);
    if (J.kind == 0) ((float*)J.dst)[r * J.dst_ld + c] = v;
    else ((bf16*)J.dst)[r * J.dst_ld + c] = (bf16)v;
  }
}

template <int D, int EPI, int ACT, bool RANK, int WAVES = 4, bool CAT = false>
static int sg_launch(SgArgs a, hipStream_t s) {
  auto kern = sg_kernel<D, EPI, ACT, RANK, WAVES, CAT>;
  // first-round phase step (tail.hip's de-synchronised rounds): 10 k cycles for the 8-wave
  // projections (QKV at M = 527 360: 0.559 -> 0.540 ms; 20 k / 30 k: 0.557 / 0.584,
  // tools/proj_micro.py); SNVRAG_SG_DESYNC overrides
  // 4-wave launches (r6, tools/sg4_desync_sweep.py): the LayerNorm form (emb_fusion: whole-tile
  // prologue and epilogue bursts) 5.5 k — 0.675 vs 0.772 ms; the others 10 k (cat GEMM 1.626 vs
  // 1.638, head 0.916 vs 0.920)
  const int64_t dz = options().sg_desync;
  a.desync = cdiv(a.M, 32 * WAVES) >= 4 * 256
                 ? (dz >= 0 ? (int)dz : (WAVES == 8 ? 10000 : EPI == SG_LN ? 5500 : 10000)) : 0;
  const size_t lds = (size_t)SG_NSLOT * SG_SLAB + SG_VEC_BYTES;
  static_assert((size_t)SG_NSLOT * SG_SLAB + SG_VEC_BYTES <= 160 * 1024, "LDS budget");
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(a.M, 32 * WAVES)), dim3(64 * WAVES), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

template <int D>
static int sg_dispatch(int epi, int act, bool rank, const SgArgs& a, hipStream_t s) {
  if (epi == SG_HEAD2) {
    if (act == SNVRAG_ACT_GELU) return sg_launch<D, SG_HEAD2, SNVRAG_ACT_GELU, false>(a, s);
    return fail("snvrag_sgemm_forward", "head epilogue supports GELU only");
  }
  if (epi == SG_LN) {
    if (act == SNVRAG_ACT_LRELU) {
      return rank ? sg_launch<D, SG_LN, SNVRAG_ACT_LRELU, true>(a, s) : sg_launch<D, SG_LN, SNVRAG_ACT_LRELU, false>(a, s);
    }
    return fail("snvrag_sgemm_forward", "LayerNorm epilogue supports LeakyReLU only");
  }
  if constexpr (D == 384) {
    // 8 waves (256 rows per workgroup) for the projections: 15-22 % faster than 4
    // (tools/proj_micro.py); SNVRAG_SG_WAVES4 forces 4 (A/B)
    const bool w8 = !options().sg_waves4;
    // (the rank and head variants need more than 256 registers: 4 waves)
    if (w8 && !rank && act == SNVRAG_ACT_NONE) return sg_launch<D, SG_ACT, SNVRAG_ACT_NONE, false, 8>(a, s);
    if (w8 && !rank && act == SNVRAG_ACT_GELU) return sg_launch<D, SG_ACT, SNVRAG_ACT_GELU, false, 8>(a, s);
  }
  switch (act) {
    case SNVRAG_ACT_NONE: return rank ? sg_launch<D, SG_ACT, SNVRAG_ACT_NONE, true>(a, s)
                                      : sg_launch<D, SG_ACT, SNVRAG_ACT_NONE, false>(a, s);
    case SNVRAG_ACT_GELU: return rank ? sg_launch<D, SG_ACT, SNVRAG_ACT_GELU, true>(a, s)
                                      : sg_launch<D, SG_ACT, SNVRAG_ACT_GELU, false>(a, s);
    default: return fail("snvrag_sgemm_forward", "activation epilogue supports none / GELU");
  }
}

}  // namespace snvrag

using namespace snvrag;

extern "C" size_t snvrag_sgemm_pack_bytes(int D, int N) {
  if (!(D == 128 || D == 256 || D == 384 || D == 768) || N <= 0 || N % 64) return 0;
  return (size_t)N * D * 2;
}

extern "C" int snvrag_sgemm_pack(int D, int N, const void* w, void* out, void* stream) {
  SNV_CHECK_ARG(snvrag_sgemm_pack_bytes(D, N) > 0, "stream GEMM needs D in {128, 256, 384, 768} and N % 64 == 0");
  SNV_CHECK_ARG(w && out, "null pointer");
  const long pieces = (long)N * D / 8;
  hipLaunchKernelGGL(sg_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), D, pieces,
                     (const bf16*)w, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_derive(const snvrag_derive_job_t* jobs, int njobs, int64_t total_pieces, void* stream) {
  SNV_CHECK_ARG(jobs && njobs > 0 && total_pieces >= 0, "bad job table");
  if (total_pieces == 0) return 0;
  hipLaunchKernelGGL(derive_kernel, dim3((unsigned)cdiv(total_pieces, 256)), dim3(256), 0, as_stream(stream), jobs,
                     njobs, (long)total_pieces);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_sgemm_forward(int64_t M, int D, int N, int epi, int act, float slope, const void* x,
                                    const void* wstream, const float* vec, const float* r1, const float* r2,
                                    int64_t period, float eps, void* out, float* probs, float* logits,
                                    void* stream) {
  SNV_CHECK_ARG(snvrag_sgemm_pack_bytes(D, N) > 0, "stream GEMM needs D in {128, 256, 384, 768} and N % 64 == 0");
  SNV_CHECK_ARG(epi == SG_ACT || epi == SG_HEAD2 || epi == SG_LN, "bad epilogue");
  SNV_CHECK_ARG(x && wstream && vec, "null pointer");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  const bool rank = r1 != nullptr;
  SNV_CHECK_ARG(!rank || (r2 && period > 0), "rank terms need r1, r2 and a period");
  SNV_CHECK_ARG(epi != SG_HEAD2 || (!rank && N == 4 * D && probs), "head epilogue: no rank terms, N = 4D, probs");
  SNV_CHECK_ARG(epi != SG_LN || (N == D && out), "LayerNorm epilogue needs N = D and out");
  SNV_CHECK_ARG(epi != SG_ACT || out, "null output");
  SNV_CHECK_ARG(epi != SG_ACT || M * N * 2 < (1L << 31), "output exceeds the 2 GiB buffer-store range");
  const int nvec = rank ? (epi == SG_LN ? sg_nvec<SG_LN, true>(N) : sg_nvec<SG_ACT, true>(N))
                        : (epi == SG_LN ? sg_nvec<SG_LN, false>(N)
                                        : epi == SG_HEAD2 ? sg_nvec<SG_HEAD2, false>(N) : sg_nvec<SG_ACT, false>(N));
  SNV_CHECK_ARG(nvec * 4 <= SG_VEC_BYTES, "vector table exceeds the LDS budget");
  SNV_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)wstream % 16) == 0 && (!out || ((uintptr_t)out % 16) == 0),
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  const SgArgs a{(int)M, N, (const bf16*)x, (bf16*)out, (const char*)wstream, vec, r1, r2, (int)period,
                 probs, logits, slope, eps, nullptr, nullptr, 0};
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  int rc;
  switch (D) {
    case 128: rc = sg_dispatch<128>(epi, act, rank, a, s); break;
    case 256: rc = sg_dispatch<256>(epi, act, rank, a, s); break;
    case 384: rc = sg_dispatch<384>(epi, act, rank, a, s); break;
    default:                                         // K = 2D: the rag fusion's cat(h, g * r) input
      if (epi != SG_ACT || act != SNVRAG_ACT_GELU || rank)
        return fail(__func__, "K = 768 supports the GELU activation epilogue only");
      rc = sg_launch<768, SG_ACT, SNVRAG_ACT_GELU, false>(a, s);
      break;
  }
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)N * D);
  return 0;
}

extern "C" int snvrag_sgemm_cat_forward(int64_t M, int Dh, int N, const void* q, const void* x2, const void* g2,
                                        int64_t period2, const void* wstream, const float* vec, void* out,
                                        void* stream) {
  SNV_CHECK_ARG(Dh == 384 && N > 0 && N % 64 == 0, "concatenated-input GEMM needs D/2 = 384 and N % 64 == 0");
  SNV_CHECK_ARG(q && x2 && g2 && wstream && vec && out, "null pointer");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31) && period2 > 0 && M * N * 2 < (1L << 31), "bad M / period");
  SNV_CHECK_ARG(N * 4 <= SG_VEC_BYTES, "vector table exceeds the LDS budget");
  SNV_CHECK_ARG(((uintptr_t)q % 16) == 0 && ((uintptr_t)x2 % 16) == 0 && ((uintptr_t)g2 % 16) == 0 &&
                    ((uintptr_t)wstream % 16) == 0 && ((uintptr_t)out % 16) == 0,
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  const SgArgs a{(int)M, N, (const bf16*)q, (bf16*)out, (const char*)wstream, vec, nullptr, nullptr, 0,
                 nullptr, nullptr, 0.f, 0.f, (const bf16*)x2, (const bf16*)g2, (int)period2};
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  const int rc = sg_launch<768, SG_ACT, SNVRAG_ACT_GELU, false, 4, true>(a, s);
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)N * 2 * Dh);
  return 0;
}

extern "C" size_t snvrag_mlp_pack_bytes(int D) {
  return D == 384 ? (size_t)2 * 4 * D * D * 2 : 0;
}

extern "C" int snvrag_mlp_pack(int D, const void* w1, const void* w2, void* out, void* stream) {
  SNV_CHECK_ARG(snvrag_mlp_pack_bytes(D) > 0, "MLP stream needs D = 384");
  SNV_CHECK_ARG(w1 && w2 && out, "null pointer");
  const long pieces = (long)snvrag_mlp_pack_bytes(D) / 16;
  hipLaunchKernelGGL(mlp_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), D, pieces,
                     (const bf16*)w1, (const bf16*)w2, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_mlp_forward(int64_t M, int D, int epi2, const void* x, const void* wstream, const float* vec,
                                  const float* r1, const float* r2, int64_t period, float eps, void* out,
                                  void* stream) {
  SNV_CHECK_ARG(D == 384, "MLP kernel needs D = 384");
  SNV_CHECK_ARG(epi2 == 0 || epi2 == 1, "epi2: 0 sigmoid, 1 LayerNorm");
  SNV_CHECK_ARG(x && wstream && vec && out, "null pointer");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  const bool rank = r1 != nullptr;
  SNV_CHECK_ARG(!rank || (r2 && period > 0), "rank terms need r1, r2 and a period");
  SNV_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)wstream % 16) == 0 && ((uintptr_t)out % 16) == 0,
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  const SgArgs a{(int)M, D, (const bf16*)x, (bf16*)out, (const char*)wstream, vec, r1, r2, (int)period,
                 nullptr, nullptr, 0.f, eps, nullptr, nullptr, 0};
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  const int rc = epi2 == 0 ? (rank ? mlp_launch<384, true, 0>(a, s) : mlp_launch<384, false, 0>(a, s))
                           : (rank ? mlp_launch<384, true, 1>(a, s) : mlp_launch<384, false, 1>(a, s));
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)D * 4 * D * 2);
  return 0;
}

extern "C" int snvrag_mlp_afgate_forward(int64_t M, int D, const float* af, const float* af_p, const void* gate_frags,
                                         float res_scale, const void* wstream, const float* vec, void* out,
                                         void* stream) {
  SNV_CHECK_ARG(D == 384, "MLP kernel needs D = 384");
  SNV_CHECK_ARG(af && af_p && gate_frags && wstream && vec && out, "null pointer");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)gate_frags % 16) == 0 && ((uintptr_t)wstream % 16) == 0 && ((uintptr_t)out % 16) == 0,
                "pointers must be 16-byte aligned");
  SNV_CHECK_ARG((4 * D + D + AFG_TAB) * 4 <= SG_VEC_BYTES, "vector table exceeds the LDS budget");
  if (M == 0) return 0;
  const SgArgs a{(int)M, D, nullptr, (bf16*)out, (const char*)wstream, vec, af, af_p, (int)M,
                 nullptr, nullptr, res_scale, 0.f, nullptr, (const bf16*)gate_frags, 0};
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  const int rc = mlp_launch<384, false, 0, true>(a, s);
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)D * 4 * D * 2);
  return 0;
}
