// Row-panel GEMM with LayerNorm-fused epilogues (gfx950 MFMA).
//
// C[128 x BN] tiles, BN = 64*NW (NW = 6 -> 384 = the model width D, so one tile
// holds whole output rows), 512 threads = 8 waves in a 2 (M) x 4 (N) grid, each
// wave 64 x 16*NW = 4 x NW MFMA 16x16 tiles.  Operands are staged with
// global_load_lds (16 B / lane, 1 KiB per wave instruction) into a 2-stage LDS
// ring of 128-B K-tile rows (one tile in flight under the MFMAs of the other).  The XOR swizzle of the ds_read_b128
// fragment reads is applied on the SOURCE address (the LDS image of a glds is
// lane-linear) — guide §5 rule 21.
//
// Epilogue options (all fused, no extra HBM pass):
//   bias, two rank-1 row*col terms (the reference's cat([x, af, af_p]) columns),
//   activation, residual add, then
//   * LN over the full output row (requires N == BN): sublayer.py:15-16 post-LN,
//     EmbeddingFusionModule / rag fusion / hap head norms, + act + (base + s*y*maf(af))
//   * or row statistics (sum, sumsq) of this tile's columns -> stats[tile_n][M]
//     (FeedForward's LayerNorm(4D), consumed by the next GEMM's A operand)
// Row-norm option: a LayerNorm of the A operand folded algebraically into the
// epilogue, acc' = rstd_m * (A W'^T) - rstd_m * mean_m * c1 with W' = W diag(gamma),
// c1 = W gamma and beta folded into the bias (feed_forward.py:20, w_2(norm(x)),
// without ever materialising norm(x)); mean/rstd from the producer's row stats.
#include "common.h"

namespace snvrag {

constexpr int R_BM = 128;

struct EpiX {
  const float* bias;
  const float* row1; long row1_stride; const float* col1;
  const float* row2; long row2_stride; const float* col2;
  long row_period;
  int act; float slope;
  const void* resid; long ld_resid;
  const float* ln_g; const float* ln_b; float ln_eps; int ln_act;
  const void* post_base; long ld_post; float post_scale; const float* post_af; long post_af_period; int post_maf;
  float* stats_out;
};

// LayerNorm of the A operand folded into the epilogue (see snvrag_rownorm_t):
//   acc' = rstd_m * acc - rstd_m * mean_m * c1[n]
struct RowNorm {
  const float* stats; int n_parts; int dim; float eps; const float* c1;
};

template <int ROWB>
__device__ __forceinline__ int rswz(int row, int chunk) {
  if constexpr (ROWB == 128) return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ void load8(const float* p, float* t) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  t[0] = a.x; t[1] = a.y; t[2] = a.z; t[3] = a.w; t[4] = b.x; t[5] = b.y; t[6] = b.z; t[7] = b.w;
}
__device__ __forceinline__ void load8(const bf16* p, float* t) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    t[2 * e] = __uint_as_float(a[e] << 16);
    t[2 * e + 1] = __uint_as_float(a[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void store8(bf16* p, const float* v) {
  bf16x8 a;
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = (bf16)v[e];
  *reinterpret_cast<bf16x8*>(p) = a;
}

__device__ __forceinline__ float maf_w(float af) {
  const float maf = fminf(af, 1.0f - af);
  return fminf(log1pf(1.0f / (maf + 1e-6f)), 3.0f);
}

// 128-B K-tile rows, 2 LDS stages: the next tile's global_load_lds in flight under this tile's
// MFMAs, vmcnt(0) + barrier per tile (a 64-B, 4-stage ring with 3 tiles in flight measured slower).
template <typename TI, typename TO, int NW, bool ROWNORM>
__global__ __launch_bounds__(512) void rows_gemm_kernel(int M, int N, int K, const TI* __restrict__ A, long lda,
                                                        const TI* __restrict__ W, long ldw, TO* __restrict__ C,
                                                        long ldc, EpiX epi, RowNorm rn, int n_tiles_n) {
  constexpr int BN = 64 * NW;
  constexpr int ROWB = 128;
  constexpr int NST = 2;
  constexpr int CPR = ROWB / 16;                   // 16-B chunks per tile row
  constexpr int RPI = 1024 / ROWB;                 // rows per 1-KiB glds wave instruction
  constexpr int EPC = 16 / sizeof(TI);
  constexpr int EPT = ROWB / sizeof(TI);           // K elements per K-tile
  constexpr int STAGE = (R_BM + BN) * ROWB;
  constexpr int A_INSTR = R_BM / RPI / 8;          // per wave (8 waves)
  constexpr int W_INSTR = BN / RPI / 8;
  constexpr int P = A_INSTR + W_INSTR;             // glds per wave per K-tile
  static_assert(BN % (RPI * 8) == 0 && R_BM % (RPI * 8) == 0, "tile rows must split over 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* rowstat = reinterpret_cast<float2*>(smem + NST * STAGE);
  float* colv = reinterpret_cast<float*>(smem + NST * STAGE + R_BM * sizeof(float2));  // [6][BN]

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tm = wg / n_tiles_n, tn = wg % n_tiles_n;
  const int m0 = tm * R_BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int wmi = wave >> 2, wni = wave & 3;
  const int wm = 64 * wmi, wn = 16 * NW * wni;
  const int mrows = min(R_BM, M - m0), nrows = min(BN, N - n0);
  const TI* Ab = A + (long)m0 * lda;
  const TI* Wb = W + (long)n0 * ldw;
  const int nk = K / EPT;

  if constexpr (ROWNORM) {
    if (tid < R_BM) {
      float s = 0.f, ss = 0.f;
      const int m = min(m0 + tid, M - 1);
      for (int p = 0; p < rn.n_parts; ++p) {
        const float2 st = reinterpret_cast<const float2*>(rn.stats)[(long)p * M + m];
        s += st.x; ss += st.y;
      }
      const float mean = s / rn.dim;
      const float var = fmaxf(ss / rn.dim - mean * mean, 0.f);
      const float rstd = 1.0f / sqrtf(var + rn.eps);
      rowstat[tid] = make_float2(rstd, -rstd * mean);
    }
  }

  // per-column epilogue vectors (c1, bias, col1, col2, ln_g, ln_b) staged once in LDS
  {
    const float* cp[6] = {ROWNORM ? rn.c1 : nullptr, epi.bias, epi.row1 ? epi.col1 : nullptr,
                          epi.row2 ? epi.col2 : nullptr, epi.ln_g, epi.ln_b};
#pragma unroll
    for (int v = 0; v < 6; ++v)
      if (cp[v] && tid < BN) colv[v * BN + tid] = cp[v][n0 + tid];
  }

  auto issue = [&](int stage, int k0) {
    char* At = smem + stage * STAGE;
    char* Wt = At + R_BM * ROWB;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) {
      const int r0 = (wave * A_INSTR + j) * RPI;
      const int r = r0 + lane / CPR, c = (lane % CPR) ^ (ROWB == 128 ? ((r >> 1) & 7) : ((r >> 2) & 3));
      const int rs = r < mrows ? r : mrows - 1;
      glds16(Ab + (long)rs * lda + k0 + c * EPC, At + r0 * ROWB);
    }
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int r0 = (wave * W_INSTR + j) * RPI;
      const int r = r0 + lane / CPR, c = (lane % CPR) ^ (ROWB == 128 ? ((r >> 1) & 7) : ((r >> 2) & 3));
      const int rs = r < nrows ? r : nrows - 1;
      glds16(Wb + (long)rs * ldw + k0 + c * EPC, Wt + r0 * ROWB);
    }
  };

  f32x4 acc[4][NW];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const char* At = smem + stage * STAGE;
    const char* Wt = At + R_BM * ROWB;
#pragma unroll
    for (int kc = 0; kc < CPR / 4; ++kc) {
      u32x4 a[4], b[NW];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const u32x4*>(At + rswz<ROWB>(wm + 16 * t + li, 4 * kc + lg));
#pragma unroll
      for (int t = 0; t < NW; ++t) b[t] = *reinterpret_cast<const u32x4*>(Wt + rswz<ROWB>(wn + 16 * t + li, 4 * kc + lg));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NW; ++nt) {
          if constexpr (sizeof(TI) == 2) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, a[mt]), __builtin_bit_cast(bf16x8, b[nt]), acc[mt][nt], 0, 0, 0);
          } else {
            const f32x4 av = __builtin_bit_cast(f32x4, a[mt]), bv = __builtin_bit_cast(f32x4, b[nt]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc[mt][nt], 0, 0, 0);
          }
        }
    }
  };

  issue(0, 0);
  vm_wait<0>();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(cur ^ 1, (kt + 1) * EPT);
    compute(cur);
    vm_wait<0>();
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue --
  // Accumulators go to LDS as f32 (one 64-row half at a time, the ring is free), then
  // every wave walks whole rows: RL lanes per row, CPL 8-column chunks per lane, so
  // every global access (bias/LN vectors, residual, output) is a 16/32-B vector and
  // the LayerNorm reductions stay inside RL lanes.
  constexpr int SLD = BN + 4;                      // f32 row stride: rows 4 apart hit different banks
  constexpr int RL = BN / 8 >= 16 ? 16 : BN / 8;   // lanes per row
  constexpr int CPL = BN / 8 / RL;                 // 8-column chunks per lane
  constexpr int RPW = 64 / RL;                     // rows per wave per pass
  static_assert(64 * SLD * 4 <= NST * STAGE, "epilogue tile must fit the LDS ring");
  float* tile = reinterpret_cast<float*>(smem);
  const int sub = lane % RL, rw = lane / RL;
  const bool do_ln = epi.ln_g != nullptr;
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    if (wmi == half) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NW; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) tile[(16 * mt + 4 * lg + i) * SLD + wn + 16 * nt + li] = acc[mt][nt][i];
    }
    __syncthreads();
    constexpr int NIT = 64 / (8 * RPW);            // row passes per wave per half
    float res[NIT][CPL][8];
    if (epi.resid) {                               // issue every residual load of this half first
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int m = m0 + 64 * half + (wave + 8 * it) * RPW + rw;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          if (m < M) load8(reinterpret_cast<const TO*>(epi.resid) + (long)m * epi.ld_resid + n0 + 8 * (sub + RL * j), res[it][j]);
          else {
#pragma unroll
            for (int e = 0; e < 8; ++e) res[it][j][e] = 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rl = (wave + 8 * it) * RPW + rw;
      const int m = m0 + 64 * half + rl;
      const bool mv = m < M;
      float v[CPL][8];
#pragma unroll
      for (int j = 0; j < CPL; ++j) load8(tile + rl * SLD + 8 * (sub + RL * j), v[j]);
      const long mr = epi.row_period > 0 ? (m % epi.row_period) : m;
      const float r1 = (epi.row1 && mv) ? epi.row1[mr * epi.row1_stride] : 0.f;
      const float r2 = (epi.row2 && mv) ? epi.row2[mr * epi.row2_stride] : 0.f;
      float2 rs = make_float2(1.f, 0.f);
      if constexpr (ROWNORM) rs = rowstat[64 * half + rl];
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const int c = 8 * (sub + RL * j);
        float t[8];
        if constexpr (ROWNORM) {
          load8(colv + 0 * BN + c, t);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] = rs.x * v[j][e] + rs.y * t[e];
        }
        if (epi.bias) {
          load8(colv + 1 * BN + c, t);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] += t[e];
        }
        if (epi.row1) {
          load8(colv + 2 * BN + c, t);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] = fmaf(r1, t[e], v[j][e]);
        }
        if (epi.row2) {
          load8(colv + 3 * BN + c, t);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] = fmaf(r2, t[e], v[j][e]);
        }
        if (epi.act == SNVRAG_ACT_LRELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] = v[j][e] >= 0.f ? v[j][e] : v[j][e] * epi.slope;
        } else if (epi.act) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] = apply_act_t<TO>(epi.act, v[j][e], epi.slope);
        }
        if (epi.resid) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] += res[it][j][e];
        }
      }
      if (do_ln) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) s += v[j][e];
        const float mean = group_sum<RL>(s) / (float)N;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) { const float d = v[j][e] - mean; q = fmaf(d, d, q); }
        const float rstd = 1.0f / sqrtf(group_sum<RL>(q) / (float)N + epi.ln_eps);
        float w = 1.0f;
        if (epi.post_maf && mv) w = maf_w(epi.post_af[epi.post_af_period > 0 ? m % epi.post_af_period : m]);
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const int c = 8 * (sub + RL * j);
          float g[8], bb[8];
          load8(colv + 4 * BN + c, g);
          load8(colv + 5 * BN + c, bb);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[j][e] = (v[j][e] - mean) * rstd * g[e] + bb[e];
          if (epi.ln_act) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[j][e] = apply_act(epi.ln_act, v[j][e], 0.f);
          }
          if (epi.post_base && mv) {
            load8(reinterpret_cast<const TO*>(epi.post_base) + (long)m * epi.ld_post + n0 + c, g);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[j][e] = g[e] + epi.post_scale * (v[j][e] * w);
          }
        }
      }
      if (epi.stats_out) {
        float s = 0.f, ss = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) { s += v[j][e]; ss = fmaf(v[j][e], v[j][e], ss); }
        s = group_sum<RL>(s);
        ss = group_sum<RL>(ss);
        if (sub == 0 && mv) reinterpret_cast<float2*>(epi.stats_out)[(long)tn * M + m] = make_float2(s, ss);
      }
      if (mv) {
#pragma unroll
        for (int j = 0; j < CPL; ++j) store8(C + (long)m * ldc + n0 + 8 * (sub + RL * j), v[j]);
      }
    }
    __syncthreads();
  }
}

template <typename TI, typename TO, int NW, bool RN>
static int launch_rows_v(long M, long N, long K, const void* A, long lda, const void* W, long ldw, void* C, long ldc,
                         const EpiX& e, const RowNorm& rn, hipStream_t s) {
  constexpr int BN = 64 * NW;
  constexpr int ROWB = 128, NST = 2;
  const int tn = cdiv(N, BN), tm = cdiv(M, R_BM);
  const long nb = (long)tn * tm;
  SNV_CHECK_ARG(nb < (1L << 31), "grid too large");
  const size_t lds = NST * (size_t)(R_BM + BN) * ROWB + R_BM * sizeof(float2) + 6 * BN * sizeof(float);
  auto kern = rows_gemm_kernel<TI, TO, NW, RN>;
  static bool attr = false;
  if (!attr) {
    SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(512), lds, s, (int)M, (int)N, (int)K, (const TI*)A, lda,
                     (const TI*)W, ldw, (TO*)C, ldc, e, rn, tn);
  SNV_LAUNCH_CHECK();
  return 0;
}

template <typename TI, typename TO, int NW>
static int launch_rows(long M, long N, long K, const void* A, long lda, const void* W, long ldw, void* C, long ldc,
                       const EpiX& e, const RowNorm* rn, hipStream_t s) {
  RowNorm r = rn ? *rn : RowNorm{};
  if (rn) return launch_rows_v<TI, TO, NW, true>(M, N, K, A, lda, W, ldw, C, ldc, e, r, s);
  return launch_rows_v<TI, TO, NW, false>(M, N, K, A, lda, W, ldw, C, ldc, e, r, s);
}

template <typename TI, typename TO>
static int dispatch_nw(int nw, long M, long N, long K, const void* A, long lda, const void* W, long ldw, void* C,
                       long ldc, const EpiX& e, const RowNorm* an, hipStream_t s) {
  switch (nw) {
    case 1: return launch_rows<TI, TO, 1>(M, N, K, A, lda, W, ldw, C, ldc, e, an, s);
    case 2: return launch_rows<TI, TO, 2>(M, N, K, A, lda, W, ldw, C, ldc, e, an, s);
    case 4: return launch_rows<TI, TO, 4>(M, N, K, A, lda, W, ldw, C, ldc, e, an, s);
    default: return launch_rows<TI, TO, 6>(M, N, K, A, lda, W, ldw, C, ldc, e, an, s);
  }
}

// tile width for an N: prefer 384 (6), then 256, 128, 64; 0 = unsupported
int rows_pick_nw(long N, bool need_full_row) {
  const int force = (int)options().gemm_nw;
  if (force && !need_full_row && N % (64L * force) == 0 && (force == 1 || force == 2 || force == 4 || force == 6))
    return force;
  const int cands[4] = {6, 4, 2, 1};
  for (int c : cands) {
    const long bn = 64L * c;
    if (need_full_row ? (N == bn) : (N % bn == 0)) return c;
  }
  return 0;
}

int rows_linear(int din, int dout, long M, long N, long K, const void* A, long lda, const void* W, long ldw,
                void* C, long ldc, const snvrag_epilogue_t* epi, const snvrag_rownorm_t* anorm, hipStream_t s) {
  const bool full = epi && epi->ln_g;
  const int nw = rows_pick_nw(N, full);
  SNV_CHECK_ARG(nw > 0, full ? "LayerNorm epilogue needs N in {64,128,256,384}" : "N must be a multiple of 64");
  const int ept = din == SNVRAG_BF16 ? 64 : 32;
  SNV_CHECK_ARG(K % ept == 0, "row-panel GEMM needs K % 64 (bf16) / 32 (f32) == 0");
  EpiX e{};
  if (epi) {
    e.bias = epi->bias; e.row1 = epi->row1; e.row1_stride = epi->row1_stride; e.col1 = epi->col1;
    e.row2 = epi->row2; e.row2_stride = epi->row2_stride; e.col2 = epi->col2; e.row_period = epi->row_period;
    e.act = epi->act; e.slope = epi->slope; e.resid = epi->resid; e.ld_resid = epi->ld_resid;
    e.ln_g = epi->ln_g; e.ln_b = epi->ln_b; e.ln_eps = epi->ln_eps; e.ln_act = epi->ln_act;
    e.post_base = epi->post_base; e.ld_post = epi->ld_post; e.post_scale = epi->post_scale;
    e.post_af = epi->post_af; e.post_af_period = epi->post_af_period; e.post_maf = epi->post_maf;
    e.stats_out = epi->stats_out;
  }
  RowNorm an{};
  if (anorm) {
    an.stats = anorm->stats; an.n_parts = anorm->n_parts; an.dim = (int)anorm->dim; an.eps = anorm->eps;
    an.c1 = anorm->c1;
    SNV_CHECK_ARG(an.stats && an.c1, "rownorm needs stats and c1");
  }
  const RowNorm* ap = anorm ? &an : nullptr;
  if (din == SNVRAG_BF16 && dout == SNVRAG_BF16) return dispatch_nw<bf16, bf16>(nw, M, N, K, A, lda, W, ldw, C, ldc, e, ap, s);
  if (din == SNVRAG_BF16) return dispatch_nw<bf16, float>(nw, M, N, K, A, lda, W, ldw, C, ldc, e, ap, s);
  if (dout == SNVRAG_F32) return dispatch_nw<float, float>(nw, M, N, K, A, lda, W, ldw, C, ldc, e, ap, s);
  return dispatch_nw<float, bf16>(nw, M, N, K, A, lda, W, ldw, C, ldc, e, ap, s);
}

}  // namespace snvrag
