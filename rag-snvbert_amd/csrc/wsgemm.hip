// Weight-streaming row GEMM (bf16, gfx950): out[M, N] = epi(A[M, K] W[N, K]^T).
//
// The encoder's K = 384 projections (QKV of multi_head_attention.py:44, the output
// projection :51 + SublayerConnection LN, sublayer.py:15-16) are too short in K for a
// K-streaming GEMM: each 128-row tile would fetch its A rows from HBM and finish after
// six K steps, so the A-load latency and the epilogue dominate (~500 TFLOP/s measured,
// hipBLASLt likewise).  Here a workgroup loads its 128 A rows ONCE into LDS (MFMA
// B-operand order, 16 rows per wave) and streams the weights through a 4-slot LDS ring
// of 16 KiB slabs packed in MFMA A-fragment order (wsg_pack) — the structure of the
// fused FFN kernel's first phase (ffn.hip).  Every MFMA computes a transposed tile
// (64 output columns x 16 rows per chunk), so a lane ends up holding one row's values;
// the pack permutes W's rows so lane group lg holds 16 CONSECUTIVE output columns
// (col = 16 lg + 4 t + i for tile t, accumulator i): 32-byte row-contiguous stores.
// Epilogues: (0) bias [+ activation] -> bf16 store per 64-column chunk;
//            (1) bias + residual + LayerNorm over the full row (N <= 384, all chunks
//                kept in registers), the out-projection + sublayer LN in one pass.
#include "common.h"

namespace snvrag {

constexpr int WS_SLAB = 16384;   // 16 fragment blocks of 1 KiB
constexpr int WS_NSLOT = 4;
constexpr int WS_PD = 3;         // slabs in flight
constexpr int WS_ROWS = 128;     // 8 waves x 16 rows

template <int K> struct WsShape {
  static constexpr int KS = K / 32;             // 32-wide k steps
  static constexpr int NB = K / 128;            // slabs per 64-column chunk
  static constexpr int XT = 8 * KS * 1024;      // A tile in LDS
  static constexpr int LDS = XT + WS_NSLOT * WS_SLAB;
};

// output column of A-row r (0..15) of tile t inside a 64-column chunk
__host__ __device__ constexpr int wsg_col(int t, int r) { return 16 * (r >> 2) + 4 * t + (r & 3); }

__device__ __forceinline__ void ws_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
template <int BPW> __device__ __forceinline__ void ws_wait(int younger) {
  switch (younger) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BPW) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * BPW) : "memory"); break;
  }
}
__device__ __forceinline__ uint32_t ws_pack2(float a, float b) {
  bf16 x = (bf16)a, y = (bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}
__device__ __forceinline__ f32x4 ws_mfma(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

struct WsEpi {
  const float* bias;       // [N]
  int act; float slope;    // EPI 0
  const bf16* resid;       // EPI 1: [M, ldr]
  long ld_resid;
  const float* ln_g; const float* ln_b; float eps;
  // EPI 2 (hap head, foundation_model.py:77-80): logits = act(.) w_out^T + b_out (2 outputs),
  // probs = softmax(logits); the 4D hidden never leaves the registers
  const float* w_out; const float* b_out; float* logits; float* probs;
  // EPI 0 / 1: rank-1 row x column terms added before the activation (the cat(x, af, af_p)
  // columns of fusion.py:355-360 / foundation_model.py:25-33 as rank updates); row index
  // taken modulo row_period when > 0
  const float* row1; const float* col1; const float* row2; const float* col2; long row_period;
};

template <int K, int NCH, int EPI>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void wsg_kernel(int M, const bf16* __restrict__ A, const char* __restrict__ ws, bf16* __restrict__ out, long ldo,
                WsEpi e) {
  using S = WsShape<K>;
  constexpr int KS = S::KS, NB = S::NB, NSLAB = NCH * NB;
  constexpr int BPW = 2;                          // 1-KiB blocks of a slab per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const long rbase = (long)blockIdx.x * WS_ROWS + wave * 16;
  char* xt = smem + wave * (KS * 1024);
  const char* xtl = xt + lane * 16;
  char* ring = smem + S::XT;
  {
    const long r = min(rbase + li, (long)M - 1);
#pragma unroll
    for (int s = 0; s < KS; ++s) ws_glds16(A + r * K + 32 * s + 8 * lg, xt + s * 1024);
  }
  // workgroups start at different chunks so concurrent CUs of an XCD read different slabs
  const int rot = (int)(blockIdx.x % NCH);
  auto chunk_of = [&](int c0) { return c0 + rot >= NCH ? c0 + rot - NCH : c0 + rot; };
  auto issue = [&](int i) {
    if (i < NSLAB) {
      const int cc = chunk_of(i / NB);
      const char* src = ws + ((long)cc * NB + i % NB) * WS_SLAB + wave * BPW * 1024 + lane * 16;
      char* dst = ring + (i % WS_NSLOT) * WS_SLAB + wave * BPW * 1024;
#pragma unroll
      for (int j = 0; j < BPW; ++j) ws_glds16(src + j * 1024, dst + j * 1024);
    }
  };
  auto step = [&](int i) -> const char* {
    ws_wait<BPW>(min(WS_PD - 1, NSLAB - 1 - i));
    __builtin_amdgcn_s_barrier();
    issue(i + WS_PD);
    return ring + (i % WS_NSLOT) * WS_SLAB + lane * 16;
  };
#pragma unroll
  for (int i = 0; i < WS_PD; ++i) issue(i);

  const long row = rbase + li;
  const bool rv = row < M;
  float rk1 = 0.f, rk2 = 0.f;
  if constexpr (EPI != 2) {
    const long rr = e.row_period > 0 ? (rv ? row : 0) % e.row_period : (rv ? row : 0);
    if (e.row1) rk1 = e.row1[rr];
    if (e.row2) rk2 = e.row2[rr];
  }
  float keep[EPI == 1 ? NCH : 1][16];
  float po0 = 0.f, po1 = 0.f;                     // EPI 2 partial logits
  int slab = 0;
#pragma unroll EPI == 1 ? NCH : 1
  for (int c0 = 0; c0 < NCH; ++c0) {
    const int c = chunk_of(c0);
    f32x4 h[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) h[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      const char* sl = step(slab++);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        u32x4 a[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const u32x4*>(sl + (t * 4 + s) * 1024);
        const u32x4 b = *reinterpret_cast<const u32x4*>(xtl + (kb * 4 + s) * 1024);
#pragma unroll
        for (int t = 0; t < 4; ++t) h[t] = ws_mfma(a[t], b, h[t]);
      }
    }
    // lane (li, lg) holds columns c*64 + 16 lg + (4 t + i) of row li
    const float* bp = e.bias + c * 64 + 16 * lg;
    float v[16];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 bb = *reinterpret_cast<const float4*>(bp + 4 * t);
      v[4 * t + 0] = h[t][0] + bb.x;
      v[4 * t + 1] = h[t][1] + bb.y;
      v[4 * t + 2] = h[t][2] + bb.z;
      v[4 * t + 3] = h[t][3] + bb.w;
    }
    if constexpr (EPI != 2) {
      if (e.row1) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float4 cc = *reinterpret_cast<const float4*>(e.col1 + c * 64 + 16 * lg + 4 * t);
          v[4 * t + 0] = fmaf(rk1, cc.x, v[4 * t + 0]);
          v[4 * t + 1] = fmaf(rk1, cc.y, v[4 * t + 1]);
          v[4 * t + 2] = fmaf(rk1, cc.z, v[4 * t + 2]);
          v[4 * t + 3] = fmaf(rk1, cc.w, v[4 * t + 3]);
        }
      }
      if (e.row2) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float4 cc = *reinterpret_cast<const float4*>(e.col2 + c * 64 + 16 * lg + 4 * t);
          v[4 * t + 0] = fmaf(rk2, cc.x, v[4 * t + 0]);
          v[4 * t + 1] = fmaf(rk2, cc.y, v[4 * t + 1]);
          v[4 * t + 2] = fmaf(rk2, cc.z, v[4 * t + 2]);
          v[4 * t + 3] = fmaf(rk2, cc.w, v[4 * t + 3]);
        }
      }
    }
    if constexpr (EPI == 2) {
      if (e.act == SNVRAG_ACT_LRELU) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = v[j] >= 0.f ? v[j] : v[j] * e.slope;
      } else if (e.act) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = apply_act_t<bf16>(e.act, v[j], e.slope);
      }
      const int col = c * 64 + 16 * lg;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float4 w0 = *reinterpret_cast<const float4*>(e.w_out + col + 4 * j4);
        const float4 w1 = *reinterpret_cast<const float4*>(e.w_out + NCH * 64 + col + 4 * j4);
        po0 += v[4 * j4] * w0.x + v[4 * j4 + 1] * w0.y + v[4 * j4 + 2] * w0.z + v[4 * j4 + 3] * w0.w;
        po1 += v[4 * j4] * w1.x + v[4 * j4 + 1] * w1.y + v[4 * j4 + 2] * w1.z + v[4 * j4 + 3] * w1.w;
      }
    } else if constexpr (EPI == 0) {
      if (e.act == SNVRAG_ACT_LRELU) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = v[j] >= 0.f ? v[j] : v[j] * e.slope;
      } else if (e.act) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = apply_act_t<bf16>(e.act, v[j], e.slope);
      }
      if (rv) {
        u32x4* op = reinterpret_cast<u32x4*>(out + row * ldo + c * 64 + 16 * lg);
        op[0] = u32x4{ws_pack2(v[0], v[1]), ws_pack2(v[2], v[3]), ws_pack2(v[4], v[5]), ws_pack2(v[6], v[7])};
        op[1] = u32x4{ws_pack2(v[8], v[9]), ws_pack2(v[10], v[11]), ws_pack2(v[12], v[13]), ws_pack2(v[14], v[15])};
      }
    } else {
      if (e.act == SNVRAG_ACT_LRELU) {   // act(.) + residual, then the LayerNorm
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = v[j] >= 0.f ? v[j] : v[j] * e.slope;
      } else if (e.act) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = apply_act_t<bf16>(e.act, v[j], e.slope);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) keep[c0][j] = v[j];
    }
  }
  if constexpr (EPI == 2) {
    po0 += __shfl_xor(po0, 16, 64);
    po0 += __shfl_xor(po0, 32, 64);
    po1 += __shfl_xor(po1, 16, 64);
    po1 += __shfl_xor(po1, 32, 64);
    if (rv && lg == 0) {
      const float l0 = po0 + e.b_out[0], l1 = po1 + e.b_out[1];
      if (e.logits) reinterpret_cast<float2*>(e.logits)[row] = make_float2(l0, l1);
      const float mx = fmaxf(l0, l1), e0 = expf(l0 - mx), e1 = expf(l1 - mx), inv = 1.0f / (e0 + e1);
      reinterpret_cast<float2*>(e.probs)[row] = make_float2(e0 * inv, e1 * inv);
    }
  }
  if constexpr (EPI == 1) {
    // residual + LayerNorm over the N = 64 NCH columns of the row (4 lanes x NCH x 16)
    constexpr int N = NCH * 64;
    float sum = 0.f;
#pragma unroll
    for (int c0 = 0; c0 < NCH; ++c0) {
      const int c = chunk_of(c0);
      const long rr = rv ? row : 0;
      const u32x4* rp = reinterpret_cast<const u32x4*>(e.resid + rr * e.ld_resid + c * 64 + 16 * lg);
      const u32x4 r0 = rp[0], r1 = rp[1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w0 = r0[j >> 1], w1 = r1[j >> 1];
        keep[c0][j] += (j & 1) ? __uint_as_float(w0 & 0xffff0000u) : __uint_as_float(w0 << 16);
        keep[c0][8 + j] += (j & 1) ? __uint_as_float(w1 & 0xffff0000u) : __uint_as_float(w1 << 16);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) sum += keep[c0][j];
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float mean = sum * (1.0f / N);
    float q = 0.f;
#pragma unroll
    for (int c0 = 0; c0 < NCH; ++c0)
#pragma unroll
      for (int j = 0; j < 16; ++j) { const float d = keep[c0][j] - mean; q = fmaf(d, d, q); }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rstd = 1.0f / sqrtf(q * (1.0f / N) + e.eps);
    if (rv) {
#pragma unroll
      for (int c0 = 0; c0 < NCH; ++c0) {
        const int col = chunk_of(c0) * 64 + 16 * lg;
        float y[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) y[j] = (keep[c0][j] - mean) * rstd * e.ln_g[col + j] + e.ln_b[col + j];
        u32x4* op = reinterpret_cast<u32x4*>(out + row * ldo + col);
        op[0] = u32x4{ws_pack2(y[0], y[1]), ws_pack2(y[2], y[3]), ws_pack2(y[4], y[5]), ws_pack2(y[6], y[7])};
        op[1] = u32x4{ws_pack2(y[8], y[9]), ws_pack2(y[10], y[11]), ws_pack2(y[12], y[13]), ws_pack2(y[14], y[15])};
      }
    }
  }
}

// one thread per 16-byte piece: slab (c*NB + kb), block b = t*4 + s, lane (li, lg):
// W[c*64 + wsg_col(t, li)][kb*128 + 32 s + 8 lg + j], j < 8
__global__ void wsg_pack_kernel(int K, long n_pieces, const bf16* __restrict__ w, bf16* __restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pieces) return;
  const int NB = K / 128;
  const long slab = p / 1024;
  const int b = (int)((p / 64) % 16), L = (int)(p % 64), li = L & 15, lg = L >> 4;
  const int c = (int)(slab / NB), kb = (int)(slab % NB);
  const int t = b / 4, s = b % 4;
  const long n = (long)c * 64 + wsg_col(t, li);
  const int k0 = kb * 128 + 32 * s + 8 * lg;
  for (int j = 0; j < 8; ++j) out[p * 8 + j] = w[n * K + k0 + j];
}

template <int K, int NCH, int EPI>
static int launch_wsg(int64_t M, const void* A, const void* ws, void* out, long ldo, const WsEpi& e, hipStream_t s) {
  constexpr size_t lds = WsShape<K>::LDS;
  auto kern = wsg_kernel<K, NCH, EPI>;
  static bool attr = false;
  if (!attr) {
    SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(M, WS_ROWS)), dim3(512), lds, s, (int)M, (const bf16*)A,
                     (const char*)ws, (bf16*)out, ldo, e);
  SNV_LAUNCH_CHECK();
  return 0;
}

}  // namespace snvrag

using namespace snvrag;

// hap head (foundation_model.py:77-80): probs = softmax(act(A W^T + b) w_out^T + b_out),
// A [M, K], W packed by snvrag_wsg_pack (N hidden), w_out [2, N] f32
extern "C" int snvrag_wsg_head2(int64_t M, int64_t N, int64_t K, const void* A, const void* wstream,
                                const float* bias, int act, float slope, const float* w_out, const float* b_out,
                                float* logits, float* probs, void* stream) {
  SNV_CHECK_ARG(A && wstream && bias && w_out && b_out && probs, "null pointer");
  SNV_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)w_out % 16) == 0 && ((uintptr_t)bias % 16) == 0,
                "A/w_out/bias must be 16-byte aligned");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  WsEpi e{bias, act, slope, nullptr, 0, nullptr, nullptr, 0.f, w_out, b_out, logits, probs,
          nullptr, nullptr, nullptr, nullptr, 0};
  int rc = -1;
  evlog_begin(s);
  if (K == 384 && N == 1536) rc = launch_wsg<384, 24, 2>(M, A, wstream, nullptr, 0, e, s);
  else if (K == 256 && N == 1024) rc = launch_wsg<256, 16, 2>(M, A, wstream, nullptr, 0, e, s);
  else if (K == 128 && N == 512) rc = launch_wsg<128, 8, 2>(M, A, wstream, nullptr, 0, e, s);
  if (rc < 0) return fail(__func__, "unsupported (N, K) for the fused head");
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)N * (K + 2));
  return 0;
}

extern "C" size_t snvrag_wsg_pack_bytes(int64_t N, int64_t K) {
  if (N % 64 || (K != 128 && K != 256 && K != 384)) return 0;
  return (size_t)(N / 64) * (K / 128) * WS_SLAB;
}

extern "C" int snvrag_wsg_pack(int64_t N, int64_t K, const void* w, void* out, void* stream) {
  SNV_CHECK_ARG(w && out, "null pointer");
  const size_t bytes = snvrag_wsg_pack_bytes(N, K);
  SNV_CHECK_ARG(bytes > 0, "weight-streaming GEMM needs N % 64 == 0 and K in {128, 256, 384}");
  const long pieces = (long)(bytes / 16);
  hipLaunchKernelGGL(wsg_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), (int)K,
                     pieces, (const bf16*)w, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_wsg_forward(int64_t M, int64_t N, int64_t K, const void* A, const void* wstream,
                                  const float* bias, int act, float slope, const void* resid, int64_t ld_resid,
                                  const float* ln_g, const float* ln_b, float eps, const float* row1,
                                  const float* col1, const float* row2, const float* col2, int64_t row_period,
                                  void* out, int64_t ldo, void* stream) {
  SNV_CHECK_ARG(A && wstream && bias && out, "null pointer");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)wstream % 16) == 0 &&
                    ((uintptr_t)bias % 16) == 0 && ldo % 8 == 0,
                "A/out/wstream/bias must be 16-byte aligned, ldo % 8 == 0");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  SNV_CHECK_ARG((!row1 || (col1 && ((uintptr_t)col1 % 16) == 0)) && (!row2 || (col2 && ((uintptr_t)col2 % 16) == 0)),
                "row terms need 16-byte aligned column vectors");
  WsEpi e{bias, act, slope, (const bf16*)resid, (long)ld_resid, ln_g, ln_b, eps, nullptr, nullptr, nullptr, nullptr,
          row1, col1, row2, col2, (long)row_period};
  const bool ln = ln_g != nullptr;
  SNV_CHECK_ARG(!ln || (ln_b && resid && ld_resid % 8 == 0), "LayerNorm epilogue needs ln_b and a residual");
  evlog_begin(s);
  int rc = -1;
  if (ln) {
    if (K == 384 && N == 384) rc = launch_wsg<384, 6, 1>(M, A, wstream, out, ldo, e, s);
    else if (K == 256 && N == 256) rc = launch_wsg<256, 4, 1>(M, A, wstream, out, ldo, e, s);
    else if (K == 128 && N == 128) rc = launch_wsg<128, 2, 1>(M, A, wstream, out, ldo, e, s);
  } else {
    const int nc = (int)(N / 64);
    if (K == 384 && nc == 18) rc = launch_wsg<384, 18, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 384 && nc == 24) rc = launch_wsg<384, 24, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 384 && nc == 6) rc = launch_wsg<384, 6, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 256 && nc == 12) rc = launch_wsg<256, 12, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 256 && nc == 16) rc = launch_wsg<256, 16, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 256 && nc == 4) rc = launch_wsg<256, 4, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 128 && nc == 6) rc = launch_wsg<128, 6, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 128 && nc == 8) rc = launch_wsg<128, 8, 0>(M, A, wstream, out, ldo, e, s);
    else if (K == 128 && nc == 2) rc = launch_wsg<128, 2, 0>(M, A, wstream, out, ldo, e, s);
  }
  if (rc < 0) return fail(__func__, "unsupported (N, K) for the weight-streaming GEMM");
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)N * K);
  return 0;
}
