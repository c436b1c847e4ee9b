// LayerNorm (+ residual, + rag-fusion tail) and small elementwise kernels.
// One wave per row, 16-B vector loads, f32 statistics (two-pass on registers).
#include "common.h"

namespace snvrag {

constexpr int LN_MAX_CHUNKS = 8;   // per lane: 8 x 16 B -> N <= 4096 (bf16) / 2048 (f32)

template <typename T> struct Vec16;
template <> struct Vec16<float> { static constexpr int n = 4; };
template <> struct Vec16<bf16> { static constexpr int n = 8; };

template <typename T>
__device__ __forceinline__ void load16(const T* p, float* v) {
  const u32x4 raw = *reinterpret_cast<const u32x4*>(p);
  if constexpr (sizeof(T) == 4) {
    const f32x4 f = __builtin_bit_cast(f32x4, raw);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = f[j];
  } else {
    const bf16x8 b = __builtin_bit_cast(bf16x8, raw);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
  }
}

template <typename T>
__device__ __forceinline__ void store16(T* p, const float* v) {
  constexpr int n = Vec16<T>::n;
  T o[n];
#pragma unroll
  for (int j = 0; j < n; ++j) o[j] = from_f32<T>(v[j]);
  *reinterpret_cast<u32x4*>(p) = *reinterpret_cast<u32x4*>(o);
}

__device__ __forceinline__ float maf_weight(float af) {
  const float maf = fminf(af, 1.0f - af);
  return fminf(log1pf(1.0f / (maf + 1e-6f)), 3.0f);
}

struct LnPostDev {
  const void* base; long ld_base; float scale; const float* af; long af_period; int maf; int act;
};

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void layernorm_kernel(long M, int N, const TI* __restrict__ X, long ldx,
                                                        const TI* __restrict__ R, long ldr,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ b, float eps,
                                                        TO* __restrict__ Y, long ldy, LnPostDev post) {
  constexpr int VI = Vec16<TI>::n;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const int nch = N / VI;
  float v[LN_MAX_CHUNKS][VI];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < LN_MAX_CHUNKS; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      load16(X + row * ldx + ch * VI, v[c]);
      if (R) {
        float rr[VI];
        load16(R + row * ldr + ch * VI, rr);
#pragma unroll
        for (int j = 0; j < VI; ++j) v[c][j] += rr[j];
      }
#pragma unroll
      for (int j = 0; j < VI; ++j) s += v[c][j];
    }
  }
  const float mean = wave_sum(s) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < LN_MAX_CHUNKS; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < VI; ++j) { const float d = v[c][j] - mean; q += d * d; }
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)N + eps);
  float w = 1.0f;
  if (post.af && post.maf) {
    const long ar = post.af_period > 0 ? row % post.af_period : row;
    w = maf_weight(post.af[ar]);
  }
#pragma unroll
  for (int c = 0; c < LN_MAX_CHUNKS; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      const int n0 = ch * VI;
      float y[VI];
#pragma unroll
      for (int j = 0; j < VI; ++j) y[j] = apply_act(post.act, (v[c][j] - mean) * rstd * g[n0 + j] + b[n0 + j], 0.f);
      if constexpr (sizeof(TI) == sizeof(TO)) {   // post.base only allowed when TI == TO
        if (post.base) {
          float bb[VI];
          load16(reinterpret_cast<const TO*>(post.base) + row * post.ld_base + n0, bb);
#pragma unroll
          for (int j = 0; j < VI; ++j) y[j] = bb[j] + post.scale * (y[j] * w);
        }
      }
      if constexpr (sizeof(TI) == sizeof(TO)) {
        store16(Y + row * ldy + n0, y);
      } else {
#pragma unroll
        for (int j = 0; j < VI; ++j) Y[row * ldy + n0 + j] = from_f32<TO>(y[j]);
      }
    }
  }
}

// ------------------------------------------------------------------------ //
template <typename T>
__global__ void rag_concat_kernel(long M, int D, const T* __restrict__ q, const T* __restrict__ rag,
                                  const T* __restrict__ wgt, long period, T* __restrict__ out) {
  constexpr int V = Vec16<T>::n;
  const int cpr = D / V;
  const long total = M * cpr;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const long m = id / cpr;
    const int c = (int)(id % cpr) * V;
    const long mw = period > 0 ? m % period : m;
    float a[V], r[V], w[V];
    load16(q + m * D + c, a);
    load16(rag + m * D + c, r);
    load16(wgt + mw * D + c, w);
#pragma unroll
    for (int j = 0; j < V; ++j) r[j] *= w[j];
    store16(out + m * 2 * D + c, a);
    store16(out + m * 2 * D + D + c, r);
  }
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_layernorm(int dtype_in, int dtype_out, int64_t M, int64_t N, const void* X,
                                int64_t ldx, const void* R, int64_t ldr, const float* gamma,
                                const float* beta, float eps, void* Y, int64_t ldy,
                                const snvrag_ln_post_t* post, void* stream) {
  SNV_CHECK_ARG(X && Y && gamma && beta, "null pointer");
  const int vi = dtype_in == SNVRAG_BF16 ? 8 : 4;
  SNV_CHECK_ARG(N % vi == 0 && N / vi <= 64 * LN_MAX_CHUNKS, "N unsupported (multiple of 16 B, <= 4096 bf16 / 2048 f32)");
  SNV_CHECK_ARG(ldx % vi == 0 && (!R || ldr % vi == 0), "ld alignment");
  LnPostDev p{};
  if (post) {
    p.base = post->base; p.ld_base = post->ld_base; p.scale = post->scale;
    p.af = post->af; p.af_period = post->af_period; p.maf = post->maf_weight; p.act = post->act;
    SNV_CHECK_ARG(!p.base || dtype_in == dtype_out, "post.base requires dtype_in == dtype_out");
  }
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)cdiv(M, 4)), block(256);
  evlog_begin(s);
#define LN_CASE(TI, TO)                                                                        \
  hipLaunchKernelGGL((layernorm_kernel<TI, TO>), grid, block, 0, s, (long)M, (int)N,           \
                     (const TI*)X, (long)ldx, (const TI*)R, (long)ldr, gamma, beta, eps, (TO*)Y, \
                     (long)ldy, p)
  if (dtype_in == SNVRAG_BF16 && dtype_out == SNVRAG_BF16) LN_CASE(bf16, bf16);
  else if (dtype_in == SNVRAG_BF16) LN_CASE(bf16, float);
  else if (dtype_out == SNVRAG_F32) LN_CASE(float, float);
  else LN_CASE(float, bf16);
#undef LN_CASE
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_LN, (double)M * N * ((dtype_in == SNVRAG_BF16 ? 2 : 4) + (dtype_out == SNVRAG_BF16 ? 2 : 4)));
  return 0;
}

extern "C" int snvrag_rag_weighted_concat(int dtype, int64_t M, int64_t D, const void* q,
                                          const void* rag, const void* wgt, int64_t period,
                                          void* out, void* stream) {
  SNV_CHECK_ARG(q && rag && wgt && out, "null pointer");
  SNV_CHECK_ARG(D % 8 == 0, "D must be a multiple of 8");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int grid = (int)std::min<long>(cdiv(M * D / 4, 256), 8192);
  if (dtype == SNVRAG_BF16)
    hipLaunchKernelGGL(rag_concat_kernel<bf16>, dim3(grid), dim3(256), 0, s, (long)M, (int)D,
                       (const bf16*)q, (const bf16*)rag, (const bf16*)wgt, (long)period, (bf16*)out);
  else
    hipLaunchKernelGGL(rag_concat_kernel<float>, dim3(grid), dim3(256), 0, s, (long)M, (int)D,
                       (const float*)q, (const float*)rag, (const float*)wgt, (long)period, (float*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}
