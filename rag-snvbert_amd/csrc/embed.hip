// Embedding gather, AF Fourier features, position-feature conv chain, AF gate,
// hap/gt heads.  Memory-bound: 16-B vector loads/stores, one thread per 16-B
// output chunk (gathers) or one wave per row (dots).
#include "common.h"

namespace snvrag {

template <typename T> struct V16 { static constexpr int n = 16 / sizeof(T); };

template <typename T>
__device__ __forceinline__ void st16(T* p, const float* v) {
  constexpr int n = V16<T>::n;
  T o[n];
#pragma unroll
  for (int j = 0; j < n; ++j) o[j] = from_f32<T>(v[j]);
  *reinterpret_cast<u32x4*>(p) = *reinterpret_cast<u32x4*>(o);
}
template <typename T>
__device__ __forceinline__ void ld16(const T* p, float* v) {
  constexpr int n = V16<T>::n;
  const u32x4 raw = *reinterpret_cast<const u32x4*>(p);
  const T* t = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int j = 0; j < n; ++j) v[j] = to_f32(t[j]);
}

// ------------------------------------------------------- AF Fourier features --
// af_embedding.py:79-84: x = af*f (f32), angle = (2*pi) * x (f32), [sin | cos]
template <typename T>
__global__ void af_features_kernel(long M, const float* __restrict__ af, const float* __restrict__ fr,
                                   int nb, T* __restrict__ feat) {
  const long total = M * nb;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const long m = id / nb;
    const int j = (int)(id % nb);
    const float x = af[m] * fr[j];
    const float a = 6.283185307179586f * x;
    feat[m * 2 * nb + j] = from_f32<T>(sinf(a));
    feat[m * 2 * nb + nb + j] = from_f32<T>(cosf(a));
  }
}

// ----------------------------------------------------------- token embedding --
// embedding/bert.py:66-75: W[tok] + pe[:L] + afemb
template <typename T, typename TA>
__global__ void embed_tokens_kernel(long nseq, int L, int D, const int64_t* __restrict__ tok,
                                    const float* __restrict__ W, long vocab, const float* __restrict__ pe,
                                    const TA* __restrict__ afemb, long af_period, T* __restrict__ out) {
  constexpr int V = V16<T>::n;
  const int cpr = D / V;
  const long total = nseq * L * cpr;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const long row = id / cpr;
    const int c = (int)(id % cpr) * V;
    const long s = row / L;
    const int l = (int)(row % L);
    long t = tok[row];
    t = t < 0 ? 0 : (t >= vocab ? vocab - 1 : t);
    float v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = W[t * D + c + j] + pe[(long)l * D + c + j];
    if (afemb) {
      const long ar = (af_period > 0 ? s % af_period : s) * L + l;
      float a[V16<TA>::n > V ? V16<TA>::n : V];
      if constexpr (sizeof(TA) == sizeof(T)) {
        ld16(afemb + ar * D + c, a);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) a[j] = to_f32(afemb[ar * D + c + j]);
      }
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] += a[j];
    }
    st16(out + row * D + c, v);
  }
}

// ----------------------------------------------------------- position feature --
// fusion.py:326-332.  One block per sequence; the three k=9 convs run out of LDS.
__global__ __launch_bounds__(256) void posfeat_kernel(int L, const float* __restrict__ pos,
                                                      snvrag_posfeat_w_t w, float* __restrict__ out) {
  extern __shared__ float sh[];
  float* x0 = sh;                 // [L + 8]
  float* x1 = x0 + (L + 8);       // [4][L + 8]
  float* x2 = x1 + 4 * (L + 8);   // [4][L + 8]
  const int b = blockIdx.x, tid = threadIdx.x;
  const int LP = L + 8;
  for (int i = tid; i < LP; i += blockDim.x) {
    const int l = i - 4;
    x0[i] = (l >= 0 && l < L) ? pos[(long)b * L + l] : 0.f;
  }
  for (int i = tid; i < 4 * LP; i += blockDim.x) { x1[i] = 0.f; x2[i] = 0.f; }
  __syncthreads();
  for (int l = tid; l < L; l += blockDim.x) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a = w.c1_b[c];
#pragma unroll
      for (int j = 0; j < 9; ++j) a = fmaf(w.c1_w[c * 9 + j], x0[l + j], a);
      a = a >= 0.f ? a : 0.05f * a;
      a = (a - w.bn1_rm[c]) / sqrtf(w.bn1_rv[c] + w.bn_eps) * w.bn1_w[c] + w.bn1_b[c];
      x1[c * LP + l + 4] = a;
    }
  }
  __syncthreads();
  for (int l = tid; l < L; l += blockDim.x) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a = w.c2_b[c];
      for (int ci = 0; ci < 4; ++ci)
#pragma unroll
        for (int j = 0; j < 9; ++j) a = fmaf(w.c2_w[(c * 4 + ci) * 9 + j], x1[ci * LP + l + j], a);
      a = a >= 0.f ? a : 0.05f * a;
      a = (a - w.bn2_rm[c]) / sqrtf(w.bn2_rv[c] + w.bn_eps) * w.bn2_w[c] + w.bn2_b[c];
      x2[c * LP + l + 4] = a;
    }
  }
  __syncthreads();
  for (int l = tid; l < L; l += blockDim.x) {
    float a = w.c3_b[0];
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int j = 0; j < 9; ++j) a = fmaf(w.c3_w[ci * 9 + j], x2[ci * LP + l + j], a);
    out[(long)b * L + l] = a >= 0.f ? a : 0.05f * a;
  }
}

// ------------------------------------------------------------------- AF gate --
// fusion.py:82-86: gate = sigmoid(W2 gelu(W1 c + b1) + b2), enc = gelu(LN(Wj c + bj)),
// out = af + rs * gate * enc.  One lane per row (AF_R rows per lane).
// Lane-per-row layout: the 32 gate hiddens of AF_R rows sit in the lane's VGPRs and the
// per-column weights (g2_w row, j_w, LN affine) are wave-uniform scalar loads shared by those
// rows, so the [D x 32] gate GEMV costs 32 v_fma per element with no cross-lane traffic.
constexpr int AF_R = 1;                 // rows per lane (4: 555 vs 304 us, occupancy 2 vs 4 waves/SIMD)
template <typename T>
__global__ __launch_bounds__(256) void af_gate_kernel(long M, int D, const float* __restrict__ af,
                                                      const float* __restrict__ afp, snvrag_afgate_w_t w,
                                                      T* __restrict__ out) {
  constexpr int V = 16 / sizeof(T);
  // 64 AF_R rows per workgroup (lane l: rows base + l + 64 r); its 4 waves split the D columns
  const long base = (long)blockIdx.x * 64 * AF_R + (threadIdx.x & 63);
  const int cpw = ((D / V + 3) / 4) * V;
  const int c_lo = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * cpw);
  const int c_hi = min(D, c_lo + cpw);
  // joint_encoder[0] is affine in (af, af_p): enc_n = j0_n a0 + j1_n a1 + jb_n, so its LayerNorm
  // statistics are mean = mu . (a0, a1, 1) and var = (a0, a1, 1) S (a0, a1, 1)^T with the
  // centred second moments S of the weight columns — reduced once per workgroup (two passes)
  // instead of two D-long loops per row
  __shared__ float red[4][6];
  const int wv = threadIdx.x >> 6;
  float m0 = 0.f, m1 = 0.f, mb = 0.f;
  for (int n = threadIdx.x; n < D; n += 256) {
    m0 += w.j_w[n * 2];
    m1 += w.j_w[n * 2 + 1];
    mb += w.j_b[n];
  }
  m0 = wave_sum(m0);
  m1 = wave_sum(m1);
  mb = wave_sum(mb);
  if ((threadIdx.x & 63) == 0) { red[wv][0] = m0; red[wv][1] = m1; red[wv][2] = mb; }
  __syncthreads();
  m0 = (red[0][0] + red[1][0] + red[2][0] + red[3][0]) / D;
  m1 = (red[0][1] + red[1][1] + red[2][1] + red[3][1]) / D;
  mb = (red[0][2] + red[1][2] + red[2][2] + red[3][2]) / D;
  __syncthreads();
  float sm[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};                // S00 S11 S01 S0b S1b Sbb
  for (int n = threadIdx.x; n < D; n += 256) {
    const float c0 = w.j_w[n * 2] - m0, c1 = w.j_w[n * 2 + 1] - m1, cb = w.j_b[n] - mb;
    sm[0] += c0 * c0;
    sm[1] += c1 * c1;
    sm[2] += c0 * c1;
    sm[3] += c0 * cb;
    sm[4] += c1 * cb;
    sm[5] += cb * cb;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    sm[i] = wave_sum(sm[i]);
    if ((threadIdx.x & 63) == 0) red[wv][i] = sm[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 6; ++i) sm[i] = (red[0][i] + red[1][i] + red[2][i] + red[3][i]) / D;
  float a0[AF_R], a1[AF_R], mean[AF_R], rstd[AF_R], hid[AF_R][32];
#pragma unroll
  for (int r = 0; r < AF_R; ++r) {
    const long m = base + 64 * r;
    const bool ok = m < M;
    a0[r] = ok ? af[m] : 0.f;
    a1[r] = ok ? afp[m] : 0.f;
    mean[r] = m0 * a0[r] + m1 * a1[r] + mb;
    const float var = a0[r] * a0[r] * sm[0] + a1[r] * a1[r] * sm[1] +
                      2.f * (a0[r] * a1[r] * sm[2] + a0[r] * sm[3] + a1[r] * sm[4]) + sm[5];
    rstd[r] = 1.0f / sqrtf(fmaxf(var, 0.f) + 1e-5f);
#pragma unroll
    for (int u = 0; u < 32; ++u)
      hid[r][u] = gelu_erf(w.g1_w[u * 2] * a0[r] + w.g1_w[u * 2 + 1] * a1[r] + w.g1_b[u]);
  }
  for (int n0 = c_lo; n0 < c_hi; n0 += V) {
    T o[AF_R][V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int n = n0 + j;
      float g[AF_R];
#pragma unroll
      for (int r = 0; r < AF_R; ++r) g[r] = w.g2_b[n];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const float wu = w.g2_w[n * 32 + u];
#pragma unroll
        for (int r = 0; r < AF_R; ++r) g[r] = fmaf(wu, hid[r][u], g[r]);
      }
      const float j0 = w.j_w[n * 2], j1 = w.j_w[n * 2 + 1], jb = w.j_b[n], lw = w.ln_w[n], lb = w.ln_b[n];
#pragma unroll
      for (int r = 0; r < AF_R; ++r) {
        const float gt = 1.0f / (1.0f + expf(-g[r]));
        const float enc = j0 * a0[r] + j1 * a1[r] + jb;
        const float e = gelu_erf((enc - mean[r]) * rstd[r] * lw + lb);
        o[r][j] = from_f32<T>(a0[r] + w.res_scale * (gt * e));
      }
    }
#pragma unroll
    for (int r = 0; r < AF_R; ++r) {
      const long m = base + 64 * r;
      if (m < M) *reinterpret_cast<u32x4*>(out + m * D + n0) = *reinterpret_cast<u32x4*>(o[r]);
    }
  }
}

// --------------------------------------------------------------- hap head out --
// foundation_model.py:77-80: Linear(4D -> 2) then softmax.  One wave per row.
template <typename T>
__global__ __launch_bounds__(256) void hap_out_kernel(long M, int K, const T* __restrict__ H, long ldh,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      float* __restrict__ logits, float* __restrict__ probs) {
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  constexpr int V = V16<T>::n;
  float s0 = 0.f, s1 = 0.f;
  for (int c = lane * V; c < K; c += 64 * V) {
    float h[V];
    ld16(H + m * ldh + c, h);
#pragma unroll
    for (int j = 0; j < V; ++j) { s0 = fmaf(h[j], w[c + j], s0); s1 = fmaf(h[j], w[K + c + j], s1); }
  }
  s0 = wave_sum(s0) + b[0];
  s1 = wave_sum(s1) + b[1];
  if (lane == 0) {
    if (logits) { logits[2 * m] = s0; logits[2 * m + 1] = s1; }
    const float mx = fmaxf(s0, s1);
    const float e0 = expf(s0 - mx), e1 = expf(s1 - mx);
    probs[2 * m] = e0 / (e0 + e1);
    probs[2 * m + 1] = e1 / (e0 + e1);
  }
}

// ----------------------------------------------------------------- gt head --
// foundation_model.py:159-176: Linear(7,16) -> LeakyReLU(0.01) -> LN(16) ->
// FeedForward(16,16) -> Linear(16,4) -> softmax.  One thread per position.
__device__ __forceinline__ void ln16(float* x, const float* g, const float* b) {
  float mu = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) mu += x[i];
  mu *= (1.0f / 16);
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) { const float d = x[i] - mu; var += d * d; }
  const float r = 1.0f / sqrtf(var * (1.0f / 16) + 1e-5f);
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = (x[i] - mu) * r * g[i] + b[i];
}

__global__ __launch_bounds__(256) void gt_head_kernel(long M, const float* __restrict__ p1, const float* __restrict__ p2,
                                                      const float* __restrict__ ref, const float* __restrict__ het,
                                                      const float* __restrict__ hom, long period,
                                                      snvrag_gt_w_t w, float* __restrict__ out) {
  __shared__ float sw[16 * 7 + 16 * 4 + 16 * 16 * 2 + 16 * 4 + 4 + 16 * 4];
  // stage weights once per block
  float* fw = sw;            float* fb = fw + 112;     float* nw = fb + 16;  float* nb = nw + 16;
  float* w1 = nb + 16;       float* b1 = w1 + 256;     float* lw = b1 + 16;  float* lb = lw + 16;
  float* w2 = lb + 16;       float* b2 = w2 + 256;     float* cw = b2 + 16;  float* cb = cw + 64;
  for (int i = threadIdx.x; i < 112; i += blockDim.x) fw[i] = w.f_w[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) { w1[i] = w.w1[i]; w2[i] = w.w2[i]; }
  for (int i = threadIdx.x; i < 64; i += blockDim.x) cw[i] = w.c_w[i];
  for (int i = threadIdx.x; i < 16; i += blockDim.x) {
    fb[i] = w.f_b[i]; nw[i] = w.n_w[i]; nb[i] = w.n_b[i]; b1[i] = w.b1[i];
    lw[i] = w.ln_w[i]; lb[i] = w.ln_b[i]; b2[i] = w.b2[i];
  }
  for (int i = threadIdx.x; i < 4; i += blockDim.x) cb[i] = w.c_b[i];
  __syncthreads();
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const long mr = period > 0 ? m % period : m;
  const float in[7] = {p1[2 * m], p1[2 * m + 1], p2[2 * m], p2[2 * m + 1], ref[mr], het[mr], hom[mr]};
  float x[16], y[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) {
    float a = fb[o];
#pragma unroll
    for (int i = 0; i < 7; ++i) a = fmaf(fw[o * 7 + i], in[i], a);
    x[o] = a >= 0.f ? a : 0.01f * a;
  }
  ln16(x, nw, nb);
#pragma unroll
  for (int o = 0; o < 16; ++o) {
    float a = b1[o];
#pragma unroll
    for (int i = 0; i < 16; ++i) a = fmaf(w1[o * 16 + i], x[i], a);
    y[o] = a >= 0.f ? a : 0.1f * a;
  }
  ln16(y, lw, lb);
#pragma unroll
  for (int o = 0; o < 16; ++o) {
    float a = b2[o];
#pragma unroll
    for (int i = 0; i < 16; ++i) a = fmaf(w2[o * 16 + i], y[i], a);
    x[o] = a >= 0.f ? a : 0.1f * a;
  }
  float lg[4], mx = -INFINITY;
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    float a = cb[o];
#pragma unroll
    for (int i = 0; i < 16; ++i) a = fmaf(cw[o * 16 + i], x[i], a);
    lg[o] = a;
    mx = fmaxf(mx, a);
  }
  float se = 0.f;
#pragma unroll
  for (int o = 0; o < 4; ++o) { lg[o] = expf(lg[o] - mx); se += lg[o]; }
#pragma unroll
  for (int o = 0; o < 4; ++o) out[4 * m + o] = lg[o] / se;
}

static int grid_for(long work, int per = 256, int cap = 65536) {
  long g = (work + per - 1) / per;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_af_features(int dtype_out, int64_t M, const float* af, const float* freqs, int nb,
                                  void* feat, void* stream) {
  SNV_CHECK_ARG(af && freqs && feat && nb > 0, "bad args");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  if (dtype_out == SNVRAG_BF16)
    hipLaunchKernelGGL(af_features_kernel<bf16>, dim3(grid_for(M * nb)), dim3(256), 0, s, (long)M, af, freqs, nb, (bf16*)feat);
  else
    hipLaunchKernelGGL(af_features_kernel<float>, dim3(grid_for(M * nb)), dim3(256), 0, s, (long)M, af, freqs, nb, (float*)feat);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_embed_tokens(int dtype_out, int64_t nseq, int64_t L, int64_t D, const int64_t* tok,
                                   const float* W, int64_t vocab, const float* pe, const void* afemb,
                                   int afemb_dtype, int64_t af_period, void* out, void* stream) {
  SNV_CHECK_ARG(tok && W && pe && out, "null pointer");
  SNV_CHECK_ARG(D % 8 == 0, "D must be a multiple of 8");
  if (nseq == 0) return 0;
  hipStream_t s = as_stream(stream);
  const long work = nseq * L * D / (dtype_out == SNVRAG_BF16 ? 8 : 4);
#define EMB_CASE(T, TA)                                                                            \
  hipLaunchKernelGGL((embed_tokens_kernel<T, TA>), dim3(grid_for(work)), dim3(256), 0, s, (long)nseq, \
                     (int)L, (int)D, tok, W, (long)vocab, pe, (const TA*)afemb, (long)af_period, (T*)out)
  if (dtype_out == SNVRAG_BF16) {
    if (afemb_dtype == SNVRAG_BF16) EMB_CASE(bf16, bf16); else EMB_CASE(bf16, float);
  } else {
    if (afemb_dtype == SNVRAG_BF16) EMB_CASE(float, bf16); else EMB_CASE(float, float);
  }
#undef EMB_CASE
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_posfeat(int64_t B, int64_t L, const float* pos, const snvrag_posfeat_w_t* w,
                              float* out, void* stream) {
  SNV_CHECK_ARG(pos && w && out, "null pointer");
  if (B == 0) return 0;
  const size_t sh = (size_t)(L + 8) * 9 * sizeof(float);
  SNV_CHECK_ARG(sh <= 160 * 1024, "sequence too long for LDS");
  hipLaunchKernelGGL(posfeat_kernel, dim3((unsigned)B), dim3(256), sh, as_stream(stream), (int)L, pos, *w, out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_af_gate(int dtype_out, int64_t M, int64_t D, const float* af, const float* af_p,
                              const snvrag_afgate_w_t* w, void* out, void* stream) {
  SNV_CHECK_ARG(af && af_p && w && out, "null pointer");
  SNV_CHECK_ARG(D % 8 == 0, "D % 8");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  if (dtype_out == SNVRAG_BF16)
    hipLaunchKernelGGL(af_gate_kernel<bf16>, dim3(cdiv(M, 64 * AF_R)), dim3(256), 0, s, (long)M, (int)D, af, af_p, *w,
                       (bf16*)out);
  else
    hipLaunchKernelGGL(af_gate_kernel<float>, dim3(cdiv(M, 64 * AF_R)), dim3(256), 0, s, (long)M, (int)D, af, af_p, *w,
                       (float*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_hap_head_out(int dtype_in, int64_t M, int64_t K, const void* H, int64_t ldh,
                                   const float* w, const float* b, float* logits, float* probs, void* stream) {
  SNV_CHECK_ARG(H && w && b && probs, "null pointer");
  SNV_CHECK_ARG(K % 8 == 0 && ldh % 8 == 0, "K/ldh must be multiples of 8");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  if (dtype_in == SNVRAG_BF16)
    hipLaunchKernelGGL(hap_out_kernel<bf16>, dim3(cdiv(M, 4)), dim3(256), 0, s, (long)M, (int)K, (const bf16*)H, (long)ldh, w, b, logits, probs);
  else
    hipLaunchKernelGGL(hap_out_kernel<float>, dim3(cdiv(M, 4)), dim3(256), 0, s, (long)M, (int)K, (const float*)H, (long)ldh, w, b, logits, probs);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_gt_head(int64_t M, const float* p1, const float* p2, const float* ref, const float* het,
                              const float* hom, int64_t period, const snvrag_gt_w_t* w, float* out, void* stream) {
  SNV_CHECK_ARG(p1 && p2 && ref && het && hom && w && out, "null pointer");
  if (M == 0) return 0;
  hipLaunchKernelGGL(gt_head_kernel, dim3(cdiv(M, 256)), dim3(256), 0, as_stream(stream), (long)M, p1, p2,
                     ref, het, hom, (long)period, *w, out);
  SNV_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------- infer post-process --
// infer_embedding_rag.py:145-152: the heads' probabilities go through softmax AGAIN,
// p = softmax(probs)[..., 1]; gt = [(1-p1)(1-p2), (1-p1)p2, p1(1-p2), p1 p2].
__global__ __launch_bounds__(256) void infer_post_kernel(long M, const float* __restrict__ ph1,
                                                         const float* __restrict__ ph2, float* __restrict__ p1o,
                                                         float* __restrict__ p2o, float* __restrict__ gt) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  auto p_alt = [](float a, float b) {          // softmax([a, b])[1]
    const float mx = fmaxf(a, b), ea = expf(a - mx), eb = expf(b - mx);
    return eb / (ea + eb);
  };
  const float p1 = p_alt(ph1[2 * m], ph1[2 * m + 1]), p2 = p_alt(ph2[2 * m], ph2[2 * m + 1]);
  p1o[m] = p1;
  p2o[m] = p2;
  f32x4 g;
  g[0] = (1.f - p1) * (1.f - p2);
  g[1] = (1.f - p1) * p2;
  g[2] = p1 * (1.f - p2);
  g[3] = p1 * p2;
  reinterpret_cast<f32x4*>(gt)[m] = g;
}

extern "C" int snvrag_infer_post(int64_t M, const float* probs_h1, const float* probs_h2, float* p1, float* p2,
                                 float* gt, void* stream) {
  SNV_CHECK_ARG(probs_h1 && probs_h2 && p1 && p2 && gt && ((uintptr_t)gt % 16) == 0, "null or misaligned pointer");
  if (M == 0) return 0;
  hipLaunchKernelGGL(infer_post_kernel, dim3(cdiv(M, 256)), dim3(256), 0, as_stream(stream), (long)M, probs_h1,
                     probs_h2, p1, p2, gt);
  SNV_LAUNCH_CHECK();
  return 0;
}
