// Training-step kernels (gfx950): focal loss forward+backward, gradient norm, fused
// Adam with gradient clipping and the bf16 compute-weight mirror, and the per-class
// confusion counts of the trainer's metrics.
//
//   focal   : FocalLoss.forward (main/optim_schedule.py:64-96) over the masked rows
//             (pretrain_with_val_optimized.py:215-217, reduction='sum'), fused with its
//             derivative.  Like the reference, the "inputs" are the heads' softmax
//             PROBABILITIES and FocalLoss applies softmax to them again.
//   sqnorm  : sum of squares of the flat gradient buffer (torch.nn.utils.clip_grad_norm_).
//   adam    : torch.optim.Adam (L2 weight decay added to the gradient, bias-corrected
//             moments; pretrain_with_val_optimized.py:73-74, :238-245) over ONE flat f32
//             parameter buffer, with the clip coefficient computed on the device from
//             sqnorm (no host round trip) and a bf16 copy of the updated parameters
//             written for the next step's MFMA GEMMs.
//   confusion: cal_pr (optim_schedule.py:167-203) as device counters (no per-batch D2H).
#include "common.h"

#include <cstdlib>
#include "attn_common.h"

#include <cmath>

namespace snvrag {

__global__ __launch_bounds__(256) void focal_kernel(long M, int C, const float* __restrict__ probs,
                                                    const int64_t* __restrict__ labels,
                                                    const uint8_t* __restrict__ mask, float gamma, float weight,
                                                    float* __restrict__ loss_sum, float* __restrict__ grad) {
  __shared__ float red[4];
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  float l = 0.f;
  if (m < M) {
    float x[4], s[4];
    float mx = -INFINITY;
    for (int j = 0; j < C; ++j) { x[j] = probs[m * C + j]; mx = fmaxf(mx, x[j]); }
    float z = 0.f;
    for (int j = 0; j < C; ++j) { s[j] = expf(x[j] - mx); z += s[j]; }
    for (int j = 0; j < C; ++j) s[j] /= z;
    const int y = (int)labels[m];
    const bool on = mask[m] != 0 && y >= 0 && y < C;
    if (on) {
      const float pt = s[y], q = 1.f - pt, lp = logf(pt + 1e-10f);
      const float qg = powf(q, gamma);
      l = -qg * lp * weight;
      // dL/dp_t, then dp_t/dx_j = p_t (delta_jy - s_j)
      const float dpt = (gamma != 0.f ? gamma * powf(q, gamma - 1.f) * lp : 0.f) - qg / (pt + 1e-10f);
      for (int j = 0; j < C; ++j) grad[m * C + j] = weight * dpt * pt * ((j == y ? 1.f : 0.f) - s[j]);
    } else {
      for (int j = 0; j < C; ++j) grad[m * C + j] = 0.f;
    }
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss_sum, red[0] + red[1] + red[2] + red[3]);
}

// Two passes with a fixed summation order (no float atomics): every rank of a data-parallel
// job holds the same reduced gradient and must derive the same clip coefficient bit for bit,
// or the replicas drift apart after the first optimizer step.
constexpr int kSqBlocks = 2048;
// the partials of snvrag_sqnorm (no workspace: one call in flight per device, stream-ordered);
// snvrag_sqnorm_ws takes the caller's buffer, so calls on different streams do not share it
__device__ float g_sq_partials[kSqBlocks];

__global__ __launch_bounds__(256) void sqnorm_kernel(long n, const float* __restrict__ x, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += 256) s += x[i] * x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) (part ? part : g_sq_partials)[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void sqnorm_final_kernel(int nblocks, const float* __restrict__ part,
                                                           float* __restrict__ acc) {
  __shared__ float red[4];
  float s = 0.f;
  const float* pp = part ? part : g_sq_partials;
  for (int i = threadIdx.x; i < nblocks; i += 256) s += pp[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *acc = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void adam_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16* __restrict__ pb, const float* __restrict__ sqnorm,
                                                   snvrag_adam_t a) {
  float coef = a.grad_scale;
  if (sqnorm && a.max_norm > 0.f) {
    const float norm = sqrtf(*sqnorm) * a.grad_scale;
    const float c = a.max_norm / (norm + 1e-6f);
    coef *= fminf(c, 1.f);
  }
  const float bc1 = 1.f - powf(a.beta1, (float)a.step), bc2 = 1.f - powf(a.beta2, (float)a.step);
  const float step_size = a.lr / bc1, rbc2 = 1.f / sqrtf(bc2);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float pi = p[i];
    const float gi = g[i] * coef + a.weight_decay * pi;
    const float mi = a.beta1 * m[i] + (1.f - a.beta1) * gi;
    const float vi = a.beta2 * v[i] + (1.f - a.beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float np = pi - step_size * mi / (sqrtf(vi) * rbc2 + a.eps);
    p[i] = np;
    if (pb) pb[i] = (bf16)np;
  }
}

__global__ __launch_bounds__(256) void confusion_kernel(long M, int C, const float* __restrict__ probs,
                                                        const int64_t* __restrict__ labels,
                                                        const uint8_t* __restrict__ mask,
                                                        const uint8_t* __restrict__ mask2,
                                                        unsigned long long* __restrict__ out) {
  __shared__ unsigned int cnt[3 * 8];
  if (threadIdx.x < 3 * 8) cnt[threadIdx.x] = 0;
  __syncthreads();
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  if (m < M && mask[m] && (!mask2 || mask2[m])) {
    int am = 0;
    float best = probs[m * C];
    for (int j = 1; j < C; ++j) {
      const float x = probs[m * C + j];
      if (x > best) { best = x; am = j; }
    }
    const int y = (int)labels[m];
    if (am == y) atomicAdd(&cnt[am], 1u);                 // tp
    else {
      atomicAdd(&cnt[8 + am], 1u);                          // fp of the predicted class
      if (y >= 0 && y < C) atomicAdd(&cnt[16 + y], 1u);     // fn of the true class
    }
  }
  __syncthreads();
  if (threadIdx.x < 3 * C) {
    const int kind = threadIdx.x / C, c = threadIdx.x % C;
    const unsigned int v = cnt[kind * 8 + c];
    if (v) atomicAdd(&out[kind * C + c], (unsigned long long)v);
  }
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_focal_loss(int64_t M, int C, const float* probs, const int64_t* labels, const uint8_t* mask,
                                 float gamma, float weight, float* loss_sum, float* grad, void* stream) {
  SNV_CHECK_ARG(probs && labels && mask && loss_sum && grad, "null pointer");
  SNV_CHECK_ARG(C >= 1 && C <= 4, "classes must be 1..4");
  if (M == 0) return 0;
  hipLaunchKernelGGL(focal_kernel, dim3(cdiv(M, 256)), dim3(256), 0, as_stream(stream), (long)M, C, probs, labels,
                     mask, gamma, weight, loss_sum, grad);
  SNV_LAUNCH_CHECK();
  return 0;
}

static int sqnorm_impl(int64_t n, const float* x, float* acc, float* part, hipStream_t s) {
  SNV_CHECK_ARG(x && acc && ((uintptr_t)x % 16) == 0, "null or misaligned pointer");
  if (n == 0) {
    SNV_HIP(hipMemsetAsync(acc, 0, sizeof(float), s));
    return 0;
  }
  const int grid = (int)std::min<long>(cdiv(n / 4 + 1, 256), kSqBlocks);
  hipLaunchKernelGGL(sqnorm_kernel, dim3(grid), dim3(256), 0, s, (long)n, x, part);
  SNV_LAUNCH_CHECK();
  hipLaunchKernelGGL(sqnorm_final_kernel, dim3(1), dim3(256), 0, s, grid, (const float*)part, acc);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_sqnorm(int64_t n, const float* x, float* acc, void* stream) {
  return sqnorm_impl(n, x, acc, nullptr, as_stream(stream));
}

extern "C" size_t snvrag_sqnorm_ws_bytes(void) { return kSqBlocks * sizeof(float); }

extern "C" int snvrag_sqnorm_ws(int64_t n, const float* x, float* acc, float* ws, size_t ws_bytes, void* stream) {
  SNV_CHECK_ARG(ws && ws_bytes >= kSqBlocks * sizeof(float), "workspace smaller than snvrag_sqnorm_ws_bytes()");
  return sqnorm_impl(n, x, acc, ws, as_stream(stream));
}

extern "C" int snvrag_adam_step(int64_t n, float* p, const float* g, float* m, float* v, void* p_bf16,
                                const float* sqnorm, const snvrag_adam_t* a, void* stream) {
  SNV_CHECK_ARG(p && g && m && v && a, "null pointer");
  SNV_CHECK_ARG(a->step >= 1, "step counts from 1");
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int grid = (int)std::min<long>(cdiv(n, 256), 8192);
  evlog_begin(s);
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, s, (long)n, p, g, m, v, (bf16*)p_bf16, sqnorm, *a);
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_TRAIN, (double)n * (4 * 4 + 3 * 4 + (p_bf16 ? 2 : 0)));   // bytes moved
  return 0;
}

extern "C" int snvrag_confusion(int64_t M, int C, const float* probs, const int64_t* labels, const uint8_t* mask,
                                const uint8_t* mask2, uint64_t* counts, void* stream) {
  SNV_CHECK_ARG(probs && labels && mask && counts, "null pointer");
  SNV_CHECK_ARG(C >= 1 && C <= 8, "classes must be 1..8");
  if (M == 0) return 0;
  hipLaunchKernelGGL(confusion_kernel, dim3(cdiv(M, 256)), dim3(256), 0, as_stream(stream), (long)M, C, probs,
                     labels, mask, mask2, (unsigned long long*)counts);
  SNV_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------- LayerNorm (training) --
// y = LN(x + r) * g + b over rows of N (sublayer.py:15-16 / nn.LayerNorm), bf16 in/out,
// f32 statistics.  Forward keeps s = x + r (bf16, only when r is given) and (mean, rstd)
// per row for the backward:
//   xh = (s - mean) * rstd,  gy = dy * g
//   ds = rstd * (gy - mean_n(gy) - xh * mean_n(gy * xh))       (= dx = dr)
//   dg = sum_rows dy * xh,  db = sum_rows dy                   (per-block partials)
// One wave per row, lanes over 8-column chunks.
namespace snvrag {
constexpr int LN_MAXC = 4;   // 8-col chunks per lane: N <= 64 * 8 * 4 = 2048
constexpr int LN_BWD_RPW = 8;  // rows per wave of ln_bwd (up to 2048 blocks)

__device__ __forceinline__ void ld8bf(const bf16* p, float* v) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(a[e] << 16);
    v[2 * e + 1] = __uint_as_float(a[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8bf(bf16* p, const float* v) {
  bf16x8 a;
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = (bf16)v[e];
  *reinterpret_cast<bf16x8*>(p) = a;
}

// Element dropout fused into the LayerNorm kernels (the SublayerConnection / TransformerBlock
// dropouts around the norms, transformer.py / sublayer.py): keep (m, n) iff half (n & 1) of
// mix24(base + m * C1 + (n >> 1) * C2) >= thresh, base = drop_base(seed, stream) with stream 0
// for the residual operand r and 1 for the output (attn_common.h's hash over (row, column)).
// sl_x / sl_r: LeakyReLU slopes applied to the input x (no residual) / to the residual operand r
// BEFORE its dropout (0: none) — the FeedForward's activations (feed_forward.py:20-21) fused into
// the LayerNorm kernels instead of separate elementwise passes; sign(LeakyReLU(v)) = sign(v), so
// the backward's derivative comes from the saved pre-activation.
struct LnDrop {
  uint32_t th_r, th_o;          // round(p * 2^16); 0: off
  float sc_r, sc_o;             // 1 / (1 - p)
  uint32_t base_r, base_o;
  float sl_x, sl_r;
};
static LnDrop make_ln_drop(float p_r, float p_o, uint64_t seed, float sl_x = 0.f, float sl_r = 0.f) {
  const AttnDrop a = make_attn_drop(p_r, seed), b = make_attn_drop(p_o, seed);
  return LnDrop{a.thresh, b.thresh, a.scale, b.scale, drop_base(seed, 0u), drop_base(seed, 1u), sl_x, sl_r};
}
__device__ __forceinline__ float ln_lrelu(float v, float sl) { return v > 0.f ? v : v * sl; }
// multipliers of the 8 columns 8 cc .. 8 cc + 7 of row m: 4 hashes
__device__ __forceinline__ void ln_drop8(uint32_t base, uint32_t th, float sc, long m, int cc, float (&mk)[8]) {
  const uint32_t row = base + (uint32_t)m * DROP_C1 + (uint32_t)(4 * cc) * DROP_C2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t h = drop_mix24(row + (uint32_t)i * DROP_C2);
    mk[2 * i] = (h & 0xFFFFu) >= th ? sc : 0.f;
    mk[2 * i + 1] = (h >> 16) >= th ? sc : 0.f;
  }
}

template <int NC>
__global__ __launch_bounds__(256) void ln_fwd_train_kernel(long M, int N, const bf16* __restrict__ x,
                                                           const bf16* __restrict__ r, const float* __restrict__ g,
                                                           const float* __restrict__ b, float eps,
                                                           bf16* __restrict__ y, bf16* __restrict__ s_out,
                                                           float2* __restrict__ stats, LnDrop dr) {
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  const int nc = N / 8;
  float v[NC][8];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cc = lane + 64 * c;
    if (cc < nc) {
      ld8bf(x + m * N + 8 * cc, v[c]);
      if (dr.sl_x != 0.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (float)(bf16)ln_lrelu(v[c][j], dr.sl_x);
      }
      if (r) {
        float t[8];
        ld8bf(r + m * N + 8 * cc, t);
        if (dr.sl_r != 0.f) {
#pragma unroll
          for (int j = 0; j < 8; ++j) t[j] = (float)(bf16)ln_lrelu(t[j], dr.sl_r);
        }
        if (dr.th_r) {
          float mk[8];
          ln_drop8(dr.base_r, dr.th_r, dr.sc_r, m, cc, mk);
#pragma unroll
          for (int j = 0; j < 8; ++j) t[j] *= mk[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (float)(bf16)(v[c][j] + t[j]);   // s is kept in bf16
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[c][j];
    }
  }
  const float mean = wave_sum(sum) / N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (lane + 64 * c < nc)
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[c][j] - mean; q += d * d; }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cc = lane + 64 * c;
    if (cc < nc) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * g[8 * cc + j] + b[8 * cc + j];
      if (dr.th_o) {
        float mk[8];
        ln_drop8(dr.base_o, dr.th_o, dr.sc_o, m, cc, mk);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] *= mk[j];
      }
      st8bf(y + m * N + 8 * cc, o);
      if (s_out) st8bf(s_out + m * N + 8 * cc, v[c]);
    }
  }
  if (lane == 0) stats[m] = make_float2(mean, rstd);
}

// RPB rows per block (one wave each, looping): the block's dg/db partials go to
// part[blockIdx.x][2][N].  Output dropout: dy is masked on load; residual dropout: dr = ds
// masked (the gradient of r), written next to ds.
// sl_x: s is the PRE-activation input x (y = LN(lrelu(x))), the normalised value is rebuilt as
// lrelu(s) and ds carries the activation's derivative; sl_r: rp is the pre-activation residual r
// and dres = ds o mask o lrelu'(r) (always written).
// NC 8-column chunks per lane (N <= 512 NC * ... : the register arrays sized to the row), and every
// wave steps through its rows TWO at a time so the two rows' loads and wave reductions overlap
// (a row alone is latency-bound on its two reductions).
template <int NC, int RP>
__global__ __launch_bounds__(256) void ln_bwd_kernel(long M, int N, int rows_per_wave, const bf16* __restrict__ dy,
                                                     const bf16* __restrict__ s, const float2* __restrict__ stats,
                                                     const float* __restrict__ g, bf16* __restrict__ ds,
                                                     bf16* __restrict__ dres, float* __restrict__ part, LnDrop dr,
                                                     const bf16* __restrict__ rp) {
  extern __shared__ float red[];                      // [4 waves][2][N]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nc = N / 8;
  float dgp[NC][8], dbp[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dgp[c][j] = dbp[c][j] = 0.f;
  const long r0 = ((long)blockIdx.x * 4 + wave) * rows_per_wave;
  const long r1 = min(M, r0 + rows_per_wave);
  for (long m0 = r0; m0 < r1; m0 += RP) {
    const bool two = RP == 2 && m0 + 1 < r1;         // wave-uniform
    float xh[RP][NC][8], gy[RP][NC][8];
    uint32_t neg[RP][NC];                             // sl_x: bit j = pre-activation x[j] <= 0
    float a1[RP], a2[RP];
    float2 st[RP];
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      a1[u] = a2[u] = 0.f;
      const long m = two ? m0 + u : m0;               // a lone last row is processed twice, counted once
      st[u] = stats[m];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int cc = lane + 64 * c;
        if (cc < nc) {
          float dv[8];
          ld8bf(s + m * N + 8 * cc, xh[u][c]);
          if (dr.sl_x != 0.f) {
            neg[u][c] = 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              neg[u][c] |= (xh[u][c][j] > 0.f ? 0u : 1u) << j;
              xh[u][c][j] = (float)(bf16)ln_lrelu(xh[u][c][j], dr.sl_x);
            }
          }
          ld8bf(dy + m * N + 8 * cc, dv);
          if (dr.th_o) {
            float mk[8];
            ln_drop8(dr.base_o, dr.th_o, dr.sc_o, m, cc, mk);
#pragma unroll
            for (int j = 0; j < 8; ++j) dv[j] *= mk[j];
          }
          const bool cnt = u == 0 || two;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            xh[u][c][j] = (xh[u][c][j] - st[u].x) * st[u].y;
            gy[u][c][j] = dv[j] * g[8 * cc + j];
            a1[u] += gy[u][c][j];
            a2[u] += gy[u][c][j] * xh[u][c][j];
            if (cnt) {
              dgp[c][j] += dv[j] * xh[u][c][j];
              dbp[c][j] += dv[j];
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      a1[u] = wave_sum(a1[u]) / N;
      a2[u] = wave_sum(a2[u]) / N;
    }
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      if (u == 1 && !two) break;
      const long m = m0 + u;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int cc = lane + 64 * c;
        if (cc < nc) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = st[u].y * (gy[u][c][j] - a1[u] - xh[u][c][j] * a2[u]);
          if (dr.sl_x != 0.f) {
            float dx[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) dx[j] = ((neg[u][c] >> j) & 1u) ? o[j] * dr.sl_x : o[j];
            st8bf(ds + m * N + 8 * cc, dx);
          } else {
            st8bf(ds + m * N + 8 * cc, o);
          }
          if (dres) {
            if (dr.th_r) {
              float mk[8];
              ln_drop8(dr.base_r, dr.th_r, dr.sc_r, m, cc, mk);
#pragma unroll
              for (int j = 0; j < 8; ++j) o[j] *= mk[j];
            }
            if (rp) {
              float rv[8];
              ld8bf(rp + m * N + 8 * cc, rv);
#pragma unroll
              for (int j = 0; j < 8; ++j) o[j] = rv[j] > 0.f ? o[j] : o[j] * dr.sl_r;
            }
            st8bf(dres + m * N + 8 * cc, o);
          }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cc = lane + 64 * c;
    if (cc < nc)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wave * 2 + 0) * N + 8 * cc + j] = dgp[c][j];
        red[(wave * 2 + 1) * N + 8 * cc + j] = dbp[c][j];
      }
  }
  __syncthreads();
  for (int n = threadIdx.x; n < 2 * N; n += 256) {
    const int which = n / N, col = n % N;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) acc += red[(w * 2 + which) * N + col];
    part[(long)blockIdx.x * 2 * N + n] = acc;
  }
}

// ---- forward on 16-lane row groups (N = 128 .. 512, the d384 model's N = 384): a wave
// normalises four rows at once, 16 lanes per row, NCH 8-column chunks per lane.  One row per wave
// left 16 of 64 lanes idle at N = 384 (48 chunks) and paid two 6-step wave reductions per row;
// here every lane works and the reductions are 4-step xor shuffles inside the group
// (tools/ln_micro.py, M = 49 440: 32.7 -> 28.2 us with residual dropout, 21.7 -> 17.6 us plain).
__device__ __forceinline__ float gsum16(float v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

template <int NCH>
__global__ __launch_bounds__(256) void ln_fwd_train_g16(long M, int N, const bf16* __restrict__ x,
                                                        const bf16* __restrict__ r, const float* __restrict__ g,
                                                        const float* __restrict__ b, float eps,
                                                        bf16* __restrict__ y, bf16* __restrict__ s_out,
                                                        float2* __restrict__ stats, LnDrop dr) {
  const int lane = threadIdx.x & 63, l16 = lane & 15;
  const long m = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
  const bool ok = m < M;
  const long mm = ok ? m : M - 1;                     // loads clamped, stores guarded
  float v[NCH][8];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cc = l16 + 16 * c;
    ld8bf(x + mm * N + 8 * cc, v[c]);
    if (dr.sl_x != 0.f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = (float)(bf16)ln_lrelu(v[c][j], dr.sl_x);
    }
    if (r) {
      float t[8];
      ld8bf(r + mm * N + 8 * cc, t);
      if (dr.sl_r != 0.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = (float)(bf16)ln_lrelu(t[j], dr.sl_r);
      }
      if (dr.th_r) {
        float mk[8];
        ln_drop8(dr.base_r, dr.th_r, dr.sc_r, mm, cc, mk);
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] *= mk[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = (float)(bf16)(v[c][j] + t[j]);   // s is kept in bf16
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += v[c][j];
  }
  const float mean = gsum16(sum) / N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = v[c][j] - mean; q += d * d; }
  const float rstd = 1.0f / sqrtf(gsum16(q) / N + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cc = l16 + 16 * c;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * g[8 * cc + j] + b[8 * cc + j];
    if (dr.th_o) {
      float mk[8];
      ln_drop8(dr.base_o, dr.th_o, dr.sc_o, mm, cc, mk);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] *= mk[j];
    }
    if (ok) {
      st8bf(y + m * N + 8 * cc, o);
      if (s_out) st8bf(s_out + m * N + 8 * cc, v[c]);
    }
  }
  if (ok && l16 == 0) stats[m] = make_float2(mean, rstd);
}

// ln_bwd_kernel<NC, 1> with the next row's s / dy / stats loads issued before the current row's
// reductions (a wave's rows are otherwise load -> reduce -> store in series, latency-bound)
__device__ __forceinline__ void unpack8bf(const u32x4& a, float* v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(a[e] << 16);
    v[2 * e + 1] = __uint_as_float(a[e] & 0xffff0000u);
  }
}
template <int NC>
__global__ __launch_bounds__(256) void ln_bwd_pf_kernel(long M, int N, int rows_per_wave, const bf16* __restrict__ dy,
                                                        const bf16* __restrict__ s, const float2* __restrict__ stats,
                                                        const float* __restrict__ g, bf16* __restrict__ ds,
                                                        bf16* __restrict__ dres, float* __restrict__ part, LnDrop dr,
                                                        const bf16* __restrict__ rp) {
  extern __shared__ float red[];                      // [4 waves][2][N]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nc = N / 8;
  float dgp[NC][8], dbp[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dgp[c][j] = dbp[c][j] = 0.f;
  const long r0 = ((long)blockIdx.x * 4 + wave) * rows_per_wave;
  const long r1 = min(M, r0 + rows_per_wave);
  u32x4 ns[NC], nd[NC];
  float2 nst = make_float2(0.f, 0.f);
  auto fetch = [&](long m) {
    nst = stats[m];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int cc = lane + 64 * c;
      if (cc < nc) {
        ns[c] = *reinterpret_cast<const u32x4*>(s + m * N + 8 * cc);
        nd[c] = *reinterpret_cast<const u32x4*>(dy + m * N + 8 * cc);
      }
    }
  };
  if (r0 < r1) fetch(r0);
  for (long m = r0; m < r1; ++m) {
    u32x4 cs[NC], cd[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      cs[c] = ns[c];
      cd[c] = nd[c];
    }
    const float2 st = nst;
    if (m + 1 < r1) fetch(m + 1);
    float xh[NC][8], gy[NC][8];
    uint32_t neg[NC];
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int cc = lane + 64 * c;
      if (cc < nc) {
        float dv[8];
        unpack8bf(cs[c], xh[c]);
        if (dr.sl_x != 0.f) {
          neg[c] = 0u;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            neg[c] |= (xh[c][j] > 0.f ? 0u : 1u) << j;
            xh[c][j] = (float)(bf16)ln_lrelu(xh[c][j], dr.sl_x);
          }
        }
        unpack8bf(cd[c], dv);
        if (dr.th_o) {
          float mk[8];
          ln_drop8(dr.base_o, dr.th_o, dr.sc_o, m, cc, mk);
#pragma unroll
          for (int j = 0; j < 8; ++j) dv[j] *= mk[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xh[c][j] - st.x) * st.y;
          gy[c][j] = dv[j] * g[8 * cc + j];
          a1 += gy[c][j];
          a2 += gy[c][j] * xh[c][j];
          dgp[c][j] += dv[j] * xh[c][j];
          dbp[c][j] += dv[j];
        }
      }
    }
    a1 = wave_sum(a1) / N;
    a2 = wave_sum(a2) / N;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int cc = lane + 64 * c;
      if (cc < nc) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = st.y * (gy[c][j] - a1 - xh[c][j] * a2);
        if (dr.sl_x != 0.f) {
          float dx[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) dx[j] = ((neg[c] >> j) & 1u) ? o[j] * dr.sl_x : o[j];
          st8bf(ds + m * N + 8 * cc, dx);
        } else {
          st8bf(ds + m * N + 8 * cc, o);
        }
        if (dres) {
          if (dr.th_r) {
            float mk[8];
            ln_drop8(dr.base_r, dr.th_r, dr.sc_r, m, cc, mk);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] *= mk[j];
          }
          if (rp) {
            float rv[8];
            ld8bf(rp + m * N + 8 * cc, rv);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = rv[j] > 0.f ? o[j] : o[j] * dr.sl_r;
          }
          st8bf(dres + m * N + 8 * cc, o);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cc = lane + 64 * c;
    if (cc < nc)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wave * 2 + 0) * N + 8 * cc + j] = dgp[c][j];
        red[(wave * 2 + 1) * N + 8 * cc + j] = dbp[c][j];
      }
  }
  __syncthreads();
  for (int n = threadIdx.x; n < 2 * N; n += 256) {
    const int which = n / N, col = n % N;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) acc += red[(w * 2 + which) * N + col];
    part[(long)blockIdx.x * 2 * N + n] = acc;
  }
}

// column sums of the ln_bwd partials [R][2N] into dg (columns < N) and db: written, or added
// to what they hold (accumulate: the parameters' .grad buffers); fixed-order (deterministic).
// 16 columns x 64 row groups per block (1 024 threads): at N = 384 the grid is only 48 blocks, so
// the rows are cut 64 ways (16 ways: ~32 dependent load rounds per thread at R = 2 048, 10.5 us)
__global__ __launch_bounds__(1024) void ln_part_sum_kernel(long R, int N, const float* __restrict__ x,
                                                           float* __restrict__ dg, float* __restrict__ db,
                                                           int accumulate) {
  __shared__ float red[64][17];
  const int cl = threadIdx.x & 15, gi = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl, W = 2 * N;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < W) {
    long r = gi;
    for (; r + 192 < R; r += 256) {
      a0 += x[r * W + c];
      a1 += x[(r + 64) * W + c];
      a2 += x[(r + 128) * W + c];
      a3 += x[(r + 192) * W + c];
    }
    for (; r < R; r += 64) a0 += x[r * W + c];
  }
  red[gi][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (gi == 0 && c < W) {
    float sum = 0.f;
#pragma unroll 8
    for (int i = 0; i < 64; ++i) sum += red[i][cl];
    float* o = c < N ? dg + c : db + (c - N);
    *o = accumulate ? *o + sum : sum;
  }
}

// out[n] (+)= sum over the R rows of f32 partials x[R, N]: 16 columns x 16 row groups per
// block (64-B row segments), four independent loads in flight per thread, fixed-order
// reduction of the groups (deterministic).  In-place use (out == x, row 0) is safe: a
// block writes only its own columns, after all of its reads.
__global__ __launch_bounds__(256) void colsum_f32_kernel(long R, int N, const float* x, float* out,
                                                         int accumulate) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < N) {
    long r = g;
    for (; r + 48 < R; r += 64) {
      a0 += x[r * N + c];
      a1 += x[(r + 16) * N + c];
      a2 += x[(r + 32) * N + c];
      a3 += x[(r + 48) * N + c];
    }
    for (; r < R; r += 16) a0 += x[r * N + c];
  }
  red[g][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (g == 0 && c < N) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) sum += red[i][cl];
    out[c] = accumulate ? out[c] + sum : sum;
  }
}

// column sums of a bf16 [M, N] matrix (bias gradients): per-block partials over row slabs
__global__ __launch_bounds__(256) void colsum_part_kernel(long M, int N, int rows_per_block, const bf16* __restrict__ x,
                                                          float* __restrict__ part) {
  const int nc = N / 8;
  const int per = 256 / nc;                         // row lanes per block (>= 1)
  const int c = threadIdx.x % nc, rl = threadIdx.x / nc;
  extern __shared__ float red2[];                   // [per][N]
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rl < per) {
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(M, r0 + rows_per_block);
    for (long m = r0 + rl; m < r1; m += per) {
      float v[8];
      ld8bf(x + m * N + 8 * c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red2[rl * N + 8 * c + j] = acc[j];
  }
  __syncthreads();
  for (int n = threadIdx.x; n < N; n += 256) {
    float s = 0.f;
    for (int w = 0; w < per; ++w) s += red2[w * N + n];
    part[(long)blockIdx.x * N + n] = s;
  }
}
// ---------------------------------------------------------------------------------------------
// Train-mode neighbour mean with the reference's dropout semantics (embedding_rag_dataset.py:
// 404-417 + bert.py:176-179): every UNIQUE retrieved haplotype u of a window is re-encoded once,
//   E[u, l] = drop_u,l( W[tok(u, l)] + pe[l] + Ar[l] ),   tok = <sos> | tok0 + code[u][l-1] | <eos> | <pad>,
// and query q takes the mean over its valid neighbours: out[q, l] = (1 / nv_q) sum_j E[inv[q, j], l].
// Fused: E is never materialised ([U, L, D] f32 is ~0.6 GB at B = 24, k = 8); every (query,
// neighbour, position, feature) recomputes the embedding from the 10-row table and the dropout
// keep bit from a counter-based hash of (seed, u, l, d pair) — the same bits in the backward,
//   dW[tok(u, l)] += g,  dAr[l] += g,  g = dout[q, l] / nv_q * keep / (1 - p),
// which accumulates per thread over its (l, d) and per token row with one atomic per block.
struct NbrArgs {
  int nq, k, L, D, n_sites, ld_codes, V;
  const int* inv;               // [nq, k] unique-neighbour index, < 0: no neighbour
  const uint8_t* codes;         // [U, ld_codes] allele codes of the unique neighbours
  const float* W;               // [V, D] token table (f32)
  const float* pe;              // [L, D]
  const float* Ar;              // [L, D]
  uint32_t thresh, base;        // keep iff hash half >= thresh (thresh 0: no dropout)
  float scale;                  // 1 / (1 - p)
  int tok0, sos, eos, pad;
};

__device__ __forceinline__ int nbr_tok(const NbrArgs& a, int u, int l) {
  if (l == 0) return a.sos;
  if (l <= a.n_sites) return a.tok0 + a.codes[(long)u * a.ld_codes + l - 1];
  return l == a.n_sites + 1 ? a.eos : a.pad;
}
// keep multipliers (0 or scale) of features d, d + 1 (d even) of (u, l)
__device__ __forceinline__ void nbr_keep2(const NbrArgs& a, int u, int l, int d, float& m0, float& m1) {
  if (!a.thresh) { m0 = m1 = 1.f; return; }
  const uint32_t h = drop_mix24(a.base + (uint32_t)u * DROP_C1 + (uint32_t)((l * a.D + d) >> 1) * DROP_C2);
  m0 = (h & 0xFFFFu) >= a.thresh ? a.scale : 0.f;
  m1 = (h >> 16) >= a.thresh ? a.scale : 0.f;
}

// grid (L, nq / 4): block = 4 queries x D / 2 feature pairs (threads: pair index, query)
__global__ __launch_bounds__(256) void nbr_mean_drop_fwd_kernel(NbrArgs a, float* __restrict__ out) {
  const int l = blockIdx.x, npair = a.D >> 1;
  const int pidx = threadIdx.x % 64, qs = threadIdx.x / 64;
  for (int q = blockIdx.y * 4 + qs; q < a.nq; q += gridDim.y * 4) {
    int nv = 0;
    for (int j = 0; j < a.k; ++j) nv += a.inv[q * a.k + j] >= 0;
    const float inv_nv = 1.f / (float)max(nv, 1);
    for (int pp = pidx; pp < npair; pp += 64) {
      const int d = 2 * pp;
      const float c0 = a.pe[(long)l * a.D + d] + a.Ar[(long)l * a.D + d];
      const float c1 = a.pe[(long)l * a.D + d + 1] + a.Ar[(long)l * a.D + d + 1];
      float s0 = 0.f, s1 = 0.f;
      for (int j = 0; j < a.k; ++j) {
        const int u = a.inv[q * a.k + j];
        if (u < 0) continue;
        const int t = nbr_tok(a, u, l);
        float m0, m1;
        nbr_keep2(a, u, l, d, m0, m1);
        s0 = fmaf(m0, a.W[(long)t * a.D + d] + c0, s0);
        s1 = fmaf(m1, a.W[(long)t * a.D + d + 1] + c1, s1);
      }
      float* o = out + ((long)q * a.L + l) * a.D + d;
      o[0] = s0 * inv_nv;
      o[1] = s1 * inv_nv;
    }
  }
}

// grid (L): block = one position x the D / 2 feature pairs (one thread each, blockDim rounded to
// whole waves); a thread loops every query and neighbour of its (position, pair); dAr[l] is owned
// by one thread (accumulated in place), dW rows get one atomic per (block, token row, feature).
// (r3: 4 positions per 256-thread block, each thread 3 pairs in series: 258 blocks = one wave per
// SIMD on a latency-bound loop, 0.50 ms per step at B = 24.)
__global__ __launch_bounds__(256) void nbr_mean_drop_bwd_kernel(NbrArgs a, const float* __restrict__ dout,
                                                                float* __restrict__ dW, float* __restrict__ dAr) {
  extern __shared__ float wacc[];                    // [V][D] block partials of dW
  const int npair = a.D >> 1;
  for (int i = threadIdx.x; i < a.V * a.D; i += blockDim.x) wacc[i] = 0.f;
  __syncthreads();
  for (int pp = threadIdx.x; pp < npair; pp += blockDim.x) {
    const int d = 2 * pp;
    {
      const int l = blockIdx.x;
      float ar0 = 0.f, ar1 = 0.f;
      float w0[2] = {0.f, 0.f}, w1[2] = {0.f, 0.f};  // the two site tokens (tok0, tok0 + 1)
      float ws0 = 0.f, ws1 = 0.f;                     // the position's single token (sos / eos / pad)
      const bool site = l >= 1 && l <= a.n_sites;
      for (int q = 0; q < a.nq; ++q) {
        int nv = 0;
        for (int j = 0; j < a.k; ++j) nv += a.inv[q * a.k + j] >= 0;
        if (nv == 0) continue;
        const float* g = dout + ((long)q * a.L + l) * a.D + d;
        const float g0 = g[0] / (float)nv, g1 = g[1] / (float)nv;
        for (int j = 0; j < a.k; ++j) {
          const int u = a.inv[q * a.k + j];
          if (u < 0) continue;
          float m0, m1;
          nbr_keep2(a, u, l, d, m0, m1);
          const float e0 = g0 * m0, e1 = g1 * m1;
          ar0 += e0;
          ar1 += e1;
          if (site) {
            const int c = a.codes[(long)u * a.ld_codes + l - 1] & 1;
            w0[c] += e0;
            w1[c] += e1;
          } else {
            ws0 += e0;
            ws1 += e1;
          }
        }
      }
      dAr[(long)l * a.D + d] += ar0;
      dAr[(long)l * a.D + d + 1] += ar1;
      if (site) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          atomicAdd(&wacc[(a.tok0 + c) * a.D + d], w0[c]);
          atomicAdd(&wacc[(a.tok0 + c) * a.D + d + 1], w1[c]);
        }
      } else {
        const int t = l == 0 ? a.sos : (l == a.n_sites + 1 ? a.eos : a.pad);
        if (t != a.pad) {                              // nn.Embedding(padding_idx = <pad>): no gradient
          atomicAdd(&wacc[t * a.D + d], ws0);
          atomicAdd(&wacc[t * a.D + d + 1], ws1);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < a.V * a.D; i += blockDim.x)
    if (wacc[i] != 0.f) unsafeAtomicAdd(dW + i, wacc[i]);
}

// ---- the hap head's last Linear(4D, 2) (foundation_model.py:25-33 net[2]) under autograd: bf16
// activations against f32 weights, f32 logits.  torch ran it as F.linear(hh.float(), W): a 300 MB
// f32 copy of hh and f32 GEMMs with N = 2 (hipBLASLt: 0.29 ms for dW alone at M = 49 440).
// fwd: a 16-lane group computes 4 rows (16 per wave), 8-column chunks, so each weight load
// serves 4 rows' activations; out[m] = (x[m] . w0 + b0, x[m] . w1 + b1)
__global__ __launch_bounds__(256) void head2_fwd_kernel(long M, int K, const bf16* __restrict__ x,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float* __restrict__ out) {
  const int lane = threadIdx.x & 63, l16 = lane & 15;
  const long m0 = (((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4)) * 4;
  if (m0 >= M) return;                                // group-uniform
  const bf16* xr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) xr[r] = x + min(m0 + r, M - 1) * K;   // tail rows: re-read the last
  float a0[4] = {}, a1[4] = {};
  for (int c = l16; c < K / 8; c += 16) {
    float v[4][8], w0[8], w1[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) ld8bf(xr[r] + 8 * c, v[r]);
    *reinterpret_cast<float4*>(w0) = *reinterpret_cast<const float4*>(w + 8 * c);
    *reinterpret_cast<float4*>(w0 + 4) = *reinterpret_cast<const float4*>(w + 8 * c + 4);
    *reinterpret_cast<float4*>(w1) = *reinterpret_cast<const float4*>(w + K + 8 * c);
    *reinterpret_cast<float4*>(w1 + 4) = *reinterpret_cast<const float4*>(w + K + 8 * c + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a0[r] = fmaf(v[r][j], w0[j], a0[r]);
        a1[r] = fmaf(v[r][j], w1[j], a1[r]);
      }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float s0 = gsum16(a0[r]), s1 = gsum16(a1[r]);
    if (l16 == r && m0 + r < M) reinterpret_cast<float2*>(out)[m0 + r] = make_float2(s0 + b[0], s1 + b[1]);
  }
}
// fwd at K = 512 NCH (the model's 4D = 1536: NCH = 3): a wave owns 16 rows (M = 49 440: 3 090
// waves, one round at 4 waves/SIMD for 128 VGPRs) and keeps its lanes'
// weight chunks in registers; per 4-row batch all 4 NCH activation loads are issued before use
template <int NCH>
__global__ __launch_bounds__(256) void head2_fwd_wave_kernel(long M, const bf16* __restrict__ x,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             float* __restrict__ out) {
  constexpr int K = 512 * NCH;
  const int lane = threadIdx.x & 63;
  const long mw = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  if (mw >= M) return;                                // wave-uniform
  float w0[NCH][8], w1[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *reinterpret_cast<float4*>(&w0[i][4 * h]) = *reinterpret_cast<const float4*>(w + 8 * (lane + 64 * i) + 4 * h);
      *reinterpret_cast<float4*>(&w1[i][4 * h]) = *reinterpret_cast<const float4*>(w + K + 8 * (lane + 64 * i) + 4 * h);
    }
  const float b0 = b[0], b1 = b[1];
  for (int rb = 0; rb < 16; rb += 4) {
    u32x4 raw[4][NCH];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < NCH; ++i)
        raw[r][i] = *reinterpret_cast<const u32x4*>(x + min(mw + rb + r, M - 1) * K + 8 * (lane + 64 * i));
    float a0[4] = {}, a1[4] = {};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < NCH; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float lo = __uint_as_float(raw[r][i][j] << 16), hi = __uint_as_float(raw[r][i][j] & 0xffff0000u);
          a0[r] = fmaf(lo, w0[i][2 * j], fmaf(hi, w0[i][2 * j + 1], a0[r]));
          a1[r] = fmaf(lo, w1[i][2 * j], fmaf(hi, w1[i][2 * j + 1], a1[r]));
        }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        a0[r] += __shfl_xor(a0[r], o, 64);
        a1[r] += __shfl_xor(a1[r], o, 64);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (lane == r && mw + rb + r < M) reinterpret_cast<float2*>(out)[mw + rb + r] = make_float2(a0[r] + b0, a1[r] + b1);
  }
}
// dx[m, k] = g[m, 0] w[0, k] + g[m, 1] w[1, k] (bf16), one thread per 8 elements
__global__ __launch_bounds__(256) void head2_dx_kernel(long M, int K, const float* __restrict__ g,
                                                       const float* __restrict__ w, bf16* __restrict__ dx) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x, n8 = (long)M * (K / 8);
  if (i >= n8) return;
  const long m = i / (K / 8);
  const int c = (int)(i % (K / 8));
  const float2 gm = reinterpret_cast<const float2*>(g)[m];
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = gm.x * w[8 * c + j] + gm.y * w[K + 8 * c + j];
  st8bf(dx + m * K + 8 * c, o);
}
// dW partials: block b sums rows [b R, (b + 1) R) of g[m, j] x[m, k] into part[b][j K + k]
// (columns over the threads, 8 per thread); ln_part_sum_kernel then sums the blocks in order
__global__ __launch_bounds__(256) void head2_dw_kernel(long M, int K, int rows_per_block, const float* __restrict__ g,
                                                       const bf16* __restrict__ x, float* __restrict__ part) {
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int c = threadIdx.x; c < K / 8; c += blockDim.x) {
    float s0[8] = {}, s1[8] = {};
    long m = r0;
    for (; m + 8 <= r1; m += 8) {                     // 8 rows' loads in flight
      float2 gm[8];
      float v[8][8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        gm[r] = reinterpret_cast<const float2*>(g)[m + r];
        ld8bf(x + (m + r) * K + 8 * c, v[r]);
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s0[j] = fmaf(gm[r].x, v[r][j], s0[j]);
          s1[j] = fmaf(gm[r].y, v[r][j], s1[j]);
        }
    }
    for (; m < r1; ++m) {
      const float2 gm = reinterpret_cast<const float2*>(g)[m];
      float v[8];
      ld8bf(x + m * K + 8 * c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s0[j] = fmaf(gm.x, v[j], s0[j]);
        s1[j] = fmaf(gm.y, v[j], s1[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      part[(long)blockIdx.x * 2 * K + 8 * c + j] = s0[j];
      part[(long)blockIdx.x * 2 * K + K + 8 * c + j] = s1[j];
    }
  }
}

// ---- weight gradient of a token table of V <= 16 rows (BERTEmbedding's TokenEmbedding,
// embedding/bert.py:63-75, under autograd): dW[v] = sum over rows m with tok[m] = v of g[m]; the
// padding row (nn.Embedding padding_idx) gets none.  Per-block partials over row ranges (every
// thread owns 2 columns and 16 x 2 accumulators, rows selected by compare, no dynamic register
// indexing), then the fixed-order column sum: deterministic.  Replaces a one-hot f32 GEMM of
// K = M (hipBLASLt: 104 us at M = 49 440, no split-K) and its one_hot / cast / fill kernels.
__global__ __launch_bounds__(256) void tokgrad_part_kernel(long M, int D, int V, int pad, int rows_per_block,
                                                           const long* __restrict__ tok, const float* __restrict__ g,
                                                           float* __restrict__ part) {
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int c = threadIdx.x; c < D / 2; c += blockDim.x) {
    float2 acc[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = make_float2(0.f, 0.f);
    for (long m0 = r0; m0 < r1; m0 += 8) {            // 8 rows' loads in flight
      long t[8];
      float2 x[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const long m = min(m0 + r, r1 - 1);
        t[r] = m0 + r < r1 ? tok[m] : -1;
        x[r] = reinterpret_cast<const float2*>(g + m * D)[c];
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const bool hit = t[r] == v && v != pad;
          acc[v].x += hit ? x[r].x : 0.f;
          acc[v].y += hit ? x[r].y : 0.f;
        }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v)
      if (v < V) reinterpret_cast<float2*>(part + (long)blockIdx.x * V * D + (long)v * D)[c] = acc[v];
  }
}

}  // namespace snvrag

extern "C" int snvrag_ln_fwd_train(int64_t M, int N, const void* x, const void* r, const float* g, const float* b,
                                   float eps, void* y, void* s_out, float* stats, float p_r, float p_out,
                                   uint64_t seed, void* stream) {
  return snvrag_ln_fwd_train_act(M, N, x, r, g, b, eps, y, s_out, stats, p_r, p_out, seed, 0.f, 0.f, stream);
}

extern "C" int snvrag_ln_fwd_train_act(int64_t M, int N, const void* x, const void* r, const float* g,
                                       const float* b, float eps, void* y, void* s_out, float* stats, float p_r,
                                       float p_out, uint64_t seed, float slope_x, float slope_r, void* stream) {
  SNV_CHECK_ARG(slope_x == 0.f || !r, "an input activation is for a norm without a residual");
  SNV_CHECK_ARG(slope_r == 0.f || r, "a residual activation needs a residual");
  SNV_CHECK_ARG(x && g && b && y && stats, "null pointer");
  SNV_CHECK_ARG(N % 8 == 0 && N <= 64 * 8 * LN_MAXC, "N must be a multiple of 8, <= 2048");
  SNV_CHECK_ARG(!r || s_out, "a residual needs s_out");
  SNV_CHECK_ARG(p_r >= 0.f && p_r < 1.f && p_out >= 0.f && p_out < 1.f, "dropout probabilities must be in [0, 1)");
  SNV_CHECK_ARG(r || p_r == 0.f, "residual dropout without a residual");
  if (M == 0) return 0;
  const LnDrop dr = make_ln_drop(p_r, p_out, seed, slope_x, slope_r);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(cdiv(M, 4)), dim3(256), 0, as_stream(stream), (long)M, N, (const bf16*)x,
                       (const bf16*)r, g, b, eps, (bf16*)y, (bf16*)s_out, (float2*)stats, dr);
  };
  const int nch = cdiv(N / 8, 64), nc = N / 8;
  if (nc % 16 == 0 && nc <= 64 && options().ln_rows1 == 0) {
    // 16-lane row groups: four rows per wave, 16 rows per workgroup
    auto go16 = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(cdiv(M, 16)), dim3(256), 0, as_stream(stream), (long)M, N, (const bf16*)x,
                         (const bf16*)r, g, b, eps, (bf16*)y, (bf16*)s_out, (float2*)stats, dr);
    };
    if (nc == 16) go16(ln_fwd_train_g16<1>);
    else if (nc == 32) go16(ln_fwd_train_g16<2>);
    else if (nc == 48) go16(ln_fwd_train_g16<3>);
    else go16(ln_fwd_train_g16<4>);
  } else if (nch == 1) go(ln_fwd_train_kernel<1>);
  else if (nch == 2) go(ln_fwd_train_kernel<2>);
  else if (nch == 3) go(ln_fwd_train_kernel<3>);
  else go(ln_fwd_train_kernel<4>);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t snvrag_ln_bwd_ws_bytes(int64_t M, int N) {
  const long nblk = std::min<long>(cdiv(M, 4 * LN_BWD_RPW), 2048);
  return (size_t)nblk * 2 * N * sizeof(float);
}

extern "C" int snvrag_ln_bwd(int64_t M, int N, const void* dy, const void* s, const float* stats, const float* g,
                             void* ds, void* dres, float* dg, float* db, int accumulate, float p_r, float p_out,
                             uint64_t seed, void* ws, size_t ws_bytes, void* stream) {
  SNV_CHECK_ARG(!dres || p_r > 0.f, "dres is the residual-dropout gradient (p_r > 0)");
  return snvrag_ln_bwd_act(M, N, dy, s, stats, g, ds, dres, nullptr, dg, db, accumulate, p_r, p_out, seed, 0.f, 0.f,
                           ws, ws_bytes, stream);
}

extern "C" int snvrag_ln_bwd_act(int64_t M, int N, const void* dy, const void* s, const float* stats, const float* g,
                                 void* ds, void* dres, const void* r_pre, float* dg, float* db, int accumulate,
                                 float p_r, float p_out, uint64_t seed, float slope_x, float slope_r, void* ws,
                                 size_t ws_bytes, void* stream) {
  SNV_CHECK_ARG(dy && s && stats && g && ds && dg && db && ws, "null pointer");
  SNV_CHECK_ARG(N % 8 == 0 && N <= 64 * 8 * LN_MAXC, "N must be a multiple of 8, <= 2048");
  SNV_CHECK_ARG(ws_bytes >= snvrag_ln_bwd_ws_bytes(M, N), "workspace too small");
  SNV_CHECK_ARG(p_r >= 0.f && p_r < 1.f && p_out >= 0.f && p_out < 1.f, "dropout probabilities must be in [0, 1)");
  SNV_CHECK_ARG(slope_r == 0.f || (dres && r_pre), "a residual activation needs dres and the pre-activation r");
  SNV_CHECK_ARG(!dres || p_r > 0.f || slope_r != 0.f, "dres is the residual operand's own gradient");
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  const long nblk = std::min<long>(cdiv(M, 4 * LN_BWD_RPW), 2048);
  const int rpw = (int)((M + nblk * 4 - 1) / (nblk * 4));
  float* part = (float*)ws;
  const LnDrop dr = make_ln_drop(p_r, p_out, seed, slope_x, slope_r);
  const bf16* rp = (const bf16*)(slope_r != 0.f ? r_pre : nullptr);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(256), 4 * 2 * N * sizeof(float), st, (long)M, N, rpw,
                       (const bf16*)dy, (const bf16*)s, (const float2*)stats, g, (bf16*)ds, (bf16*)dres, part, dr, rp);
  };
  const int nch = cdiv(N / 8, 64);
  // one row per wave step (2 rows: 174 -> 209 us at N = 1536, tools/ln_micro.py); for N > 512 the
  // next row's loads issued ahead (N = 1536: 147-150 vs 174 us; N = 384: 55 vs 52 us, so not there)
  // unless SNVRAG_LN_BWD_NOPF (A/B)
  const bool pf = !options().ln_bwd_nopf;
  // (16-lane row groups as in the forward: 62 vs 51 us at N = 384 — the per-lane dg / db
  // partials of 3 chunks cost occupancy, 198 VGPRs — so the backward keeps one row per wave)
  if (pf && nch > 1) {
    if (nch == 2) go(ln_bwd_pf_kernel<2>);
    else if (nch == 3) go(ln_bwd_pf_kernel<3>);
    else go(ln_bwd_pf_kernel<4>);
  } else if (nch == 1) go(ln_bwd_kernel<1, 1>);
  else if (nch == 2) go(ln_bwd_kernel<2, 1>);
  else if (nch == 3) go(ln_bwd_kernel<3, 1>);
  else go(ln_bwd_kernel<4, 1>);
  SNV_LAUNCH_CHECK();
  // dg = sum over blocks of part[:, 0, :], db of part[:, 1, :] (written or accumulated)
  hipLaunchKernelGGL(ln_part_sum_kernel, dim3(cdiv(2 * N, 16)), dim3(1024), 0, st, (long)nblk, N, (const float*)part,
                     dg, db, accumulate);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t snvrag_colsum_ws_bytes(int64_t M, int N) {
  const long nblk = std::min<long>(cdiv(M, 256), 1024);
  return (size_t)nblk * N * sizeof(float);
}

extern "C" int snvrag_colsum_bf16(int64_t M, int N, const void* x, float* out, void* ws, size_t ws_bytes,
                                  void* stream) {
  SNV_CHECK_ARG(x && out && ws, "null pointer");
  SNV_CHECK_ARG(N % 8 == 0 && N / 8 <= 256, "N must be a multiple of 8, <= 2048");
  SNV_CHECK_ARG(ws_bytes >= snvrag_colsum_ws_bytes(M, N), "workspace too small");
  hipStream_t st = as_stream(stream);
  if (M == 0) return (int)hipMemsetAsync(out, 0, N * sizeof(float), st);
  const long nblk = std::min<long>(cdiv(M, 256), 1024);
  const int rpb = (int)((M + nblk - 1) / nblk);
  const int per = 256 / (N / 8);
  hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)nblk), dim3(256), per * N * sizeof(float), st, (long)M, N,
                     rpb, (const bf16*)x, (float*)ws);
  SNV_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_f32_kernel, dim3(cdiv(N, 16)), dim3(256), 0, st, (long)nblk, N, (const float*)ws, out,
                     0);
  SNV_LAUNCH_CHECK();
  return 0;
}

static int nbr_args(NbrArgs& a, int64_t nq, int k, int64_t L, int D, int n_sites, int64_t ld_codes, int V,
                    const int32_t* inv, const uint8_t* codes, const float* W, const float* pe, const float* Ar,
                    float p, uint64_t seed, int tok0, int sos, int eos, int pad) {
  SNV_CHECK_ARG(inv && codes && W && pe && Ar, "null pointer");
  SNV_CHECK_ARG(D % 2 == 0 && D <= 2048 && V >= 1 && V * D <= 16384, "D even, V x D <= 16384");
  SNV_CHECK_ARG(n_sites + 2 <= L && ld_codes >= n_sites && k >= 1, "shape");
  SNV_CHECK_ARG(p >= 0.f && p < 1.f, "dropout probability must be in [0, 1)");
  SNV_CHECK_ARG(tok0 >= 0 && tok0 + 1 < V && sos < V && eos < V && pad < V, "token ids");
  const AttnDrop dr = make_attn_drop(p, seed);
  a = NbrArgs{(int)nq, k, (int)L, D, n_sites, (int)ld_codes, V, inv, codes, W, pe, Ar, dr.thresh,
              drop_base(seed, 7u), dr.scale, tok0, sos, eos, pad};
  return 0;
}

extern "C" int snvrag_nbr_mean_drop_fwd(int64_t nq, int k, int64_t L, int D, int n_sites, int64_t ld_codes, int V,
                                        const int32_t* inv, const uint8_t* codes, const float* W, const float* pe,
                                        const float* Ar, float p, uint64_t seed, int tok0, int sos, int eos, int pad,
                                        float* out, void* stream) {
  NbrArgs a;
  if (int rc = nbr_args(a, nq, k, L, D, n_sites, ld_codes, V, inv, codes, W, pe, Ar, p, seed, tok0, sos, eos, pad))
    return rc;
  SNV_CHECK_ARG(out, "null pointer");
  if (nq == 0) return 0;
  const unsigned gy = (unsigned)std::min<int64_t>((nq + 3) / 4, 64);
  hipLaunchKernelGGL(nbr_mean_drop_fwd_kernel, dim3((unsigned)L, gy), dim3(256), 0, as_stream(stream), a, out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_nbr_mean_drop_bwd(int64_t nq, int k, int64_t L, int D, int n_sites, int64_t ld_codes, int V,
                                        const int32_t* inv, const uint8_t* codes, const float* W, const float* pe,
                                        const float* Ar, float p, uint64_t seed, int tok0, int sos, int eos, int pad,
                                        const float* dout, float* dW, float* dAr, void* stream) {
  NbrArgs a;
  if (int rc = nbr_args(a, nq, k, L, D, n_sites, ld_codes, V, inv, codes, W, pe, Ar, p, seed, tok0, sos, eos, pad))
    return rc;
  SNV_CHECK_ARG(dout && dW && dAr, "null pointer");
  if (nq == 0) return 0;
  const int nthr = (int)std::min<long>(256, (D / 2 + 63) / 64 * 64);
  hipLaunchKernelGGL(nbr_mean_drop_bwd_kernel, dim3((unsigned)L), dim3(nthr), (size_t)V * D * sizeof(float),
                     as_stream(stream), a, dout, dW, dAr);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_head2_fwd(int64_t M, int K, const void* x, const float* w, const float* b, float* out,
                                void* stream) {
  if (M == 0) return 0;
  SNV_CHECK_ARG(x && w && b && out, "null pointer");
  SNV_CHECK_ARG(K % 8 == 0 && K > 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0,
                "K % 8 == 0, 16-byte aligned x and w");
  if (K == 1536)
    hipLaunchKernelGGL(head2_fwd_wave_kernel<3>, dim3((unsigned)cdiv(M, 64)), dim3(256), 0, as_stream(stream),
                       (long)M, (const bf16*)x, w, b, out);
  else
    hipLaunchKernelGGL(head2_fwd_kernel, dim3((unsigned)cdiv(M, 64)), dim3(256), 0, as_stream(stream), (long)M, K,
                       (const bf16*)x, w, b, out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t snvrag_head2_ws_bytes(int64_t M, int K) {
  const long nblk = std::min<long>(cdiv(M, 64), 1024);
  return (size_t)nblk * 2 * K * sizeof(float);
}

extern "C" int snvrag_head2_bwd(int64_t M, int K, const float* g, const void* x, const float* w, void* dx, float* dw,
                                int accumulate, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t st = as_stream(stream);
  if (M == 0) {                                       // empty batch: dW = 0
    if (dw && !accumulate) SNV_HIP(hipMemsetAsync(dw, 0, (size_t)2 * K * sizeof(float), st));
    return 0;
  }
  SNV_CHECK_ARG(g && x && w && ws, "null pointer");
  SNV_CHECK_ARG(K % 8 == 0 && K > 0 && ((uintptr_t)x % 16) == 0 && (!dx || ((uintptr_t)dx % 16) == 0),
                "K % 8 == 0, 16-byte aligned x / dx");
  SNV_CHECK_ARG(ws_bytes >= snvrag_head2_ws_bytes(M, K), "workspace too small");
  if (dx) {
    const long n8 = (long)M * (K / 8);
    hipLaunchKernelGGL(head2_dx_kernel, dim3((unsigned)cdiv(n8, 256)), dim3(256), 0, st, (long)M, K, g, w, (bf16*)dx);
    SNV_LAUNCH_CHECK();
  }
  if (dw) {
    const long nblk = std::min<long>(cdiv(M, 64), 1024);
    const int rpb = (int)cdiv(M, nblk);
    hipLaunchKernelGGL(head2_dw_kernel, dim3((unsigned)nblk), dim3(std::min(256, (K / 8 + 63) / 64 * 64)), 0, st, (long)M, K, rpb, g, (const bf16*)x,
                       (float*)ws);
    SNV_LAUNCH_CHECK();
    // rows of dW = "dg" (columns < K) and "db" (columns >= K) of the LayerNorm partial-sum kernel
    hipLaunchKernelGGL(ln_part_sum_kernel, dim3(cdiv(2 * K, 16)), dim3(1024), 0, st, nblk, K, (const float*)ws, dw,
                       dw + K, accumulate);
    SNV_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" size_t snvrag_tokgrad_ws_bytes(int64_t M, int V, int D) {
  const long nblk = std::max<long>(1, std::min<long>(cdiv(M, 64), 1024));
  return (size_t)nblk * V * D * sizeof(float);
}

extern "C" int snvrag_tokgrad(int64_t M, int V, int D, int padding_idx, const int64_t* tok, const float* g, float* dw,
                              void* ws, size_t ws_bytes, void* stream) {
  SNV_CHECK_ARG(dw && ws, "null pointer");
  SNV_CHECK_ARG(V >= 1 && V <= 16 && D % 2 == 0 && D > 0, "1 <= V <= 16 rows, even D");
  SNV_CHECK_ARG(M == 0 || (tok && g && ((uintptr_t)g % 8) == 0), "tok / g (8-byte aligned)");
  SNV_CHECK_ARG(ws_bytes >= snvrag_tokgrad_ws_bytes(M, V, D), "workspace too small");
  hipStream_t st = as_stream(stream);
  if (M == 0) {
    SNV_HIP(hipMemsetAsync(dw, 0, (size_t)V * D * sizeof(float), st));
    return 0;
  }
  const long nblk = std::max<long>(1, std::min<long>(cdiv(M, 64), 1024));
  const int rpb = (int)cdiv(M, nblk);
  hipLaunchKernelGGL(tokgrad_part_kernel, dim3((unsigned)nblk), dim3(std::min(256, (D / 2 + 63) / 64 * 64)), 0, st,
                     (long)M, D, V, padding_idx, rpb, (const long*)tok, g, (float*)ws);
  SNV_LAUNCH_CHECK();
  // the V x D partial rows summed in block order: ln_part_sum_kernel over 2 N = V D columns
  const int VD = V * D;                              // even (D even)
  hipLaunchKernelGGL(ln_part_sum_kernel, dim3(cdiv(VD, 16)), dim3(1024), 0, st, nblk, VD / 2, (const float*)ws, dw,
                     dw + VD / 2, 0);
  SNV_LAUNCH_CHECK();
  return 0;
}
