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

__global__ __launch_bounds__(256) void sqnorm_kernel(long n, const float* __restrict__ x, float* __restrict__ acc) {
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
  if (threadIdx.x == 0) atomicAdd(acc, red[0] + red[1] + red[2] + red[3]);
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

extern "C" int snvrag_sqnorm(int64_t n, const float* x, float* acc, void* stream) {
  SNV_CHECK_ARG(x && acc && ((uintptr_t)x % 16) == 0, "null or misaligned pointer");
  hipStream_t s = as_stream(stream);
  SNV_HIP(hipMemsetAsync(acc, 0, sizeof(float), s));
  if (n == 0) return 0;
  const int grid = (int)std::min<long>(cdiv(n / 4 + 1, 256), 2048);
  hipLaunchKernelGGL(sqnorm_kernel, dim3(grid), dim3(256), 0, s, (long)n, x, acc);
  SNV_LAUNCH_CHECK();
  return 0;
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
