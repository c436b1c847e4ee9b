// Issue rate of the transcendental candidates for the attention softmax (one wave per SIMD
// and four waves per SIMD): v_exp_f32, v_exp_f16 (half2: two per dword), v_cvt_pkrtz_f16_f32.
// Each thread runs 8 independent chains so latency is hidden; prints cycles per
// wave-instruction from clock64 deltas and the kernel time.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdio>

constexpr int ITERS = 4096;

__global__ void k_exp32(float* out, float seed) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i) * 1e-6f - 1.0f;
  const long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_amdgcn_exp2f(a[i]) - 1.5f;
  }
  const long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)(t1 - t0) / (ITERS * 8);
}

__global__ void k_exp16(float* out, float seed) {
  _Float16 a[16];
  for (int i = 0; i < 16; ++i) a[i] = (_Float16)(seed * (threadIdx.x + i) * 1e-6f - 1.0f);
  const long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = __builtin_elementwise_exp2(a[i]) - (_Float16)1.5f;
  }
  const long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += (float)a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)(t1 - t0) / (ITERS * 16);
}

__global__ void k_add32(float* out, float seed) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i) * 1e-6f - 1.0f;
  const long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = a[i] * 0.999f - 1.5f;
  }
  const long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)(t1 - t0) / (ITERS * 8);
}

template <typename K>
void run(const char* name, K kern, int waves_per_simd) {
  float* d;
  hipMalloc(&d, 256 * 1024 * 16 * sizeof(float));
  const int blocks = 256 * waves_per_simd;          // 256-thread blocks: one wave per SIMD each
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  float cyc;
  hipMemcpy(&cyc, d, sizeof(float), hipMemcpyDeviceToHost);
  printf("%-10s waves/SIMD %d: %.2f cycles per instruction per wave (clock64), kernel %.3f ms\n", name,
         waves_per_simd, cyc, ms);
  hipFree(d);
}

int main() {
  for (int w : {1, 4}) {
    run("add_f32", k_add32, w);
    run("exp_f32", k_exp32, w);
    run("exp_f16", k_exp16, w);
  }
  return 0;
}
