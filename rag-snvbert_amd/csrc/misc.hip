// Error reporting, ABI/device queries and MFMA layout self-tests.
#include "common.h"

#include <cctype>
#include <cstdlib>
#include <cstring>

namespace snvrag {

static thread_local std::string g_err;

struct EvLog {
  bool on = false;
  int cap = 0, n = 0;
  hipEvent_t* ev = nullptr;     // 2 * cap
  int* kind = nullptr;
  double* work = nullptr;
};
static EvLog g_ev;

bool evlog_on() { return g_ev.on && g_ev.n < g_ev.cap; }
void evlog_begin(hipStream_t s) {
  if (evlog_on()) (void)hipEventRecord(g_ev.ev[2 * g_ev.n], s);
}
void evlog_end(hipStream_t s, int kind, double work) {
  if (!evlog_on()) return;
  (void)hipEventRecord(g_ev.ev[2 * g_ev.n + 1], s);
  g_ev.kind[g_ev.n] = kind;
  g_ev.work[g_ev.n] = work;
  g_ev.n++;
}

void set_error(const std::string& msg) { g_err = msg; }
int fail(const char* where, const std::string& msg) {
  g_err = std::string(where) + ": " + msg;
  return 1;
}

// One wave: D = A B with exact small-integer data for the three MFMA forms the
// kernels use, in the operand/accumulator maps the kernels assume; lane 0 also
// computes the product with scalar loops and counts mismatches.
__global__ void mfma_selftest_kernel(int* errors) {
  const int lane = threadIdx.x, li = lane & 15, lg = lane >> 4;
  __shared__ int A[16][64], B[64][16];
  for (int i = lane; i < 16 * 64; i += 64) {
    const int r = i / 64, k = i % 64;
    A[r][k] = ((r * 7 + k * 3) % 11) - 5;
    B[k][r] = ((k * 5 + r * 13) % 9) - 4;   // asymmetric
  }
  __syncthreads();
  int err = 0;
  // i8 16x16x64: A[row li][k = 16 lg + j], B[k = 16 lg + j][col li]
  {
    int8_t a8[16], b8[16];
    for (int j = 0; j < 16; ++j) { a8[j] = (int8_t)A[li][16 * lg + j]; b8[j] = (int8_t)B[16 * lg + j][li]; }
    i32x4 av = *reinterpret_cast<i32x4*>(a8), bv = *reinterpret_cast<i32x4*>(b8);
    i32x4 c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, i32x4{0, 0, 0, 0}, 0, 0, 0);
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * lg + i, col = li;
      int ref = 0;
      for (int k = 0; k < 64; ++k) ref += A[row][k] * B[k][col];
      err += c[i] != ref;
    }
  }
  // bf16 16x16x32: A[li][8 lg + j], B[8 lg + j][li]
  {
    bf16x8 av, bv;
    for (int j = 0; j < 8; ++j) { av[j] = (bf16)(float)A[li][8 * lg + j]; bv[j] = (bf16)(float)B[8 * lg + j][li]; }
    f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, f32x4{0, 0, 0, 0}, 0, 0, 0);
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * lg + i, col = li;
      int ref = 0;
      for (int k = 0; k < 32; ++k) ref += A[row][k] * B[k][col];
      err += c[i] != (float)ref;
    }
  }
  // f32 16x16x4: A[li][lg], B[lg][li]
  {
    f32x4 c = __builtin_amdgcn_mfma_f32_16x16x4f32((float)A[li][lg], (float)B[lg][li], f32x4{0, 0, 0, 0}, 0, 0, 0);
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * lg + i, col = li;
      int ref = 0;
      for (int k = 0; k < 4; ++k) ref += A[row][k] * B[k][col];
      err += c[i] != (float)ref;
    }
  }
  atomicAdd(errors, err);
}

}  // namespace snvrag

using namespace snvrag;

namespace snvrag {
namespace {
struct OptDesc { const char* name; int64_t Options::*field; int64_t dflt; };
const OptDesc kOpts[] = {
    {"knn_no_reduce", &Options::knn_no_reduce, 0}, {"scan_mode", &Options::scan_mode, 0},
    {"scan_nt", &Options::scan_nt, -1},            {"unfused_ln", &Options::unfused_ln, 0},
    {"encoder_chunk", &Options::encoder_chunk, 0}, {"gemm_tile128", &Options::gemm_tile128, 0},
    {"gemm_nw", &Options::gemm_nw, 0},             {"tail_variant", &Options::tail_variant, 0},
    {"tail_desync", &Options::tail_desync, -1},    {"sg_desync", &Options::sg_desync, -1},      {"mlp_desync", &Options::mlp_desync, -1},      {"g2_desync", &Options::g2_desync, -1},
    {"sg_waves4", &Options::sg_waves4, 0},         {"ln_bwd_nopf", &Options::ln_bwd_nopf, 0},
    {"attn_variant", &Options::attn_variant, 0},   {"dw_xcd", &Options::dw_xcd, 1},
    {"ln_rows1", &Options::ln_rows1, 0},           {"tail_persist", &Options::tail_persist, 0},
    {"tail_wide", &Options::tail_wide, 1},         {"proj_wide", &Options::proj_wide, 1},
    {"g2_variant", &Options::g2_variant, 0},     {"g2_groups", &Options::g2_groups, 0},
    {"tail_split", &Options::tail_split, 64},
};
Options make_options() {
  Options o{};
  for (const OptDesc& d : kOpts) {
    std::string env = "SNVRAG_";
    for (const char* c = d.name; *c; ++c) env += (char)toupper(*c);
    const char* v = getenv(env.c_str());
    o.*(d.field) = v ? atoll(v) : d.dflt;
  }
  return o;
}
const OptDesc* find_opt(const char* name) {
  for (const OptDesc& d : kOpts)
    if (name && strcmp(d.name, name) == 0) return &d;
  return nullptr;
}
}  // namespace
Options& options() {
  static Options o = make_options();
  return o;
}
}  // namespace snvrag

extern "C" int snvrag_set_option(const char* name, int64_t value) {
  const snvrag::OptDesc* d = snvrag::find_opt(name);
  if (!d) return fail(__func__, std::string("unknown option ") + (name ? name : "(null)"));
  snvrag::options().*(d->field) = value;
  return 0;
}

extern "C" int snvrag_get_option(const char* name, int64_t* value) {
  const snvrag::OptDesc* d = snvrag::find_opt(name);
  if (!d || !value) return fail(__func__, std::string("unknown option ") + (name ? name : "(null)"));
  *value = snvrag::options().*(d->field);
  return 0;
}

extern "C" int snvrag_abi_version(void) { return SNVRAG_ABI_VERSION; }
extern "C" const char* snvrag_last_error(void) { return g_err.c_str(); }

extern "C" int snvrag_device_info(int device, char* name, int name_len) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return -1;
  if (name && name_len > 0) {
    std::strncpy(name, p.gcnArchName, name_len - 1);
    name[name_len - 1] = 0;
  }
  return p.multiProcessorCount;
}

extern "C" int snvrag_evlog_enable(int capacity) {
  if (g_ev.ev) {
    for (int i = 0; i < 2 * g_ev.cap; ++i) (void)hipEventDestroy(g_ev.ev[i]);
    delete[] g_ev.ev; delete[] g_ev.kind; delete[] g_ev.work;
    g_ev = EvLog{};
  }
  if (capacity <= 0) return 0;
  g_ev.ev = new hipEvent_t[2 * capacity];
  g_ev.kind = new int[capacity];
  g_ev.work = new double[capacity];
  for (int i = 0; i < 2 * capacity; ++i) SNV_HIP(hipEventCreate(&g_ev.ev[i]));
  g_ev.cap = capacity;
  g_ev.n = 0;
  g_ev.on = true;
  return 0;
}

extern "C" int snvrag_evlog_pause(int paused) { g_ev.on = !paused && g_ev.cap > 0; return 0; }
extern "C" int snvrag_evlog_reset(void) { g_ev.n = 0; return 0; }

extern "C" int snvrag_evlog_read(int* kinds, float* ms, double* work, int max) {
  const int n = g_ev.n < max ? g_ev.n : max;
  for (int i = 0; i < n; ++i) {
    SNV_HIP(hipEventSynchronize(g_ev.ev[2 * i + 1]));
    float t = 0.f;
    SNV_HIP(hipEventElapsedTime(&t, g_ev.ev[2 * i], g_ev.ev[2 * i + 1]));
    kinds[i] = g_ev.kind[i];
    ms[i] = t;
    work[i] = g_ev.work[i];
  }
  return n;
}

extern "C" int snvrag_selftest_mfma(void* stream) {
  int* d = nullptr;
  SNV_HIP(hipMalloc(&d, sizeof(int)));
  hipStream_t s = as_stream(stream);
  SNV_HIP(hipMemsetAsync(d, 0, sizeof(int), s));
  hipLaunchKernelGGL(mfma_selftest_kernel, dim3(1), dim3(64), 0, s, d);
  int h = -1;
  SNV_HIP(hipMemcpyAsync(&h, d, sizeof(int), hipMemcpyDeviceToHost, s));
  SNV_HIP(hipStreamSynchronize(s));
  SNV_HIP(hipFree(d));
  return h;
}
