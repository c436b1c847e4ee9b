// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of libsnvrag.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>
#include <type_traits>

// the inline-asm LDS-DMA (dma_x4) names m0, which the compiler reserves: it rematerialises m0
// before each of its own uses, so the clobber is safe here
#pragma clang diagnostic ignored "-Winline-asm"

#include "../../include/snvrag.h"

namespace snvrag {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

void set_error(const std::string& msg);

// ---- event log (bench.py live per-kernel timing; off by default) ----
enum EvKind { EV_GEMM = 1, EV_ATTN = 2, EV_LN = 3, EV_KNN_SCAN = 4, EV_KNN_LUT = 5, EV_MERGE = 6, EV_OTHER = 7, EV_BLOCK = 8,
              EV_ATTN_BWD = 10, EV_TRAIN = 11 };
bool evlog_on();
void evlog_begin(hipStream_t s);
void evlog_end(hipStream_t s, int kind, double work);
int fail(const char* where, const std::string& msg);

#define SNV_CHECK_ARG(cond, msg)                                     \
  do {                                                               \
    if (!(cond)) return ::snvrag::fail(__func__, (msg));             \
  } while (0)

#define SNV_HIP(expr)                                                \
  do {                                                               \
    hipError_t e_ = (expr);                                          \
    if (e_ != hipSuccess)                                            \
      return ::snvrag::fail(__func__, hipGetErrorString(e_));        \
  } while (0)

// launch + error check (kernel launch errors surface via hipGetLastError)
#define SNV_LAUNCH_CHECK()                                           \
  do {                                                               \
    hipError_t e_ = hipGetLastError();                               \
    if (e_ != hipSuccess)                                            \
      return ::snvrag::fail(__func__, hipGetErrorString(e_));        \
  } while (0)

// Library options: tuning switches of the micro-benchmarks (tools/) and test hooks.  Each is
// initialised ONCE from the environment variable SNVRAG_<NAME> (upper case) at first use and can
// be changed through snvrag_set_option; launch paths read this struct, never the environment.
struct Options {
  int64_t knn_no_reduce;   // 1: the kNN scan always runs both int8 limbs (test: == the reduced scan)
  int64_t scan_mode;       // scan2 pipeline variant (tools/knn_probe.py), 0 = default
  int64_t scan_nt;         // -1 auto (non-temporal code stream when one query group reads it), 0 / 1
  int64_t unfused_ln;      // 1: the encoder without the fused block tail (test: fused == unfused)
  int64_t encoder_chunk;   // sequences per encoder chunk, 0 = auto
  int64_t gemm_tile128;    // 1: the 128-tile GEMM instead of the row-panel GEMM (tools/gemm_micro.py)
  int64_t gemm_nw;         // row-panel GEMM tile width (1, 2, 4, 6 x 64 columns), 0 = auto
  int64_t tail_variant;    // block-tail diagnostic instantiation (tools/tail_micro.py), 0 = default
  int64_t tail_desync;     // block-tail first-round stagger in cycles, -1 = auto
  int64_t sg_desync;       // stream-GEMM first-round stagger in cycles, -1 = auto
  int64_t mlp_desync;      // MLP kernel first-round stagger in cycles, -1 = auto
  int64_t g2_desync;       // wide-row GEMM first-round stagger in cycles, -1 = auto
  int64_t sg_waves4;       // 1: 4-wave stream GEMM for the rank-free projections (A/B)
  int64_t ln_bwd_nopf;     // 1: LayerNorm backward without the next-row prefetch (A/B)
  int64_t attn_variant;    // inference attention (dh 32) A/B variant, 0 = default (attention.hip tile)
  int64_t dw_xcd;          // 1: dW workgroups of one M chunk dealt to one XCD (0: plain grid order, A/B)
  int64_t ln_rows1;        // 1: training LayerNorm forward one row per wave also at N <= 512 (A/B)
  int64_t g2_groups;       // wide-row GEMM token groups per workgroup (4 .. 8; 0: by M)
  int64_t g2_variant;      // wide-row GEMM diagnostics: 1 no LDS-DMA, 2 no MFMA (wrong results; timing only),
                           // 3 stamps into the snvrag_tail_stamps buffer
  int64_t tail_persist;    // 1: the persistent block tail (tailp_kernel, A/B); 0 (default): tail_kernel
  int64_t tail_split;      // wide-row tail: split a last partial round of <= this many 128-row tiles into 32-row tiles (0: off)
  int64_t proj_wide;       // 1 (default): snvrag_proj_forward at D = 384 on the wide-row projection (tailw.hip,
                           // 0.62 vs 0.68 ms, bit-identical); 0: tail.hip PROJ mode
  int64_t tail_wide;       // block tail at D = 384 (PRE): 1 (default) the wide-row form (tailw.hip), 0 tail_kernel,
                           // 2 the wide-row form with phase stamps into the snvrag_tail_stamps buffer
};
Options& options();
// the diagnostic stamp buffer set by snvrag_tail_stamps (null unless a tool set one)
unsigned long long* diag_stamps();

// the wide-row block tail (tailw.hip), D = 384, PRE mode (out = LN2(FFN(LN1(x + att W_o^T))) in place)
int tailw_launch(int M, const void* att, const void* resid, void* out, const void* ws, const float* vec,
                 const float* b_o, const float* g1, const float* be1, float eps, int desync, int var, hipStream_t s);

// the wide-row projection (tailw.hip), D = 384: out[M, NC D] = x W^T + b on a snvrag_proj_pack stream
int projw_launch(int M, int NC, const void* x, const void* ws, const float* bias, void* out, int desync, hipStream_t s);

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------ device --
// A buffer resource (V#) in four SGPRs for the inline-asm LDS-DMA below: base, stride 0,
// num_records = ``bytes`` (clamped to 2^31 - 1; reads past it return 0), dword 3 = 0x00020000
// (the same raw-buffer format __builtin_amdgcn_make_buffer_rsrc is given in this library).
__device__ __forceinline__ i32x4 dma_rsrc(const void* base, long bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL));
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA of one 16-B piece per lane (1 KiB per wave): buffer_load_dwordx4 ... lds into the LDS
// bytes [lds, lds + 1024) (lane i -> lds + 16 i), source = base + voffset + soffset.  Issued by
// inline asm so that the compiler's waitcnt pass does not see an LDS store: with the builtin it
// treats every later ds_read of the same __shared__ array as aliasing EVERY DMA in flight and
// inserts s_waitcnt vmcnt before it (e.g. vmcnt(0) before each tile's reads in a prefetch ring:
// the ring collapses to synchronous loads).  The caller owns the ordering: a counted
// s_waitcnt vmcnt (this wave's pieces) and a barrier (the other waves') before reading — and
// must retire any compiler-visible global load whose first use is inside the ring loop before
// the loop (asm volatile("" : "+v"(x))), or its wait lands in the loop as vmcnt(0).
// ``lds`` is the wave-uniform LDS byte address (lds_addr()).
__device__ __forceinline__ void dma_x4(const i32x4& rsrc, uint32_t lds, int voffset, int soffset) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds), "v"(voffset), "s"(rsrc), "s"(soffset)
               : "memory", "m0");
}
// LDS byte address of a pointer into a __shared__ array: the low 32 bits of its flat address
// (the shared aperture is the high dword), without the null check of an address-space cast
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)p);
}

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// exact-erf GELU x * Phi(x) without the branchy library erff: Phi from
// erfc(|x|/sqrt2) = t (a1 + t (a2 + ... a5 t)) exp(-x^2/2), t = 1 / (1 + p |x|/sqrt2)
// (Abramowitz & Stegun 7.1.26, |erfc error| <= 1.5e-7): one v_rcp + one v_exp and
// nine FMA-class ops, max |error| 4.2e-7 over R (library erff in f32: 4.5e-7).
__device__ __forceinline__ float gelu_erf(float x) {
  const float ax = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float q = fmaf(t, 1.061405429f, -1.453152027f);
  q = fmaf(t, q, 1.421413741f);
  q = fmaf(t, q, -0.284496736f);
  q = fmaf(t, q, 0.254829592f);
  q = t * q * __builtin_amdgcn_exp2f(ax * ax * -1.4426950408889634f);   // erfc(ax)
  return x * (x >= 0.f ? fmaf(-0.5f, q, 1.0f) : 0.5f * q);
}
// GELU for bf16-output epilogues: x * sigmoid(p(x)), p(x) = x (a + b x^2 + c x^4) a minimax
// fit to the exact-erf GELU with the argument clamped to |x| <= 8 (beyond it the sigmoid is
// 0 / 1 to f32 precision): max |error| 2.6e-5 over R, below a tenth of the bf16 output spacing
// wherever the error peaks (|y| ~ 0.1 at x ~ -1.3), and relative error -> 0 as x -> 0.
// One v_exp + one v_rcp and six FMA-class ops (gelu_erf: nine) — the GELU epilogues of the
// D -> 4D projections are VALU-issue bound.
__device__ __forceinline__ float gelu_bf16(float x) {
  constexpr float L2E = 1.4426950408889634f;
  const float xc = __builtin_amdgcn_fmed3f(x, -8.f, 8.f);
  const float x2 = xc * xc;
  const float z = xc * fmaf(x2, fmaf(x2, 7.03033577e-4f * L2E, -7.40112920e-2f * L2E), -1.59501577f * L2E);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ float apply_act(int act, float x, float slope) {
  switch (act) {
    case SNVRAG_ACT_GELU: return gelu_erf(x);
    case SNVRAG_ACT_LRELU: return x >= 0.f ? x : x * slope;
    case SNVRAG_ACT_SIGMOID: return 1.0f / (1.0f + expf(-x));
    default: return x;
  }
}
// activation of an epilogue whose output is rounded to TO (bf16: the fast GELU)
template <typename TO> __device__ __forceinline__ float apply_act_t(int act, float x, float slope) {
  if constexpr (std::is_same<TO, bf16>::value) {
    if (act == SNVRAG_ACT_GELU) return gelu_bf16(x);
  }
  return apply_act(act, x, slope);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Sum over aligned groups of W (2/4/8/16) consecutive lanes, result in every lane of the
// group; DPP lane moves (quad_perm xor1/xor2, row_half_mirror, row_mirror) instead of
// ds_bpermute round trips through the LDS.
template <int CTRL> __device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int W> __device__ __forceinline__ float group_sum(float v) {
  static_assert(W == 2 || W == 4 || W == 8 || W == 16, "group width");
  v += dpp_mov<0xB1>(v);                    // quad_perm [1,0,3,2]
  if constexpr (W >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (W >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: quad q <-> 1-q
  if constexpr (W >= 16) v += dpp_mov<0x140>(v); // row_mirror: half h <-> 1-h
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace snvrag
