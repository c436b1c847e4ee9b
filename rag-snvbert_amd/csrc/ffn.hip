// Fused FFN sublayer as ONE kernel (bf16, eval):
//
//   h   = lrelu(x1 W1^T + b1)                           feed_forward.py:20 (w_1, LeakyReLU 0.1)
//   out = LN2(x1 + lrelu(LN_f(h) W2^T + b2))            feed_forward.py:20-21, sublayer.py:15-16
//
// The [M, 4D] hidden never reaches HBM.  A workgroup owns 128 token rows (4 waves
// x 32 rows, one wave per SIMD).  Each wave's x1 rows sit in LDS in MFMA B-operand
// order (96 KiB at D = 384); the weights stream once per workgroup through a
// 4-slot LDS ring of 16 KiB slabs (LDS-DMA, three slabs in flight across raw
// barriers).  Every MFMA computes a TRANSPOSED tile (weight rows x token rows), so
// a lane ends up holding one token row's values:
//   * phase 1 (W1):  h^T   = W1_c . x1^T       per 64-wide hidden chunk c;
//   * phase 2 (W2):  out^T += W2'_c . h_c^T     with h_c^T taken straight from the
//                    phase-1 accumulators (bf16), its k order baked into W2'.
// The FFN LayerNorm over the 4D hidden is folded: with
// W2' = W2 diag(g_f), c1 = rowsum(W2') and b2' = b2 + W2 b_f,
//   LN_f(h) W2^T + b2 = rstd*(h W2'^T) - rstd*mean*c1 + b2',
// mean/rstd from per-lane running sums of h (f32, before bf16 rounding).
// W2' rows are permuted so lane (li, lg) holds output columns 32s + 8lg + j (j < 8):
// residual, LayerNorm and the 16-byte stores work on whole 8-column runs of one
// row, and the row reductions are two lane shuffles.
//
// PRE variant (snvrag_block_tail_forward): the attention output projection runs in
// the same workgroup first, x1 = LN1(x + att W_o^T + b_o), from att rows staged in
// the x1 LDS tile and a W_o' stream (18 slabs at D = 384, phase-2 format) ahead of
// the FFN stream; x1 is written over att in LDS and never reaches HBM.
#include "common.h"

namespace snvrag {

constexpr int FF_SLAB = 16384;   // bytes per weight slab = 16 fragment blocks of 1 KiB
constexpr int FF_NSLOT = 4;      // LDS ring slots
constexpr int FF_PD = 3;         // slabs in flight (<= NSLOT - 1)

// vector table (f32) offsets, in units of D: b1[4D] b2' c1 g2 be2
enum { FV_B1 = 0, FV_B2 = 4, FV_C1 = 5, FV_G2 = 6, FV_BE2 = 7, FV_N = 8 };

// output column held by A-row r (0..15) of 16-row weight tile T (see header comment)
__host__ __device__ constexpr int ffn_perm(int T, int r) { return 32 * (T >> 1) + 8 * (r >> 2) + 4 * (T & 1) + (r & 3); }

template <int D> struct FfnShape {
  static constexpr int KS = D / 32;              // 32-wide k steps over D
  static constexpr int NT = D / 16;              // 16-wide column tiles over D
  static constexpr int NB = D / 128;             // 128-wide blocks (W1 k blocks / W2 column blocks)
  static constexpr int NCH = 4 * D / 64;         // 64-wide hidden chunks
  static constexpr int SPC = 2 * NB;             // slabs per hidden chunk (W1 then W2)
  static constexpr int NSLAB = NCH * SPC;
  static constexpr int XT = 4 * 2 * KS * 1024;   // x1 tile bytes in LDS
  static constexpr int LDS = XT + FF_NSLOT * FF_SLAB;
};

__device__ __forceinline__ void ff_glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
// streaming (read-once) rows: non-temporal, so they do not push the weight stream out of L2
__device__ __forceinline__ void ff_glds16_nt(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 2);
}

// wait until at most `younger` (<= MAXY) slabs (BPW LDS-DMA instructions each) of this wave
// are still in flight
template <int BPW, int MAXY> __device__ __forceinline__ void ff_wait(int younger) {
  static_assert(BPW * MAXY <= 63, "vmcnt range");
  if constexpr (MAXY <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (younger >= MAXY) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BPW * MAXY) : "memory");
      return;
    }
    ff_wait<BPW, MAXY - 1>(younger);
  }
}

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  bf16 x = (bf16)a, y = (bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}
// element j (0..7) of a bf16x8 held as u32x4
__device__ __forceinline__ float bfx(const u32x4& v, int j) { return (j & 1) ? bf_hi(v[j >> 1]) : bf_lo(v[j >> 1]); }

__device__ __forceinline__ f32x4 mfma_bf16(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// RT 16-row tiles per wave, NWV waves: RT = 2, NWV = 4 (one wave per SIMD, 512 registers)
// or RT = 1, NWV = 8 (two waves per SIMD, 256 registers each); 128 rows either way.
struct FfnPre {            // PRE: x1 = LN1(resid + att W_o^T + b_o)
  const bf16* resid; const char* wo; const float* b_o; const float* g1; const float* be1;
};

// G: slabs per wait+barrier (1: three slabs in flight, slab-wise; 2, 4: G landed, G in flight).
// XREG: this wave's x1 (and, PRE, att) rows live in VGPRs instead of LDS; the whole LDS is ring.
// SLOTS: ring slots for G = 1 (SLOTS - 1 slabs in flight); WPE: waves per SIMD the register
// budget is sized for (2 with NWV = 4 means two workgroups per CU).
template <int D, int RT, int NWV, int DBG, bool PRE = false, bool PRIO = false, int G = 1, bool XREG = false,
          bool NTS = false, int SLOTS = FF_NSLOT, int WPE = NWV / 4>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void ffn_kernel(int M, const bf16* __restrict__ x1, bf16* out, const char* __restrict__ ws,
                const float* __restrict__ vec, float eps, FfnPre pre) {
  using S = FfnShape<D>;
  constexpr int KS = S::KS, NT = S::NT, NB = S::NB;
  constexpr int NCHP = PRE ? D / 64 : 0;           // W_o' chunks (64 k each) ahead of the FFN stream
  constexpr int NPRE = NCHP * NB;
  constexpr int NSLAB = NPRE + S::NSLAB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  constexpr int BPW = 16 / NWV;                    // 1-KiB blocks of a slab loaded per wave
  constexpr int ROWS = RT * 16 * NWV;
  constexpr int PD = SLOTS - 1;
  const long rbase = (long)blockIdx.x * ROWS + wave * 16 * RT;
  // this wave's x1 rows, B-operand fragment blocks [rt][s], lane-linear 16 B each
  char* xt = smem + wave * (RT * KS * 1024);
  const char* xtl = xt + lane * 16;
  char* ring = smem + (XREG ? 0 : NWV * RT * KS * 1024);
  constexpr int NSLOT = G == 1 ? SLOTS : 2 * G;
  u32x4 xr[XREG ? RT : 1][XREG ? KS : 1];
  // B operand block idx (32 k) of row tile rt: registers or the LDS tile
  auto xb = [&](int rt, int idx) -> u32x4 {
    if constexpr (XREG) return xr[rt][idx];
    else return *reinterpret_cast<const u32x4*>(xtl + (rt * KS + idx) * 1024);
  };

#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const long r = min(rbase + rt * 16 + li, (long)M - 1);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if constexpr (XREG) xr[rt][s] = *reinterpret_cast<const u32x4*>(x1 + r * D + 32 * s + 8 * lg);
      else if constexpr (NTS) ff_glds16_nt(x1 + r * D + 32 * s + 8 * lg, xt + (rt * KS + s) * 1024);
      else ff_glds16(x1 + r * D + 32 * s + 8 * lg, xt + (rt * KS + s) * 1024);
    }
  }

  // Workgroups start at different hidden chunks (the FFN sums over chunks, so any
  // order is the same sum): concurrent CUs of an XCD then read different slabs
  // instead of all hitting the same L2 channels with the same 16 KiB.
  const int rot = (int)(blockIdx.x % S::NCH);
  const int rotp = (PRE && !XREG) ? (int)(blockIdx.x % (NCHP > 0 ? NCHP : 1)) : 0;
  auto issue = [&](int i) {
    if (DBG != 1 && i < NSLAB) {
      const char* src;
      if (PRE && i < NPRE) {
        int cc = i / NB + rotp;
        cc = cc >= NCHP ? cc - NCHP : cc;
        src = pre.wo + ((long)cc * NB + i % NB) * FF_SLAB + wave * BPW * 1024 + lane * 16;
      } else {
        const int k = i - NPRE;
        int cc = k / S::SPC + rot;
        cc = cc >= S::NCH ? cc - S::NCH : cc;
        src = ws + ((long)cc * S::SPC + k % S::SPC) * FF_SLAB + wave * BPW * 1024 + lane * 16;
      }
      char* dst = ring + (i % NSLOT) * FF_SLAB + wave * BPW * 1024;
#pragma unroll
      for (int j = 0; j < BPW; ++j) ff_glds16(src + j * 1024, dst + j * 1024);
    }
  };
  // slab i landed for every wave (and, at i = 0, this wave's x1 rows), slab i-1's slot
  // free; then keep FF_PD slabs in flight
  // PAIR: one wait + barrier per two slabs (slabs i, i+1 landed; i+2, i+3 go into the
  // slots of i-2, i-1), so a wave's LDS reads of the second slab overlap the MFMAs of
  // the first; two slabs in flight instead of three.
  auto step = [&](int i) -> const char* {
    if constexpr (G > 1) {
      if (i % G == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int g = 0; g < G; ++g) issue(i + G + g);
      }
    } else {
      if (DBG != 1) {
        ff_wait<BPW, PD - 1>(min(PD - 1, NSLAB - 1 - i));
        __builtin_amdgcn_s_barrier();
      }
      issue(i + PD);
    }
    return ring + (i % NSLOT) * FF_SLAB + lane * 16;
  };
#pragma unroll
  for (int i = 0; i < (G > 1 ? G : PD); ++i) issue(i);

  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  int slab = 0;
  if constexpr (PRE) {
    // ---- acc = att W_o'^T (att rows are this wave's LDS tile, k order of the x1 layout)
#pragma unroll
    for (int c0 = 0; c0 < NCHP; ++c0) {
      const int c = c0 + rotp >= NCHP ? c0 + rotp - NCHP : c0 + rotp;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const char* sl = step(slab++);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u32x4 a[8], b[RT];
#pragma unroll
          for (int t = 0; t < 8; ++t) a[t] = *reinterpret_cast<const u32x4*>(sl + (t * 2 + s2) * 1024);
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) b[rt] = xb(rt, 2 * c + s2);
          if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) acc[rt][nb * 8 + t] = mfma_bf16(a[t], b[rt], acc[rt][nb * 8 + t]);
          if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        }
      }
    }
    // ---- x1 = LN1(resid + acc + b_o) -> this wave's LDS tile (over att), acc reset
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const long r = min(rbase + rt * 16 + li, (long)M - 1);
      float sum = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const u32x4 rv = *reinterpret_cast<const u32x4*>(pre.resid + r * D + 32 * s + 8 * lg);
        const float* bo = pre.b_o + 32 * s + 8 * lg;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = acc[rt][2 * s + (j >> 2)][j & 3] + bo[j] + bfx(rv, j);
          acc[rt][2 * s + (j >> 2)][j & 3] = v;
          sum += v;
        }
      }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      const float mean = sum * (1.0f / D);
      float q = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) { const float d = acc[rt][t][i] - mean; q = fmaf(d, d, q); }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      const float rstd = 1.0f / sqrtf(q * (1.0f / D) + eps);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float* g = pre.g1 + 32 * s + 8 * lg;
        const float* b = pre.be1 + 32 * s + 8 * lg;
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (acc[rt][2 * s + (j >> 2)][j & 3] - mean) * rstd * g[j] + b[j];
        const u32x4 xv{pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]), pack_bf2(y[4], y[5]), pack_bf2(y[6], y[7])};
        if constexpr (XREG) xr[rt][s] = xv;
        else *reinterpret_cast<u32x4*>(xt + (rt * KS + s) * 1024 + lane * 16) = xv;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  float st1[RT], st2[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) st1[rt] = st2[rt] = 0.f;
#pragma unroll 1
  for (int c0 = 0; c0 < S::NCH; ++c0) {
    const int c = c0 + rot >= S::NCH ? c0 + rot - S::NCH : c0 + rot;
    float4 bias1[4];                                 // b1 of this chunk's hidden units (L2-resident)
#pragma unroll
    for (int t = 0; t < 4; ++t) bias1[t] = *reinterpret_cast<const float4*>(vec + FV_B1 * D + c * 64 + 16 * t + 4 * lg);
    f32x4 h[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) h[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {               // W1 slabs: 4 hidden tiles x 4 k steps
      const char* sl = step(slab++);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        u32x4 a[4], b[RT];
#pragma unroll
        for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const u32x4*>(sl + (t * 4 + s) * 1024);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) b[rt] = xb(rt, kb * 4 + s);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            if (DBG == 2) h[rt][t][0] += __builtin_bit_cast(float, a[t][0] ^ b[rt][0]);
            else h[rt][t] = mfma_bf16(a[t], b[rt], h[rt][t]);
          }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      }
    }
    // bias + LeakyReLU(0.1) + LN_f running sums; pack h^T as phase-2 B operands
    u32x4 hf[RT][2];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float hv[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float bb[4] = {bias1[t].x, bias1[t].y, bias1[t].z, bias1[t].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = h[rt][t][i] + bb[i];
          v = v >= 0.f ? v : 0.1f * v;
          st1[rt] += v;
          st2[rt] = fmaf(v, v, st2[rt]);
          hv[t][i] = v;
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        hf[rt][s2] = u32x4{pack_bf2(hv[2 * s2][0], hv[2 * s2][1]), pack_bf2(hv[2 * s2][2], hv[2 * s2][3]),
                           pack_bf2(hv[2 * s2 + 1][0], hv[2 * s2 + 1][1]),
                           pack_bf2(hv[2 * s2 + 1][2], hv[2 * s2 + 1][3])};
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {               // W2' slabs: 8 column tiles x 2 k steps
      const char* sl = step(slab++);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 a[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) a[t] = *reinterpret_cast<const u32x4*>(sl + (t * 2 + s2) * 1024);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            if (DBG == 2) acc[rt][nb * 8 + t][0] += __builtin_bit_cast(float, a[t][0] ^ hf[rt][s2][0]);
            else acc[rt][nb * 8 + t] = mfma_bf16(a[t], hf[rt][s2], acc[rt][nb * 8 + t]);
          }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      }
    }
  }

  // ---------------- epilogue: out = LN2(x1 + lrelu(rstd*acc - rstd*mean*c1 + b2'))
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float s1 = st1[rt], s2 = st2[rt];
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const float hm = s1 * (1.0f / (4 * D));
    const float hr = 1.0f / sqrtf(fmaxf(s2 * (1.0f / (4 * D)) - hm * hm, 0.f) + eps);
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const u32x4 xrs = xb(rt, s);
      const float* c1 = vec + FV_C1 * D + 32 * s + 8 * lg;
      const float* b2 = vec + FV_B2 * D + 32 * s + 8 * lg;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float u = hr * acc[rt][2 * s + (j >> 2)][j & 3] - hr * hm * c1[j] + b2[j];
        u = u >= 0.f ? u : 0.1f * u;
        const float v = u + bfx(xrs, j);
        acc[rt][2 * s + (j >> 2)][j & 3] = v;
        sum += v;
      }
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float mean = sum * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) { const float d = acc[rt][t][i] - mean; q = fmaf(d, d, q); }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rstd = 1.0f / sqrtf(q * (1.0f / D) + eps);
    const long r = rbase + rt * 16 + li;
    if (r < M) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float* g = vec + FV_G2 * D + 32 * s + 8 * lg;
        const float* b = vec + FV_BE2 * D + 32 * s + 8 * lg;
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (acc[rt][2 * s + (j >> 2)][j & 3] - mean) * rstd * g[j] + b[j];
        const u32x4 ov{pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]), pack_bf2(y[4], y[5]), pack_bf2(y[6], y[7])};
        if constexpr (NTS) __builtin_nontemporal_store(ov, reinterpret_cast<u32x4*>(out + r * D + 32 * s + 8 * lg));
        else *reinterpret_cast<u32x4*>(out + r * D + 32 * s + 8 * lg) = ov;
      }
    }
  }
}

// one thread per 16-byte piece of the stream: per hidden chunk, NB W1 slabs
// (block t*4+s: W1[hidden 16t+li][k 128kb+32s+8lg..]) then NB W2' slabs (block
// t*2+s2: W2'[perm(8nb+t, li)][hidden 32s2 + 16(j/4) + 4lg + j%4, j < 8])
__global__ void ffn_pack_kernel(int D, long n_pieces, const bf16* __restrict__ w1, const bf16* __restrict__ w2g,
                                bf16* __restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pieces) return;
  const int NB = D / 128, SPC = 2 * NB;
  const long slab = p / 1024;
  const int b = (int)((p / 64) % 16), L = (int)(p % 64), li = L & 15, lg = L >> 4;
  const int c = (int)(slab / SPC), r = (int)(slab % SPC);
  bf16 v[8];
  if (r < NB) {
    const int t = b / 4, s = b % 4;
    const long hid = (long)c * 64 + 16 * t + li;
    const int k0 = r * 128 + 32 * s + 8 * lg;
    for (int j = 0; j < 8; ++j) v[j] = w1[hid * D + k0 + j];
  } else {
    const int nb = r - NB, t = b / 2, s2 = b % 2;
    const int n = ffn_perm(nb * 8 + t, li);
    for (int j = 0; j < 8; ++j) {
      const long hid = (long)c * 64 + 32 * s2 + 16 * (j >> 2) + 4 * lg + (j & 3);
      v[j] = w2g[(long)n * 4 * D + hid];
    }
  }
  for (int j = 0; j < 8; ++j) out[p * 8 + j] = v[j];
}

// W_o' stream of the PRE variant: per 64-k chunk c, NB slabs; block t*2+s2 of slab
// (c, nb): W_o[perm(8nb+t, li)][64c + 32s2 + 8lg + j]
__global__ void ffn_pre_pack_kernel(int D, long n_pieces, const bf16* __restrict__ wo, bf16* __restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pieces) return;
  const int NB = D / 128;
  const long slab = p / 1024;
  const int b = (int)((p / 64) % 16), L = (int)(p % 64), li = L & 15, lg = L >> 4;
  const int c = (int)(slab / NB), nb = (int)(slab % NB), t = b / 2, s2 = b % 2;
  const int n = ffn_perm(nb * 8 + t, li);
  const long k0 = (long)c * 64 + 32 * s2 + 8 * lg;
  for (int j = 0; j < 8; ++j) out[p * 8 + j] = wo[(long)n * D + k0 + j];
}

static bool ffn_d_ok(int D) { return D == 128 || D == 256 || D == 384; }

// variant (SNVRAG_FFN_VARIANT): 0 = slab-wise ring (3 in flight), x1 in LDS; 1 = slab pairs, x1 in
// LDS (default); 2 = 4-slab groups, x1 in VGPRs; 4 = 4 waves x 16 rows, two workgroups per CU
static int ffn_variant() {
  const char* e = getenv("SNVRAG_FFN_VARIANT");
  return e ? atoi(e) : 1;
}

template <int D, bool PRE, int NWV, int G, bool XREG, bool NTS, int SLOTS, int WPE, int RT = 1>
static int launch_ffn_k(int64_t M, const void* x1, void* out, const void* ws, const float* vec, float eps,
                        const FfnPre& pre, hipStream_t s) {
  auto kern = ffn_kernel<D, RT, NWV, 0, PRE, true, G, XREG, NTS, SLOTS, WPE>;
  constexpr int KS = D / 32;
  const size_t ring = (size_t)(G == 1 ? SLOTS : 2 * G) * FF_SLAB;
  const size_t lds = XREG ? ring : (size_t)NWV * RT * KS * 1024 + ring;
  static_assert((XREG ? 0 : NWV * RT * KS * 1024) + (G == 1 ? SLOTS : 2 * G) * FF_SLAB <= 160 * 1024, "LDS budget");
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(M, 16 * NWV * RT)), dim3(64 * NWV), lds, s, (int)M, (const bf16*)x1,
                     (bf16*)out, (const char*)ws, vec, eps, pre);
  SNV_LAUNCH_CHECK();
  return 0;
}

template <int D, bool PRE>
static int launch_ffn_v(int64_t M, const void* x1, void* out, const void* ws, const float* vec, float eps,
                        const FfnPre& pre, hipStream_t s) {
  switch (ffn_variant()) {
    case 0: return launch_ffn_k<D, PRE, 8, 1, false, false, 4, 2>(M, x1, out, ws, vec, eps, pre, s);
    // measured slower at D = 384, M = 527 360 (tools/gemm_micro.py): x1 in VGPRs with 4-slab groups (+3 %),
    // 64-row workgroups two per CU (+4 %: the weight stream is read twice as often)
    case 2: return launch_ffn_k<D, PRE, 8, 4, true, false, 4, 2>(M, x1, out, ws, vec, eps, pre, s);
    case 4: return launch_ffn_k<D, PRE, 4, 1, false, false, 2, 2>(M, x1, out, ws, vec, eps, pre, s);
    // x1 in VGPRs, the whole LDS a slab-wise ring: 8 / 6 slabs (128 / 96 KiB) in flight
    case 5: return launch_ffn_k<D, PRE, 8, 1, true, false, 9, 2>(M, x1, out, ws, vec, eps, pre, s);
    case 6: return launch_ffn_k<D, PRE, 8, 1, true, false, 7, 2>(M, x1, out, ws, vec, eps, pre, s);
    // one wave per SIMD, two 16-row tiles per wave (each A fragment read from LDS feeds two MFMAs)
    case 7: return launch_ffn_k<D, PRE, 4, 1, false, false, 4, 1, 2>(M, x1, out, ws, vec, eps, pre, s);
    case 8: return launch_ffn_k<D, PRE, 4, 2, false, false, 4, 1, 2>(M, x1, out, ws, vec, eps, pre, s);
    // ... with x1 in VGPRs and a deep slab-wise ring
    case 9: return launch_ffn_k<D, PRE, 4, 1, true, false, 9, 1, 2>(M, x1, out, ws, vec, eps, pre, s);
    default: return launch_ffn_k<D, PRE, 8, 2, false, false, 4, 2>(M, x1, out, ws, vec, eps, pre, s);
  }
}

template <int D>
static int launch_ffn(int64_t M, const void* x1, void* out, const void* ws, const float* vec, float eps, hipStream_t s) {
  return launch_ffn_v<D, false>(M, x1, out, ws, vec, eps, FfnPre{}, s);
}

template <int D>
static int launch_ffn_pre(int64_t M, const void* att, void* x, const void* ws, const float* vec, float eps,
                          const FfnPre& pre, hipStream_t s) {
  return launch_ffn_v<D, true>(M, att, x, ws, vec, eps, pre, s);
}

}  // namespace snvrag

using namespace snvrag;

extern "C" size_t snvrag_ffn_pack_bytes(int D) {
  switch (D) {
    case 128: return (size_t)FfnShape<128>::NSLAB * FF_SLAB;
    case 256: return (size_t)FfnShape<256>::NSLAB * FF_SLAB;
    case 384: return (size_t)FfnShape<384>::NSLAB * FF_SLAB;
    default: return 0;
  }
}

extern "C" int snvrag_ffn_pack(int D, const void* w1, const void* w2g, void* out, void* stream) {
  SNV_CHECK_ARG(ffn_d_ok(D), "fused FFN needs D in {128, 256, 384}");
  SNV_CHECK_ARG(w1 && w2g && out, "null pointer");
  const long pieces = (long)(snvrag_ffn_pack_bytes(D) / 16);
  hipLaunchKernelGGL(ffn_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), D, pieces,
                     (const bf16*)w1, (const bf16*)w2g, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_ffn_forward(int64_t M, int D, const void* x1, void* out, const void* wstream,
                                  const float* vec, float eps, void* stream) {
  SNV_CHECK_ARG(ffn_d_ok(D), "fused FFN needs D in {128, 256, 384}");
  SNV_CHECK_ARG(x1 && out && wstream && vec, "null pointer");
  SNV_CHECK_ARG(x1 != out, "x1 and out must not alias");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)x1 % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)wstream % 16) == 0 &&
                    ((uintptr_t)vec % 16) == 0,
                "x1/out/wstream/vec must be 16-byte aligned");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  int rc;
  switch (D) {
    case 128: rc = launch_ffn<128>(M, x1, out, wstream, vec, eps, s); break;
    case 256: rc = launch_ffn<256>(M, x1, out, wstream, vec, eps, s); break;
    default: rc = launch_ffn<384>(M, x1, out, wstream, vec, eps, s); break;
  }
  if (rc) return rc;
  evlog_end(s, EV_BLOCK, 2.0 * M * (double)D * D * 8);
  return 0;
}

extern "C" size_t snvrag_ffn_pre_pack_bytes(int D) {
  return ffn_d_ok(D) ? (size_t)(D / 64) * (D / 128) * FF_SLAB : 0;
}

extern "C" int snvrag_ffn_pre_pack(int D, const void* w_o, void* out, void* stream) {
  SNV_CHECK_ARG(ffn_d_ok(D), "fused block tail needs D in {128, 256, 384}");
  SNV_CHECK_ARG(w_o && out, "null pointer");
  const long pieces = (long)(snvrag_ffn_pre_pack_bytes(D) / 16);
  hipLaunchKernelGGL(ffn_pre_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), D,
                     pieces, (const bf16*)w_o, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_block_tail_forward(int64_t M, int D, const void* att, void* x, const void* wo_stream,
                                         const float* b_o, const float* ln1_g, const float* ln1_b,
                                         const void* ffn_stream, const float* ffn_vec, float eps, void* stream) {
  SNV_CHECK_ARG(ffn_d_ok(D), "fused block tail needs D in {128, 256, 384}");
  SNV_CHECK_ARG(att && x && wo_stream && b_o && ln1_g && ln1_b && ffn_stream && ffn_vec, "null pointer");
  SNV_CHECK_ARG(att != x, "att and x must not alias");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)att % 16) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)wo_stream % 16) == 0 &&
                    ((uintptr_t)ffn_stream % 16) == 0 && ((uintptr_t)ffn_vec % 16) == 0 && ((uintptr_t)b_o % 16) == 0 &&
                    ((uintptr_t)ln1_g % 16) == 0 && ((uintptr_t)ln1_b % 16) == 0,
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const FfnPre pre{(const bf16*)x, (const char*)wo_stream, b_o, ln1_g, ln1_b};
  evlog_begin(s);
  int rc;
  switch (D) {
    case 128: rc = launch_ffn_pre<128>(M, att, x, ffn_stream, ffn_vec, eps, pre, s); break;
    case 256: rc = launch_ffn_pre<256>(M, att, x, ffn_stream, ffn_vec, eps, pre, s); break;
    default: rc = launch_ffn_pre<384>(M, att, x, ffn_stream, ffn_vec, eps, pre, s); break;
  }
  if (rc) return rc;
  evlog_end(s, EV_BLOCK, 2.0 * M * (double)D * D * 9);
  return 0;
}
