// Reference-panel kNN on the HBM-resident token index (gfx950).
//
// Replaces the reference's per-window fp32 embedding index + torch.cdist/topk
// (src/dataset/embedding_rag_dataset.py:334-402) and the FAISS IndexFlatL2 of
// inference (embedding_rag_infer_dataset.py:176, :279-285).  Because the
// embedding is position-wise, dist^2(q,r) = C_q + sum_s Delta_q[s] * a_r[s]
// (a_r[s] in {0,1}: allele of panel haplotype r at window site s), so the index
// is the panel's allele codes (1 B / site / haplotype) and the per-query work
// is a length-n_sites LUT.  DESIGN.md §3 has the derivation and the canonical
// (distance, index) order these kernels reproduce bit-exactly.
//
//   lut_kernel    : Delta in f32 -> per-query power-of-two fixed point -> int8
//                   limbs laid out in MFMA A-fragment order.
//   scan_kernel   : v_mfma_i32_16x16x64_i8 distance tiles (16 queries x 16
//                   haplotypes x 64 sites), codes streamed straight from HBM to
//                   VGPRs (no reuse to stage), exact per-range top-k kept in LDS
//                   with a strict-threshold filter + wave bitonic compaction.
//   merge_kernel  : hierarchical LDS bitonic merge of the per-range lists.
#include "common.h"

namespace snvrag {

constexpr uint64_t KEY_MAX = ~0ull;
constexpr int KEY_BIAS = 1 << 30;
constexpr int SCAN_CAP = 64;      // candidate slots per query per wave
constexpr int SCAN_TH = SCAN_CAP - 16;

__device__ __forceinline__ uint64_t make_key(int d, uint32_t idx) {
  return ((uint64_t)(uint32_t)(d + KEY_BIAS) << 32) | idx;
}

__device__ __forceinline__ int gcd_u(int a, int b) {   // a, b >= 0; gcd(0, b) = b
  uint32_t x = (uint32_t)a, y = (uint32_t)b;
  while (y) { const uint32_t t = x % y; x = y; y = t; }
  return (int)x;
}

// ------------------------------------------------------------------- LUT ---
// General-path Delta (query offsets A_q and/or panel offsets A_r: every position's squared
// distances need their own D-length reductions) spread over (position chunk of 64, query)
// workgroups: lut_kernel alone ran one workgroup per query, i.e. nq of 256 CUs at training's
// 48 queries (1.15 ms per step).  delta [nq][n_sites_pad] (sites), cpart [nq][nch]: the chunk's
// sum of the constant-term contributions (4 wave partials in fixed order: deterministic).
constexpr int LUT_CH = 64;
// chunk slots per query: a sequence may run past its window (training: 512 sites in a 1 030-token
// sequence, padding tokens after <eos>) and the last chunk takes every position past the grid, so
// the grid covers up to 2 n_sites_pad + 256 positions (with n_sites_pad / 64 + 4 slots that last
// chunk held 326 positions against 64 and set the launch time: 115 us per training step)
__host__ __device__ inline int lut_nch_max(int n_sites_pad) { return 2 * n_sites_pad / LUT_CH + 4; }

__global__ __launch_bounds__(256) void lut_delta_kernel(int L, int D, const int64_t* __restrict__ tok_q,
                                                        const float* __restrict__ W, const float* __restrict__ Wp,
                                                        const float* __restrict__ Aq,
                                                        long aq_period, const float* __restrict__ Ar,
                                                        const uint8_t* __restrict__ site_mask, int n_sites,
                                                        int n_sites_pad, int tok0, int tok1, int mask_tok,
                                                        float* __restrict__ delta, float* __restrict__ cpart) {
  const int c = blockIdx.x, q = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = lut_nch_max(n_sites_pad);
  const long arow = Aq ? ((aq_period > 0 ? q % aq_period : q) * (long)L) : 0;
  __shared__ float wc[4];
  float cacc = 0.f;
  // the last chunk also takes every position past the grid (padding tokens of a sequence longer
  // than the window: constant-term contributions only), so the grid is capped at nch
  const int lend = c == (int)gridDim.x - 1 ? L : min(L, (c + 1) * LUT_CH);
  // 16 lanes per position, 4 positions per wave, 16 per workgroup step: the D-length sums are
  // 4-step reductions inside the 16-lane group, 4 positions at a time (one position per wave with
  // three 6-step wave reductions each kept the loop latency-bound: 355 us per training step)
  const int g = lane >> 4, l16 = lane & 15;
  for (int base = c * LUT_CH; base < lend; base += 16) {
    const int l = base + 4 * wave + g;
    if (l >= lend) continue;                       // group-uniform: shuffles stay inside the group
    const int t = (int)tok_q[(long)q * L + l];
    const bool is_site = l >= 1 && l <= n_sites;
    const bool varying = is_site && !site_mask[l - 1];
    int rt;                                        // panel token at l when not varying
    if (l == 0) rt = 2; else if (is_site) rt = mask_tok; else if (l == n_sites + 1) rt = 3; else rt = 0;
    float t0 = 0.f, t1 = 0.f, tc = 0.f;
    for (int d = 4 * l16; d < D; d += 64) {
      f32x4 u = *reinterpret_cast<const f32x4*>(W + (long)t * D + d);
      if (Aq) u += *reinterpret_cast<const f32x4*>(Aq + (arow + l) * D + d);
      if (Ar) u -= *reinterpret_cast<const f32x4*>(Ar + (long)l * D + d);
      if (varying) {
        const f32x4 a = u - *reinterpret_cast<const f32x4*>(Wp + (long)tok0 * D + d);
        const f32x4 b = u - *reinterpret_cast<const f32x4*>(Wp + (long)tok1 * D + d);
#pragma unroll
        for (int e = 0; e < 4; ++e) { t0 = fmaf(a[e], a[e], t0); t1 = fmaf(b[e], b[e], t1); }
      } else {
        const f32x4 cc = u - *reinterpret_cast<const f32x4*>(Wp + (long)rt * D + d);
#pragma unroll
        for (int e = 0; e < 4; ++e) tc = fmaf(cc[e], cc[e], tc);
      }
    }
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      t0 += __shfl_xor(t0, o, 64);
      t1 += __shfl_xor(t1, o, 64);
      tc += __shfl_xor(tc, o, 64);
    }
    if (l16 == 0) {
      if (is_site) delta[(long)q * n_sites_pad + l - 1] = varying ? (t1 - t0) : 0.f;
      cacc += varying ? t0 : tc;
    }
  }
  cacc += __shfl_xor(cacc, 16, 64);                // the four groups' partials (zero off group leaders)
  cacc += __shfl_xor(cacc, 32, 64);
  if (lane == 0) wc[wave] = cacc;
  __syncthreads();
  if (threadIdx.x == 0) cpart[(long)q * nch + c] = (wc[0] + wc[1]) + (wc[2] + wc[3]);
}

// One workgroup per query.  Positions l = 0..L-1 contribute to the constant
// C_q; unmasked sites s (l = s + 1) contribute Delta_q[s].
__global__ __launch_bounds__(256) void lut_kernel(int L, int D, const int64_t* __restrict__ tok_q,
                                                  const float* __restrict__ W, const float* __restrict__ Wp,
                                                  const float* __restrict__ Aq,
                                                  long aq_period, const float* __restrict__ Ar,
                                                  const uint8_t* __restrict__ site_mask, int n_sites,
                                                  int n_sites_pad, int nq, int tok0, int tok1, int mask_tok,
                                                  int limbs, int8_t* __restrict__ lut, int* __restrict__ exps,
                                                  float* __restrict__ consts, const float* __restrict__ gdelta,
                                                  const float* __restrict__ gcpart) {
  extern __shared__ float sdelta[];              // [n_sites_pad] + [4] scratch
  float* red = sdelta + n_sites_pad;
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float cacc = 0.f;
  // Without AF terms u = W[t]: every squared distance depends on (token, panel token)
  // only, so the block tabulates them once (same lane order and wave_sum as the
  // per-position loop, hence identical values) for tokens < 8 and looks them up.
  __shared__ float tab[8][6];                     // [t][tok0, tok1, sos, eos, pad, mask]
  const bool fast = !Aq && !Ar;
  if (fast) {
    for (int e = wave; e < 48; e += 4) {
      const int t = e / 6, c = e % 6;
      const int rt = c == 0 ? tok0 : c == 1 ? tok1 : c == 2 ? 2 : c == 3 ? 3 : c == 4 ? 0 : mask_tok;
      float acc = 0.f;
      if (t < 7)
        for (int d = lane; d < D; d += 64) {
          const float a = W[(long)t * D + d] - Wp[(long)rt * D + d];
          acc = fmaf(a, a, acc);
        }
      acc = wave_sum(acc);
      if (lane == 0) tab[t][c] = acc;
    }
    __syncthreads();
  }
  bool done = false;
  if (fast) {
    // one position per thread; a token >= 7 anywhere sends the query to the general loop
    float cpart = 0.f;
    int odd = 0;
    for (int l = tid; l < L; l += 256) {
      const int t = (int)tok_q[(long)q * L + l];
      if (t >= 7 || t < 0) { odd = 1; continue; }
      const bool is_site = l >= 1 && l <= n_sites;
      const bool varying = is_site && !site_mask[l - 1];
      const int c = l == 0 ? 2 : is_site ? 5 : l == n_sites + 1 ? 3 : 4;
      if (is_site) sdelta[l - 1] = varying ? (tab[t][1] - tab[t][0]) : 0.f;
      cpart += varying ? tab[t][0] : tab[t][c];
    }
    done = !__syncthreads_or(odd);
    if (done) {
      cpart = wave_sum(cpart);
      if (lane == 0) cacc = cpart;
    }
  }
  if (!fast) {
    // general path: Delta and the constant's chunk sums from lut_delta_kernel
    for (int s = tid; s < n_sites; s += 256) sdelta[s] = gdelta[(long)q * n_sites_pad + s];
    if (tid == 0) {
      const int stride = lut_nch_max(n_sites_pad), nch = min((L + LUT_CH - 1) / LUT_CH, stride);
      for (int c = 0; c < nch; ++c) cacc += gcpart[(long)q * stride + c];
    }
  }
  // no offsets but a token outside the tabulated range: the per-position loop
  for (int l = wave; l < L && fast && !done; l += 4) {
    const int t = (int)tok_q[(long)q * L + l];
    const bool is_site = l >= 1 && l <= n_sites;
    const bool varying = is_site && !site_mask[l - 1];
    int rt;                                        // panel token at l when not varying
    if (l == 0) rt = 2; else if (is_site) rt = mask_tok; else if (l == n_sites + 1) rt = 3; else rt = 0;
    float t0 = 0.f, t1 = 0.f, tc = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float u = W[(long)t * D + d];
      if (varying) {
        const float a = u - Wp[(long)tok0 * D + d], b = u - Wp[(long)tok1 * D + d];
        t0 = fmaf(a, a, t0);
        t1 = fmaf(b, b, t1);
      } else {
        const float c = u - Wp[(long)rt * D + d];
        tc = fmaf(c, c, tc);
      }
    }
    t0 = wave_sum(t0); t1 = wave_sum(t1); tc = wave_sum(tc);
    if (lane == 0) {
      if (is_site) sdelta[l - 1] = varying ? (t1 - t0) : 0.f;
      cacc += varying ? t0 : tc;
    }
  }
  for (int s = n_sites + tid; s < n_sites_pad; s += 256) sdelta[s] = 0.f;
  if (lane == 0) red[wave] = cacc;
  __syncthreads();
  // block max |Delta|
  float mx = 0.f;
  for (int s = tid; s < n_sites; s += 256) mx = fmaxf(mx, fabsf(sdelta[s]));
  mx = wave_max(mx);
  __shared__ float wmax[4];
  __shared__ int sexp;
  if (lane == 0) wmax[wave] = mx;
  __syncthreads();
  const int qmax = (1 << (7 * limbs)) - 1;
  if (tid == 0) {
    const float m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    int e = 0;
    if (m > 0.f) {
      e = (int)floor(log2((double)qmax / (double)m));
      if ((double)m * exp2((double)e) > (double)qmax) e -= 1;
    }
    sexp = e;
    exps[q] = e;
    if (consts) consts[q] = red[0] + red[1] + red[2] + red[3];
  }
  __syncthreads();
  const float sc = exp2f((float)sexp);
  // quantise + scatter into fragment order: [qt][limb][ks][lane(64)][16]
  const int qt = q >> 4, qr = q & 15;
  const int KS = n_sites_pad / 64;
  auto quant = [&](int s) {
    float v = rintf(sdelta[s] * sc);
    v = fminf(fmaxf(v, (float)-qmax), (float)qmax);
    return (int)v;
  };
  auto frag = [&](int s) {               // offset of site s of this query inside one [ks][lane][16] plane
    const int ks = s >> 6, within = s & 63, g = within >> 4, j = within & 15;
    return ((long)ks * 64 + g * 16 + qr) * 16 + j;
  };
  int gl = 0;                            // gcd of the nonzero |dq| of this thread's sites
  for (int s = tid; s < n_sites_pad; s += 256) {
    const int dq = quant(s);
    if (limbs == 2) {
      const int hi = dq >> 7, lo = dq & 127;
      lut[((long)qt * 2 + 0) * KS * 1024 + frag(s)] = (int8_t)hi;
      lut[((long)qt * 2 + 1) * KS * 1024 + frag(s)] = (int8_t)lo;
      gl = gcd_u(gl, dq < 0 ? -dq : dq);
    } else {
      lut[(long)qt * KS * 1024 + frag(s)] = (int8_t)dq;
    }
  }
  if (limbs != 2) return;
  // 1-limb reduction: with g = gcd_s |dq_s|, D_2limb = g * sum_s (dq_s/g) a_r[s],
  // so when max |dq|/g fits int8 the scan may run one limb of dq/g and multiply by g —
  // identical integer distances, identical (distance, index) order.
  __shared__ int sg[4];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) gl = gcd_u(gl, __shfl_xor(gl, o, 64));
  if (lane == 0) sg[wave] = gl;
  __syncthreads();
  const int g = gcd_u(gcd_u(sg[0], sg[1]), gcd_u(sg[2], sg[3]));
  int8_t* lut1 = lut + (long)((nq + 15) >> 4) * 2 * KS * 1024;
  int* mult = reinterpret_cast<int*>(lut1 + (long)((nq + 15) >> 4) * KS * 1024);
  int* any_wide = mult + ((nq + 15) & ~15);
  bool fits = true;
  for (int s = tid; s < n_sites_pad; s += 256) {
    const int dq = quant(s);
    const int r = g ? dq / g : 0;
    fits &= r >= -127 && r <= 127;
    lut1[(long)qt * KS * 1024 + frag(s)] = (int8_t)r;
  }
  fits = __syncthreads_and(fits);
  if (tid == 0) {
    mult[q] = g;
    if (!fits) atomicOr(any_wide, 1);
  }
}

// padding rows of the last query tile must be zero
__global__ void lut_zero_pad_kernel(int8_t* lut, int nq, int KS, int limbs) {
  const int qt = nq >> 4, nqt = (nq + 15) >> 4;
  const long per_tile = (long)limbs * KS * 64 * 16;
  int8_t* lut1 = lut + (long)nqt * 2 * KS * 1024;      // one-limb region (limbs == 2)
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < per_tile; i += (long)gridDim.x * blockDim.x) {
    const int ln = (int)((i / 16) % 64);
    if ((ln & 15) >= (nq & 15)) {
      lut[qt * per_tile + i] = 0;
      if (limbs == 2 && i < per_tile / 2) lut1[(long)qt * KS * 1024 + i] = 0;
    }
  }
}

// ------------------------------------------------------------------ scan ---
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// ascending bitonic sort of one key per lane across the wave
__device__ __forceinline__ uint64_t wave_sort64(uint64_t key, int lane) {
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t other = shfl_xor64(key, stride);
      const bool up = (lane & size) == 0;
      const bool low = (lane & stride) == 0;
      const uint64_t mn = key < other ? key : other, mxv = key < other ? other : key;
      key = (low == up) ? mn : mxv;
    }
  }
  return key;
}

// compact the candidate list of query row `row` (wave-uniform) to its top-k.
__device__ __forceinline__ void compact_row(uint64_t* buf, int row, int cnt, int k, int lane,
                                            int& new_cnt, int& new_th) {
  uint64_t key = lane < cnt ? buf[row * SCAN_CAP + lane] : KEY_MAX;
  key = wave_sort64(key, lane);
  if (lane < k) buf[row * SCAN_CAP + lane] = key;
  new_cnt = cnt < k ? cnt : k;
  const uint64_t kth = shfl64(key, k - 1);
  new_th = (cnt >= k) ? (int)(kth >> 32) - KEY_BIAS : INT_MAX;
}

template <int KSMAX, int LIMBS>
__global__ __launch_bounds__(256) void scan_kernel(const uint8_t* __restrict__ codes, long n_ref, long ld,
                                                   int KS, const int8_t* __restrict__ lut, int nq, int k,
                                                   long range, long ref_offset, uint64_t* __restrict__ parts,
                                                   const int* __restrict__ th_init) {
  __shared__ __attribute__((aligned(16))) uint64_t sbuf[4][16 * SCAN_CAP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int nqt = (nq + 15) >> 4;
  const int qt = blockIdx.y * 4 + wave;
  if (qt >= nqt) return;                     // no block-level barriers below
  uint64_t* buf = sbuf[wave];
  const int part = blockIdx.x;
  const long r_begin = part * range;
  const long r_end = min(n_ref, r_begin + range);

  // A fragments (LUT limbs) for this query tile: registers for the whole scan
  i32x4 a[LIMBS][KSMAX];
#pragma unroll
  for (int lb = 0; lb < LIMBS; ++lb)
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks)
      if (ks < KS)
        a[lb][ks] = *reinterpret_cast<const i32x4*>(lut + ((((long)qt * LIMBS + lb) * KS + ks) * 64 + lane) * 16);
      else
        a[lb][ks] = i32x4{0, 0, 0, 0};

  int th[4], cnt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = qt * 16 + 4 * lg + i;
    th[i] = (th_init && q < nq) ? th_init[q] : INT_MAX;
    cnt[i] = 0;
  }

  for (long r0 = r_begin; r0 < r_end; r0 += 16) {
    const long r = r0 + li;
    const bool rv = r < r_end;
    const uint8_t* row = codes + (rv ? r : r_begin) * ld + 16 * lg;
    i32x4 b[KSMAX];
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks)
      if (ks < KS) b[ks] = *reinterpret_cast<const i32x4*>(row + 64 * ks);
    i32x4 acc[LIMBS];
#pragma unroll
    for (int lb = 0; lb < LIMBS; ++lb) acc[lb] = i32x4{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks)
      if (ks < KS)
#pragma unroll
        for (int lb = 0; lb < LIMBS; ++lb)
          acc[lb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[lb][ks], b[ks], acc[lb], 0, 0, 0);

    // filter: lane holds D[q = 4*lg + i][ref = r]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = LIMBS == 2 ? acc[0][i] * 128 + acc[1][i] : acc[0][i];
      const bool pass = rv && d < th[i];
      const uint64_t m = __ballot(pass);
      if (m) {
        const uint32_t gb = (uint32_t)(m >> (16 * lg)) & 0xFFFFu;
        if (pass) {
          const int pre = __popc(gb & ((1u << li) - 1u));
          buf[(4 * lg + i) * SCAN_CAP + cnt[i] + pre] = make_key(d, (uint32_t)(r + ref_offset));
        }
        cnt[i] += __popc(gb);
      }
    }
    // compaction of rows close to capacity (wave-uniform loop)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint64_t need = __ballot(cnt[i] > SCAN_TH);
      while (need) {
        const int src = __builtin_ctzll(need);
        const int g = src >> 4;
        need &= ~(0xFFFFull << (16 * g));
        int nc, nt;
        compact_row(buf, 4 * g + i, __shfl(cnt[i], src, 64), k, lane, nc, nt);
        if (lg == g) { cnt[i] = nc; th[i] = nt; }
      }
    }
  }
  // final compaction of every row; emit the per-range top-k
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    for (int g = 0; g < 4; ++g) {
      const int row = 4 * g + i;
      const int c = __shfl(cnt[i], 16 * g, 64);
      int nc, nt;
      compact_row(buf, row, c, k, lane, nc, nt);
      const int q = qt * 16 + row;
      if (q < nq && lane < k)
        parts[((long)part * nq + q) * k + lane] = lane < nc ? buf[row * SCAN_CAP + lane] : KEY_MAX;
    }
  }
}

// ----------------------------------------------------------------- merge ---
// block (256 threads) per (query, group of G lists): bitonic sort of <= 1024 keys in LDS
__global__ __launch_bounds__(256) void merge_kernel(const uint64_t* __restrict__ in, int n_lists, int nq,
                                                    int k, int G, uint64_t* __restrict__ out) {
  __shared__ uint64_t s[1024];
  const int q = blockIdx.y, grp = blockIdx.x, tid = threadIdx.x;
  const int l0 = grp * G, nl = min(G, n_lists - l0);
  const int n = nl * k;
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = tid; i < P; i += 256) {
    uint64_t v = KEY_MAX;
    if (i < n) {
      const int li = i / k, j = i % k;
      v = in[((long)(l0 + li) * nq + q) * k + j];
    }
    s[i] = v;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P / 2; i += 256) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = s[lo], b = s[hi];
        if ((a > b) == up) { s[lo] = b; s[hi] = a; }
      }
      __syncthreads();
    }
  }
  for (int j = tid; j < k; j += 256) out[((long)grp * nq + q) * k + j] = s[j];
}

__global__ void decode_kernel(const uint64_t* __restrict__ keys, int nq, int k, const int* __restrict__ exps,
                              const float* __restrict__ consts, int64_t* __restrict__ idx, float* __restrict__ dist) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)nq * k) return;
  const int q = (int)(i / k);
  const uint64_t key = keys[i];
  if (key == KEY_MAX) {
    idx[i] = -1;
    if (dist) dist[i] = INFINITY;
    return;
  }
  idx[i] = (int64_t)(key & 0xFFFFFFFFull);
  if (dist) {
    const int d = (int)(key >> 32) - KEY_BIAS;
    dist[i] = (consts ? consts[q] : 0.f) + ldexpf((float)d, -exps[q]);
  }
}

// ------------------------------------------------------------- rag mean ---
// A workgroup owns RM_P token positions x RM_Q queries: the per-position rows
// (W[tok0], W[tok1] - W[tok0], pe, A_r) are loaded once and reused for all RM_Q
// queries, and the neighbour alt-allele counts come from independent byte loads
// (neighbour indices staged in LDS first), so no load waits on another.
constexpr int RM_P = 8, RM_Q = 16, RM_KMAX = 128;

// CNT: `codes` holds per-query alt-allele counts over the k neighbours ([nq][ld], the
// sharded-panel form, see neighbor_counts_kernel) instead of panel rows indexed by idx;
// idx still gives the number of valid neighbours.
template <typename T, bool CNT = false>
__global__ __launch_bounds__(256) void rag_mean_kernel(int nq, int L, int D, int k, const int64_t* __restrict__ idx,
                                                       const uint8_t* __restrict__ codes, long ld, int n_sites,
                                                       const float* __restrict__ W, const float* __restrict__ pe,
                                                       const float* __restrict__ Ar, int tok0, int tok1, int sos,
                                                       int eos, int pad, T* __restrict__ out) {
  __shared__ int64_t sidx[RM_Q * RM_KMAX];
  __shared__ float frac[RM_Q][RM_P];
  __shared__ int nvalid[RM_Q];
  const int l0 = blockIdx.x * RM_P, q0 = blockIdx.y * RM_Q, tid = threadIdx.x;
  for (int i = tid; i < RM_Q * k; i += 256) {
    const int q = q0 + i / k;
    sidx[i] = q < nq ? idx[(long)q * k + i % k] : -1;
  }
  __syncthreads();
  if (tid < RM_Q * RM_P) {
    const int qq = tid / RM_P, p = tid % RM_P, l = l0 + p;
    const bool site = l >= 1 && l <= n_sites;
    int c = 0, nv = 0;
#pragma unroll 8
    for (int j = 0; j < k; ++j) {
      const int64_t r = sidx[qq * k + j];
      nv += r >= 0;
      if constexpr (!CNT) c += (r >= 0 && site) ? codes[r * ld + (l - 1)] : 0;
    }
    if constexpr (CNT) c = (site && q0 + qq < nq) ? codes[(long)(q0 + qq) * ld + (l - 1)] : 0;
    frac[qq][p] = nv > 0 ? (float)c / (float)nv : 0.f;
    if (p == 0) nvalid[qq] = nv;
  }
  __syncthreads();
  constexpr int V = 16 / sizeof(T);
  const int cpr = D / V;
  const int nqb = min(RM_Q, nq - q0);
  for (int id = tid; id < RM_P * cpr; id += 256) {
    const int p = id / cpr, c = (id % cpr) * V;
    const int l = l0 + p;
    if (l >= L) break;
    int t;
    const bool site = l >= 1 && l <= n_sites;
    if (l == 0) t = sos; else if (site) t = tok0; else if (l == n_sites + 1) t = eos; else t = pad;
    float w0[V], dw[V], pp[V], ar[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      w0[j] = W[(long)t * D + c + j];
      dw[j] = site ? W[(long)tok1 * D + c + j] - w0[j] : 0.f;
      pp[j] = pe[(long)l * D + c + j];
      ar[j] = Ar ? Ar[(long)l * D + c + j] : 0.f;
    }
    for (int qq = 0; qq < nqb; ++qq) {
      const float f = frac[qq][p];
      const bool any = nvalid[qq] > 0;
      T o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float w = w0[j];
        if (site) w = any ? w + f * dw[j] : 0.f;
        float x = w + pp[j];
        if (Ar) x += ar[j];
        o[j] = from_f32<T>(x);
      }
      *reinterpret_cast<u32x4*>(out + ((long)(q0 + qq) * L + l) * D + c) = *reinterpret_cast<u32x4*>(o);
    }
  }
}

// ---------------------------------------------------------- panel synth ---
__device__ __forceinline__ double hash_u01(uint64_t seed, uint64_t r, uint64_t c) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + r * 0xD1B54A32D192ED03ull + c * 0x8CB92BA72F3D8DD7ull;
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x = x ^ (x >> 31);
  return (double)(x >> 40) / (double)(1 << 24);
}

// Alt-allele counts over the neighbours a panel SHARD owns: counts[q][s] = sum over j of
// codes[idx[q][j] - row0][s] for the idx[q][j] in [row0, row0 + n_rows) (global indices).
// One thread per (query, 16-site chunk); the shards' partial counts sum (all-reduce) to the
// full count, which rag_mean_kernel<T, true> turns into the neighbour mean.
__global__ __launch_bounds__(256) void neighbor_counts_kernel(int nq, int k, const int64_t* __restrict__ idx,
                                                              const uint8_t* __restrict__ codes, long ld,
                                                              long row0, long n_rows, uint8_t* __restrict__ counts,
                                                              long ld_out) {
  const long chunks = ld_out / 16;
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)nq * chunks) return;
  const int q = (int)(id / chunks);
  const int c0 = (int)(id % chunks) * 16;
  uint32_t acc[4] = {0, 0, 0, 0};                    // 16 byte counters (k <= 128: no carries)
  for (int j = 0; j < k; ++j) {
    const long r = idx[(long)q * k + j] - row0;
    if (r < 0 || r >= n_rows || c0 >= ld) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(codes + r * ld + c0);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += v[i];      // codes are 0/1 bytes: packed byte adds
  }
  *reinterpret_cast<u32x4*>(counts + (long)q * ld_out + c0) = u32x4{acc[0], acc[1], acc[2], acc[3]};
}

__global__ void panel_synth_kernel(uint8_t* __restrict__ codes, long n_ref, long ld, int n_sites,
                                   const float* __restrict__ af, uint64_t seed, long row0) {
  const long chunks_per_row = ld / 16;
  const long total = n_ref * chunks_per_row;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const long r = id / chunks_per_row;
    const int c0 = (int)(id % chunks_per_row) * 16;
    uint8_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int s = c0 + j;
      v[j] = (s < n_sites && hash_u01(seed, (uint64_t)(r + row0), (uint64_t)s) < (double)af[s]) ? 1 : 0;
    }
    *reinterpret_cast<u32x4*>(codes + r * ld + c0) = *reinterpret_cast<u32x4*>(v);
  }
}

// ------------------------------------------------------------ scan v2 ---
// One workgroup = 8 waves = 8 query tiles (128 queries) over one contiguous panel
// range.  The panel codes stream HBM -> LDS ONCE per workgroup (global_load_lds,
// 1 KiB per wave instruction, 3-stage ring of 32 haplotypes with counted vmcnt)
// and every wave reads them from LDS for its own query tile, whose LUT limbs stay
// in VGPRs for the whole scan — the v1 kernel instead had each wave fetch the
// codes itself (8x the L2->CU traffic).  Rows are n_sites_pad bytes (multiple of
// 256); the 16-B chunk c of row r sits at c ^ (r & 15) so the 16 rows of a
// ds_read_b128 B fragment hit 16 different bank groups.
constexpr int S2_CAP = 64;                // candidate slots per query (k <= 32 plus 32 of slack)
constexpr int S2_TH = S2_CAP - 16;        // compact when more than 48 held (a row gains <= 16 between checks)
constexpr int S2_LDS = 160 * 1024;        // whole LDS of a CU: one workgroup per CU
constexpr int S2_CAND = 8 * 16 * S2_CAP * 8;
// 32 haplotypes per LDS stage, ring of up to 3 stages in the LDS left beside the
// candidate lists.  Measured (1 M haplotypes x 1024 sites, 48/96/128 queries): 16-row
// stages in a 6-deep ring are 15-17 % slower (per-stage barrier + filter overhead
// dominates, not HBM latency), and 48-slot candidate lists another 12 % (compaction
// after every insert once k = 32 slots are held).
__host__ __device__ constexpr int s2_rows(int KS) { return 32; }
__host__ __device__ constexpr int s2_nst(int KS) {
  return (S2_LDS - S2_CAND) / (s2_rows(KS) * KS * 64) > 3 ? 3 : (S2_LDS - S2_CAND) / (s2_rows(KS) * KS * 64);
}

// s_waitcnt vmcnt(PPW * min(y, V)): retire all but the y (<= V) youngest stages' loads
template <int PPW, int V>
__device__ __forceinline__ void vm_wait_stages(int y) {
  if constexpr (V <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (y >= V) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * V) : "memory");
      return;
    }
    vm_wait_stages<PPW, V - 1>(y);
  }
}
#ifndef S2_QTW1
#define S2_QTW1 1                         // query tiles per wave of the reduced one-limb scan
#endif

__device__ __forceinline__ void compact_row2(uint64_t* buf, int row, int cnt, int k, int lane, int& new_cnt,
                                             int& new_th) {
  uint64_t key = lane < cnt ? buf[row * S2_CAP + lane] : KEY_MAX;
  key = wave_sort64(key, lane);
  if (lane < k) buf[row * S2_CAP + lane] = key;
  new_cnt = cnt < k ? cnt : k;
  const uint64_t kth = shfl64(key, k - 1);
  new_th = (cnt >= k) ? (int)(kth >> 32) - KEY_BIAS : INT_MAX;
}

// One body, two shapes:
//   LIMBS = 2, QTW = 1: 8 computing waves, one 16-query tile each (LUT hi/lo limbs);
//   LIMBS = 1, QTW = 2: the reduced LUT (lut_kernel: dq/g fits one limb, distance = g *
//                       D_1limb): 4 computing waves, two query tiles each, so every B
//                       fragment read from LDS feeds two MFMAs — half the LDS read traffic
//                       of the 2-limb shape, whose 8 waves x 32 KiB per stage saturate
//                       the 128 B/clk LDS port.  Waves 4..7 only stream codes.
template <int KS, int LIMBS, int QTW, int MODE>
__device__ __forceinline__ void scan2_body(char* smem, const uint8_t* __restrict__ codes, long n_ref, long ld,
                                           const int8_t* __restrict__ lut, const int* __restrict__ mult, int nq,
                                           int k, long range, long ref_offset, uint64_t* __restrict__ parts,
                                           const int* __restrict__ th_init, int part, int group, int ntpol) {
  constexpr int ROWB = KS * 64;                        // staged row bytes
  constexpr int S2_R = s2_rows(KS);
  constexpr int STAGE = S2_R * ROWB;
  constexpr int PPW = STAGE / 1024 / 8;                // glds pieces per wave per stage
  constexpr int NST = s2_nst(KS);                      // ring depth
  static_assert(NST >= 2, "stage too large");
  static_assert(PPW * (NST - 2) <= 63, "vmcnt range");
  static_assert(ROWB % 256 == 0 && PPW >= 1, "rows must be multiples of 256 B");
  uint64_t* cand = reinterpret_cast<uint64_t*>(smem + NST * STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int nqt = (nq + 15) >> 4;
  const int qt0 = group * 8 + wave * QTW;
  const bool active = wave * QTW < 8 && qt0 < nqt;     // wave-uniform; every wave still loads + syncs
  const long r_begin = (long)part * range;
  const long r_end = min(n_ref, r_begin + range);
  const int nstage = r_end > r_begin ? (int)((r_end - r_begin + S2_R - 1) / S2_R) : 0;

  // LUT limbs: unconditional loads (inactive tiles read the last tile) retired BEFORE the
  // loop — a load still pending inside it would make hipcc wait vmcnt(0), draining the ring
  int qtc[QTW];
#pragma unroll
  for (int t = 0; t < QTW; ++t) qtc[t] = min(qt0 + t, nqt - 1);
  i32x4 a[LIMBS][QTW][KS];
#pragma unroll
  for (int lb = 0; lb < LIMBS; ++lb)
#pragma unroll
    for (int t = 0; t < QTW; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        a[lb][t][ks] = *reinterpret_cast<const i32x4*>(lut + ((((long)qtc[t] * LIMBS + lb) * KS + ks) * 64 + lane) * 16);
#pragma unroll
  for (int lb = 0; lb < LIMBS; ++lb)
#pragma unroll
    for (int t = 0; t < QTW; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(a[lb][t][ks]));

  auto issue = [&](int st, long r0) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int piece = wave * PPW + j;
      const int byte = piece * 1024 + lane * 16;
      const int row = byte / ROWB, ch = (byte % ROWB) >> 4;
      long r = r0 + row;
      r = r < r_end ? r : r_end - 1;
      const int src_ch = ch ^ (row & 15);
      const auto* gsrc = (const __attribute__((address_space(1))) void*)(codes + r * ld + src_ch * 16);
      auto* ldst = (__attribute__((address_space(3))) void*)(smem + st * STAGE + piece * 1024);
      if (ntpol) __builtin_amdgcn_global_load_lds(gsrc, ldst, 16, 0, 2);   // streamed once: nt policy
      else __builtin_amdgcn_global_load_lds(gsrc, ldst, 16, 0, 0);
    }
  };

  int th[QTW][4], cnt[QTW][4], mul[QTW][4];
#pragma unroll
  for (int t = 0; t < QTW; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = qtc[t] * 16 + 4 * lg + i;
      th[t][i] = (th_init && q < nq) ? th_init[q] : INT_MAX;
      mul[t][i] = mult ? mult[q] : 1;
      cnt[t][i] = 0;
    }
#pragma unroll
  for (int t = 0; t < QTW; ++t)   // retire before the ring starts
    asm volatile("" ::"v"(th[t][0]), "v"(th[t][1]), "v"(th[t][2]), "v"(th[t][3]), "v"(mul[t][0]), "v"(mul[t][1]),
                 "v"(mul[t][2]), "v"(mul[t][3]));

#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (j < nstage) issue(j, r_begin + (long)j * S2_R);
  for (int it = 0; it < nstage; ++it) {
    // retire stage it; up to NST-2 younger stages stay in flight across the barrier
    vm_wait_stages<PPW, NST - 2>(nstage - 1 - it);
    __builtin_amdgcn_s_barrier();
    if (MODE != 2 && it + NST - 1 < nstage) issue((it + NST - 1) % NST, r_begin + (long)(it + NST - 1) * S2_R);
    if (!active || MODE == 1) continue;
    const char* st = smem + (it % NST) * STAGE;
    const long r0 = r_begin + (long)it * S2_R;
    // B fragments (16 haplotypes x 64 sites) of both 16-row groups as one stream,
    // read PF ahead of their MFMAs so LDS latency hides under the MFMA chain
    constexpr int RG = S2_R / 16, F = RG * KS, PF = 4;
    auto bfrag = [&](int f) {
      const int row = 16 * (f / KS) + li, ks = f % KS;
      return *reinterpret_cast<const i32x4*>(st + row * ROWB + (((4 * ks + lg) ^ (row & 15)) << 4));
    };
    i32x4 bq[PF];
#pragma unroll
    for (int f = 0; f < PF; ++f) bq[f] = bfrag(f);
    i32x4 acc[RG][QTW][LIMBS];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
      for (int t = 0; t < QTW; ++t)
#pragma unroll
        for (int lb = 0; lb < LIMBS; ++lb) acc[rg][t][lb] = i32x4{0, 0, 0, 0};
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const i32x4 b = bq[f % PF];
      if (f + PF < F) bq[f % PF] = bfrag(f + PF);
#pragma unroll
      for (int t = 0; t < QTW; ++t)
#pragma unroll
        for (int lb = 0; lb < LIMBS; ++lb)
          acc[f / KS][t][lb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[lb][t][f % KS], b, acc[f / KS][t][lb], 0, 0, 0);
    }
    // pin the interleave (hipcc otherwise sinks each read to just before its MFMA):
    // PF reads, then per fragment {1 read, QTW*LIMBS MFMAs}
    __builtin_amdgcn_sched_group_barrier(0x100, PF, 0);
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if (f + PF < F) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, QTW * LIMBS, 0);
    }
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
      const long r = r0 + 16 * rg + li;
      const bool rv = r < r_end;
#pragma unroll
      for (int t = 0; t < QTW; ++t) {
        uint64_t* buf = cand + (wave * QTW + t) * 16 * S2_CAP;
        int dd[4];
        bool anyp = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dd[i] = LIMBS == 2 ? acc[rg][t][0][i] * 128 + acc[rg][t][1][i] : acc[rg][t][0][i] * mul[t][i];
          anyp |= dd[i] < th[t][i];
        }
        if (!__ballot(rv && anyp)) continue;   // the common case once the threshold is tight
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int d = dd[i];
          const bool pass = rv && d < th[t][i];
          const uint64_t m = __ballot(pass);
          if (m) {
            const uint32_t gb = (uint32_t)(m >> (16 * lg)) & 0xFFFFu;
            if (pass) {
              const int pre = __popc(gb & ((1u << li) - 1u));
              buf[(4 * lg + i) * S2_CAP + cnt[t][i] + pre] = make_key(d, (uint32_t)(r + ref_offset));
            }
            cnt[t][i] += __popc(gb);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint64_t need = __ballot(cnt[t][i] > S2_TH);
          while (need) {
            const int src = __builtin_ctzll(need);
            const int g = src >> 4;
            need &= ~(0xFFFFull << (16 * g));
            int nc, nt;
            compact_row2(buf, 4 * g + i, __shfl(cnt[t][i], src, 64), k, lane, nc, nt);
            if (lg == g) { cnt[t][i] = nc; th[t][i] = nt; }
          }
        }
      }
    }
  }
  if (!active) return;
#pragma unroll
  for (int t = 0; t < QTW; ++t) {
    if (qt0 + t >= nqt) break;
    uint64_t* buf = cand + (wave * QTW + t) * 16 * S2_CAP;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      for (int g = 0; g < 4; ++g) {
        const int row = 4 * g + i;
        const int c = __shfl(cnt[t][i], 16 * g, 64);
        int nc, nt;
        compact_row2(buf, row, c, k, lane, nc, nt);
        const int q = (qt0 + t) * 16 + row;
        if (q < nq && lane < k)
          parts[((long)part * nq + q) * k + lane] = lane < nc ? buf[row * S2_CAP + lane] : KEY_MAX;
      }
    }
  }
}

// MODE (diagnostics only): 1 = loads only, 2 = compute only.  A 2-limb launch whose LUT
// reduced to one limb for every query (wide == 0, written by lut_kernel) runs the
// 1-limb two-tile body instead — decided on the device, no host round trip.
template <int KS, int LIMBS, int MODE = 0>
__global__ __launch_bounds__(512) void scan2_kernel(const uint8_t* __restrict__ codes, long n_ref, long ld,
                                                    const int8_t* __restrict__ lut, int nq, int k, long range,
                                                    long ref_offset, uint64_t* __restrict__ parts,
                                                    const int* __restrict__ th_init, const int* __restrict__ wide,
                                                    int n_parts, int n_groups, int nt) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // XCD co-scheduling: the G query groups of one panel range get consecutive dispatch
  // slots 8 apart (same XCD, same round), so the range streams from HBM once and the
  // other G-1 workgroups read it from that XCD's L2 (one pass over the panel per launch)
  const int i = blockIdx.x, G = n_groups;
  const int slot = i / 8, group = slot % G, part = (slot / G) * 8 + i % 8;
  if (part >= n_parts) return;                        // whole workgroup, before any barrier
  if constexpr (LIMBS == 2 && KS <= 16) {   // (KS = 20: two tiles of A would spill)
    if (wide && *wide == 0) {
      const long nqt = (nq + 15) >> 4;
      const int8_t* lut1 = lut + nqt * 2 * KS * 1024;
      const int* mult = reinterpret_cast<const int*>(lut1 + nqt * KS * 1024);
      scan2_body<KS, 1, S2_QTW1, MODE>(smem, codes, n_ref, ld, lut1, mult, nq, k, range, ref_offset, parts, th_init,
                                       part, group, nt);
      return;
    }
  }
  scan2_body<KS, LIMBS, 1, MODE>(smem, codes, n_ref, ld, lut, nullptr, nq, k, range, ref_offset, parts, th_init,
                                 part, group, nt);
}

template <int KS, int LB>
static void launch_scan2(int n_parts, int nq, hipStream_t s, const uint8_t* codes, long n_ref, long ld,
                         const int8_t* lut, int k, long range, long off, uint64_t* parts, const int* th,
                         const int* wide) {
  constexpr size_t STAGE = (size_t)s2_rows(KS) * KS * 64;
  constexpr size_t NST = s2_nst(KS);
  const size_t lds = NST * STAGE + S2_CAND;
  static_assert(NST * STAGE + S2_CAND <= S2_LDS, "LDS budget");
  auto kern = scan2_kernel<KS, LB, 0>;
  if constexpr (KS == 16 && LB == 2) {
    if (options().scan_mode == 1) kern = scan2_kernel<KS, LB, 1>;
    if (options().scan_mode == 2) kern = scan2_kernel<KS, LB, 2>;
  }
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int G = ((nq + 15) / 16 + 7) / 8;
  const long nwg = (long)((n_parts + 7) / 8) * 8 * G;
  // one query group: every code byte is read by exactly one workgroup, so stream it with
  // the non-temporal policy; with G > 1 the other groups read the range from L2 (default)
  const int nt = options().scan_nt >= 0 ? (int)(options().scan_nt != 0) : (G == 1);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(512), lds, s, codes, n_ref, ld, lut, nq, k, range, off, parts, th,
                     wide, n_parts, G, nt);
}

static int scan_parts(long n_ref, int nq) {
  // ~2048 refs per range at least; large panels get a multiple of 256 ranges (one
  // workgroup per CU per round, no tail round)
  long p = (n_ref + 2047) / 2048;
  if (p >= 256) p = 256 * ((n_ref + 256L * 8192 - 1) / (256L * 8192));
  // small panels (training: 10 000 haplotypes were 5 ranges = 5 workgroups, 190 us): ranges down
  // to 64 refs, so the scan still spreads over the chip — up to 256 workgroups counting the query
  // groups (G of them run per range): many queries fill the chip by themselves, and each range
  // adds nq x k partial entries to the merge
  else {
    const long G = std::max<long>(1, ((long)(nq > 0 ? nq : 1) + 127) / 128);
    const long spread = std::max<long>(1, 256 / G);
    p = std::min<long>(256, std::max<long>(p, std::min<long>(spread, (n_ref + 63) / 64)));
  }
  if (p < 1) p = 1;
  if (p > 4096) p = 4096;
  return (int)p;
}

template <int KSM, int LB>
static void launch_scan(dim3 g, hipStream_t s, const uint8_t* codes, long n_ref, long ld, int KS,
                        const int8_t* lut, int nq, int k, long range, long off, uint64_t* parts, const int* th) {
  hipLaunchKernelGGL((scan_kernel<KSM, LB>), g, dim3(256), 0, s, codes, n_ref, ld, KS, lut, nq, k, range, off, parts,
                     th);
}

}  // namespace snvrag

using namespace snvrag;

// LUT buffer: [nqt][limbs][KS][64 lanes][16 B] fragments; for limbs == 2 followed by the
// reduced one-limb fragments [nqt][KS][64][16], int32 mult[nqt*16] and int32 wide flag.
static size_t lut_tail_offset(int64_t nq, int32_t n_sites_pad) {
  return (size_t)((nq + 15) / 16) * 3 * (n_sites_pad / 64) * 1024;
}
static size_t lut_ws_offset(int64_t nq, int32_t n_sites_pad, int limbs) {
  const size_t main = (size_t)((nq + 15) / 16) * limbs * (n_sites_pad / 64) * 64 * 16;
  const size_t end = limbs != 2 ? main : lut_tail_offset(nq, n_sites_pad) + (size_t)((nq + 15) / 16) * 16 * 4 + 16;
  return (end + 255) / 256 * 256;
}

// the LUT, then (256-B aligned) the general-path workspace: delta [nq][n_sites_pad] f32 and the
// constant's chunk sums [nq][lut_nch_max] f32
extern "C" size_t snvrag_knn_lut_bytes(int64_t nq, int32_t n_sites_pad, int limbs) {
  return lut_ws_offset(nq, n_sites_pad, limbs) + (size_t)nq * (n_sites_pad + lut_nch_max(n_sites_pad)) * 4;
}

extern "C" int snvrag_knn_lut(int64_t nq, int64_t L, int64_t D, const int64_t* tok_q, const float* W,
                              const float* Aq, int64_t aq_period, const float* Ar, const uint8_t* site_mask,
                              int32_t n_sites, int32_t n_sites_pad, int tok0, int tok1, int mask_tok, int limbs,
                              void* lut_out, int32_t* exp_out, float* const_out, void* stream) {
  return snvrag_knn_lut_panel(nq, L, D, tok_q, W, W, Aq, aq_period, Ar, site_mask, n_sites, n_sites_pad, tok0, tok1,
                              mask_tok, limbs, lut_out, exp_out, const_out, stream);
}

extern "C" int snvrag_knn_lut_panel(int64_t nq, int64_t L, int64_t D, const int64_t* tok_q, const float* W,
                                    const float* Wp, const float* Aq, int64_t aq_period, const float* Ar,
                                    const uint8_t* site_mask, int32_t n_sites, int32_t n_sites_pad, int tok0,
                                    int tok1, int mask_tok, int limbs, void* lut_out, int32_t* exp_out,
                                    float* const_out, void* stream) {
  SNV_CHECK_ARG(tok_q && W && Wp && site_mask && lut_out && exp_out, "null pointer");
  SNV_CHECK_ARG(limbs == 1 || limbs == 2, "limbs must be 1 or 2");
  SNV_CHECK_ARG(n_sites_pad % 64 == 0 && n_sites_pad >= n_sites && n_sites + 2 <= L, "site padding");
  SNV_CHECK_ARG(n_sites_pad <= 20 * 64, "window longer than 1280 sites");
  if (nq == 0) return 0;
  hipStream_t s = as_stream(stream);
  const size_t sh = (size_t)(n_sites_pad + 4) * sizeof(float);
  if (limbs == 2) {   // mult[] and the wide flag start at zero
    char* tail = (char*)lut_out + lut_tail_offset(nq, n_sites_pad);
    SNV_HIP(hipMemsetAsync(tail, 0, (size_t)((nq + 15) / 16) * 16 * 4 + 16, s));
  }
  float* gdelta = (float*)((char*)lut_out + lut_ws_offset(nq, n_sites_pad, limbs));
  float* gcpart = gdelta + (size_t)nq * n_sites_pad;
  if (Aq || Ar) {
    auto a16 = [](const void* p) { return p == nullptr || ((uintptr_t)p % 16) == 0; };
    SNV_CHECK_ARG(D % 4 == 0 && a16(W) && a16(Wp) && a16(Aq) && a16(Ar),
                  "offset LUT: D % 4 == 0 and 16-byte aligned W / Wp / Aq / Ar (float4 rows)");
    const int64_t nch = std::min<int64_t>((L + LUT_CH - 1) / LUT_CH, lut_nch_max(n_sites_pad));
    hipLaunchKernelGGL(lut_delta_kernel, dim3((unsigned)nch, (unsigned)nq), dim3(256), 0, s,
                       (int)L, (int)D, tok_q, W, Wp, Aq, (long)aq_period, Ar, site_mask, n_sites, n_sites_pad, tok0,
                       tok1, mask_tok, gdelta, gcpart);
    SNV_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(lut_kernel, dim3((unsigned)nq), dim3(256), sh, s, (int)L, (int)D, tok_q, W, Wp, Aq,
                     (long)aq_period, Ar, site_mask, n_sites, n_sites_pad, (int)nq, tok0, tok1, mask_tok,
                     limbs, (int8_t*)lut_out, exp_out, const_out, gdelta, gcpart);
  SNV_LAUNCH_CHECK();
  if (nq % 16)
    hipLaunchKernelGGL(lut_zero_pad_kernel, dim3(64), dim3(256), 0, s, (int8_t*)lut_out, (int)nq,
                       n_sites_pad / 64, limbs);
  SNV_LAUNCH_CHECK();
  return 0;
}

__global__ void threshold_kernel(const uint64_t* __restrict__ keys, int nq, int k, int* __restrict__ th) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const uint64_t key = keys[(long)q * k + k - 1];
  th[q] = key == KEY_MAX ? INT_MAX : (int)(key >> 32) - KEY_BIAS + 1;
}

extern "C" int snvrag_knn_threshold(const uint64_t* keys, int32_t nq, int k, int32_t* th_out, void* stream) {
  SNV_CHECK_ARG(keys && th_out && k >= 1, "bad arguments");
  if (nq == 0) return 0;
  hipLaunchKernelGGL(threshold_kernel, dim3((nq + 255) / 256), dim3(256), 0, as_stream(stream), keys, (int)nq, k,
                     (int*)th_out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_knn_scan_parts(int64_t n_ref, int32_t nq) { return scan_parts(n_ref, nq); }

extern "C" int snvrag_knn_scan(const uint8_t* codes, int64_t n_ref, int64_t ld_codes, int32_t n_sites_pad,
                               const void* lut, int32_t nq, int limbs, int k, int64_t ref_offset,
                               uint64_t* part_keys, int32_t n_parts, const int32_t* th_init, void* stream) {
  SNV_CHECK_ARG(codes && lut && part_keys, "null pointer");
  SNV_CHECK_ARG(k >= 1 && k <= 32, "k must be in [1, 32]");
  SNV_CHECK_ARG(limbs == 1 || limbs == 2, "limbs");
  SNV_CHECK_ARG(n_sites_pad % 64 == 0 && ld_codes >= n_sites_pad &&
                    n_sites_pad <= (n_sites_pad % 256 == 0 ? 20 * 64 : 17 * 64), "site padding");
  SNV_CHECK_ARG(ld_codes % 16 == 0 && ((uintptr_t)codes % 16) == 0, "codes must be 16-byte aligned rows");
  SNV_CHECK_ARG(n_parts >= 1, "n_parts");
  SNV_CHECK_ARG(n_ref + ref_offset < (1LL << 32), "panel index must fit 32 bits");
  if (nq == 0) return 0;
  long range = (n_ref + n_parts - 1) / n_parts;
  range = ((range + 15) / 16) * 16;
  if (range == 0) range = 16;
  const int KS = n_sites_pad / 64;
  dim3 g((unsigned)n_parts, (unsigned)(((nq + 15) / 16 + 3) / 4));
  hipStream_t s = as_stream(stream);
  const int8_t* L8 = (const int8_t*)lut;
  // lut_kernel's "some query needs two limbs" flag (limbs == 2 buffers only)
  const int* wide = (limbs == 2 && !options().knn_no_reduce)
                        ? reinterpret_cast<const int*>(L8 + lut_tail_offset(nq, n_sites_pad) +
                                                       (size_t)((nq + 15) / 16) * 16 * 4)
                        : nullptr;
  evlog_begin(s);
  const bool v2 = n_sites_pad % 256 == 0 && n_sites_pad <= 1280;
  if (v2) {
#define SCAN2(K_)                                                                                          \
  case K_:                                                                                                 \
    if (limbs == 2) launch_scan2<K_, 2>(n_parts, nq, s, codes, n_ref, ld_codes, L8, k, range, ref_offset, part_keys, th_init, wide); \
    else launch_scan2<K_, 1>(n_parts, nq, s, codes, n_ref, ld_codes, L8, k, range, ref_offset, part_keys, th_init, nullptr);          \
    break;
    switch (KS) { SCAN2(4) SCAN2(8) SCAN2(12) SCAN2(16) SCAN2(20) }
#undef SCAN2
  } else {
#define SCAN(KSM)                                                                                   \
  do {                                                                                              \
    if (limbs == 2) launch_scan<KSM, 2>(g, s, codes, n_ref, ld_codes, KS, L8, nq, k, range, ref_offset, part_keys, th_init); \
    else launch_scan<KSM, 1>(g, s, codes, n_ref, ld_codes, KS, L8, nq, k, range, ref_offset, part_keys, th_init);           \
  } while (0)
  if (KS <= 4) SCAN(4);
  else if (KS <= 8) SCAN(8);
  else if (KS <= 16) SCAN(16);
  else SCAN(17);
#undef SCAN
  }
  SNV_LAUNCH_CHECK();
  // algorithmic bytes: every code byte of the window once + LUT + partial lists
  evlog_end(s, EV_KNN_SCAN, (double)n_ref * n_sites_pad + (double)nq * n_sites_pad * limbs +
                            (double)n_parts * nq * k * 8.0);
  return 0;
}

static int merge_group(int k) {
  int kp = 1;
  while (kp < k) kp <<= 1;
  return 1024 / kp;
}

extern "C" size_t snvrag_topk_merge_ws_bytes(int32_t n_lists, int32_t nq, int k) {
  const int G = merge_group(k);
  const long l1 = (n_lists + G - 1) / G;
  return (size_t)2 * (size_t)l1 * nq * k * sizeof(uint64_t) + 256;
}

extern "C" int snvrag_topk_merge(const uint64_t* keys, int32_t n_lists, int32_t nq, int k, uint64_t* out_keys,
                                 void* ws, size_t ws_bytes, void* stream) {
  SNV_CHECK_ARG(keys && out_keys, "null pointer");
  SNV_CHECK_ARG(k >= 1 && k <= 1024, "k");
  if (nq == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int G = merge_group(k);
  const uint64_t* cur = keys;
  int n = n_lists;
  uint64_t* bufs[2] = {nullptr, nullptr};
  if (n > G) {
    SNV_CHECK_ARG(ws && ws_bytes >= snvrag_topk_merge_ws_bytes(n_lists, nq, k), "merge workspace too small");
    const size_t half = (size_t)((n_lists + G - 1) / G) * nq * k;
    bufs[0] = (uint64_t*)ws;
    bufs[1] = bufs[0] + half;
  }
  int flip = 0;
  while (true) {
    const int groups = (n + G - 1) / G;
    uint64_t* dst = groups == 1 ? out_keys : bufs[flip];
    hipLaunchKernelGGL(merge_kernel, dim3(groups, nq), dim3(256), 0, s, cur, n, nq, k, G, dst);
    SNV_LAUNCH_CHECK();
    if (groups == 1) break;
    cur = dst;
    n = groups;
    flip ^= 1;
  }
  return 0;
}

extern "C" int snvrag_knn_decode(const uint64_t* keys, int32_t nq, int k, const int32_t* exps, const float* consts,
                                 int64_t* idx_out, float* dist_out, void* stream) {
  SNV_CHECK_ARG(keys && idx_out && (!dist_out || exps), "null pointer");
  const long n = (long)nq * k;
  if (n == 0) return 0;
  hipLaunchKernelGGL(decode_kernel, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), keys, nq, k, exps,
                     consts, idx_out, dist_out);
  SNV_LAUNCH_CHECK();
  return 0;
}

template <bool CNT>
static int rag_mean_launch(int dtype_out, int64_t nq, int64_t L, int64_t D, int k, const int64_t* idx,
                           const uint8_t* codes, int64_t ld_codes, int32_t n_sites, const float* W, const float* pe,
                           const float* Ar, int tok0, int tok1, int sos, int eos, int pad, void* out, void* stream) {
  SNV_CHECK_ARG(idx && codes && W && pe && out, "null pointer");
  SNV_CHECK_ARG(D % 8 == 0 && n_sites + 2 <= L, "shape");
  if (nq == 0) return 0;
  SNV_CHECK_ARG(k >= 1 && k <= RM_KMAX, "k must be in [1, 128]");
  SNV_CHECK_ARG(!CNT || ld_codes >= n_sites, "counts row shorter than the window");
  dim3 g((unsigned)cdiv(L, RM_P), (unsigned)cdiv(nq, RM_Q));
  hipStream_t s = as_stream(stream);
  if (dtype_out == SNVRAG_BF16)
    hipLaunchKernelGGL((rag_mean_kernel<bf16, CNT>), g, dim3(256), 0, s, (int)nq, (int)L, (int)D, k, idx, codes,
                       (long)ld_codes, n_sites, W, pe, Ar, tok0, tok1, sos, eos, pad, (bf16*)out);
  else
    hipLaunchKernelGGL((rag_mean_kernel<float, CNT>), g, dim3(256), 0, s, (int)nq, (int)L, (int)D, k, idx, codes,
                       (long)ld_codes, n_sites, W, pe, Ar, tok0, tok1, sos, eos, pad, (float*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_rag_mean(int dtype_out, int64_t nq, int64_t L, int64_t D, int k, const int64_t* idx,
                               const uint8_t* codes, int64_t ld_codes, int32_t n_sites, const float* W,
                               const float* pe, const float* Ar, int tok0, int tok1, int sos, int eos, int pad,
                               void* out, void* stream) {
  return rag_mean_launch<false>(dtype_out, nq, L, D, k, idx, codes, ld_codes, n_sites, W, pe, Ar, tok0, tok1, sos,
                                eos, pad, out, stream);
}

extern "C" int snvrag_rag_mean_counts(int dtype_out, int64_t nq, int64_t L, int64_t D, int k, const int64_t* idx,
                                      const uint8_t* counts, int64_t ld_counts, int32_t n_sites, const float* W,
                                      const float* pe, const float* Ar, int tok0, int tok1, int sos, int eos, int pad,
                                      void* out, void* stream) {
  return rag_mean_launch<true>(dtype_out, nq, L, D, k, idx, counts, ld_counts, n_sites, W, pe, Ar, tok0, tok1, sos,
                               eos, pad, out, stream);
}

extern "C" int snvrag_neighbor_counts(int64_t nq, int k, const int64_t* idx, const uint8_t* codes, int64_t ld,
                                      int64_t row0, int64_t n_rows, uint8_t* counts, int64_t ld_out, void* stream) {
  SNV_CHECK_ARG(idx && counts && (codes || n_rows == 0), "null pointer");
  SNV_CHECK_ARG(k >= 1 && k <= RM_KMAX, "k must be in [1, 128]");
  SNV_CHECK_ARG(ld % 16 == 0 && ld_out % 16 == 0 && ld_out >= ld && ((uintptr_t)counts % 16) == 0 &&
                    ((uintptr_t)codes % 16) == 0,
                "rows must be 16-byte multiples, counts row >= codes row");
  if (nq == 0) return 0;
  const long work = nq * (ld_out / 16);
  hipLaunchKernelGGL(neighbor_counts_kernel, dim3((unsigned)cdiv(work, 256)), dim3(256), 0, as_stream(stream),
                     (int)nq, k, idx, codes, (long)ld, (long)row0, (long)n_rows, counts, (long)ld_out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_panel_synth_rows(uint8_t* codes, int64_t row0, int64_t n_rows, int64_t ld, int32_t n_sites,
                                       const float* af, uint64_t seed, void* stream) {
  SNV_CHECK_ARG(codes && af && ld % 16 == 0 && ld >= n_sites && row0 >= 0, "bad args");
  if (n_rows == 0) return 0;
  const long work = n_rows * (ld / 16);
  const int grid = (int)std::min<long>(cdiv(work, 256), 65536);
  hipLaunchKernelGGL(panel_synth_kernel, dim3(grid), dim3(256), 0, as_stream(stream), codes, (long)n_rows, (long)ld,
                     n_sites, af, seed, (long)row0);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_panel_synth(uint8_t* codes, int64_t n_ref, int64_t ld, int32_t n_sites, const float* af,
                                  uint64_t seed, void* stream) {
  return snvrag_panel_synth_rows(codes, 0, n_ref, ld, n_sites, af, seed, stream);
}
