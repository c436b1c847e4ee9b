// Transformer block tail as ONE kernel on 32x32x16 bf16 MFMAs (gfx950), eval:
//
//   x1  = LN1(x + att W_o^T + b_o)                     multi_head_attention.py:51, sublayer.py:15-16
//   x   = LN2(x1 + lrelu(LN_f(lrelu(x1 W1^T + b1)) W2^T + b2))   feed_forward.py:18-21
//
// A workgroup owns 128 token rows: 4 waves (one per SIMD, up to 512 registers each) x 32
// rows.  Every MFMA computes a TRANSPOSED 32x32 tile (32 weight rows x 32 tokens), so the
// weight fragment (A operand, 1 KiB) read from LDS feeds 2 x 32 x 32 x 16 FLOP — twice the
// work per LDS byte of a 16x16x32 tile — and each lane ends up holding one token's values.
//
// Operands:
//   * activations (att, then x1) live in VGPRs as B fragments for the whole launch
//     (96 registers at D = 384); the LDS is ONE ring of 16 KiB weight slabs streamed
//     once per workgroup by LDS-DMA, 7 slabs (112 KiB) in flight, one barrier per slab
//     placed PF fragments before the slab boundary so LDS reads run ahead across it;
//   * the 4D hidden of a 64-unit chunk stays in registers: phase-1 accumulators are
//     packed straight into phase-2 B fragments (k order baked into W2');
//   * the FFN LayerNorm is folded: W2' = W2 diag(g_f), c1 = rowsum W2',
//     b2' = b2 + W2 b_f, LN_f(h) W2^T + b2 = rstd (h W2'^T) - rstd mean c1 + b2'.
// Lane (token n = lane % 32, half hh = lane / 32) holds output features 32T + 16hh + i
// (i < 16) of tile T: weight ROWS are permuted at pack time (tail_out_feat), the input
// feature order of every B fragment (tail_in_feat) is shared by W_o', W1 and the
// activation loads, so the LN epilogues, the x1 hand-over and the 32-B stores need no
// lane exchange except one xor-32 shuffle per row reduction.
#include "common.h"

#include <utility>

namespace snvrag {

constexpr int TL_FRAG = 1024;               // one A fragment: 32 rows x 16 k bf16
constexpr int TL_SLAB = 16 * TL_FRAG;
constexpr int TL_NSLOT = 9;                 // ring slots (144 KiB)
constexpr int TL_PF4 = 4;                   // A fragments read ahead: the template default and tail_variant 1
constexpr int TL_PF_DEFAULT = 8;             // launch_tail's default (r3: 4: 1.634 ms, 8: 1.659 spilling; r5: 8 faster)
constexpr int TL_ROWS = 128;
constexpr int TL_VEC_LDS = 11 * 1024;       // b1 [4D] + g1, be1, b_o [D] (f32, D <= 384)

template <int D> struct TailShape {
  static constexpr int NT = D / 32;             // 32-feature output tiles
  static constexpr int KS = D / 16;             // 16-wide k steps over D
  static constexpr int NCH = 4 * D / 64;        // 64-unit hidden chunks
  static constexpr int FW1 = 2 * KS;            // W1 fragments per chunk
  static constexpr int FW2 = 4 * NT;            // W2' fragments per chunk
  static constexpr int FPC = FW1 + FW2;         // fragments per chunk
  static constexpr int SPC = FPC / 16;          // slabs per chunk
  static constexpr int FPRE = NT * KS;          // W_o' fragments
  static constexpr int NPRE = FPRE / 16;        // W_o' slabs
  static constexpr int NSLAB = NPRE + NCH * SPC;
  static_assert(FW1 % 16 == 0 && FW2 % 16 == 0 && FPRE % 16 == 0, "parts are whole slabs");
};

// output feature held by MFMA row m of 32-row tile T (lane half hh = (m/4)%2, acc i = 4(m/8) + m%4)
__host__ __device__ constexpr int tail_out_feat(int T, int m) { return 32 * T + 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3); }
// input feature at k = 8 kh + j of k-step s (B fragments of att / x1; columns of W_o', W1)
__host__ __device__ constexpr int tail_in_feat(int s, int kh, int j) { return 32 * (s >> 1) + 16 * kh + 8 * (s & 1) + j; }
// hidden unit (within a 64-unit chunk) at k = 8 kh + j of phase-2 k-step s2 (columns of W2')
__host__ __device__ constexpr int tail_hid(int s2, int kh, int j) {
  return 32 * (s2 >> 1) + 8 * ((8 * (s2 & 1) + j) >> 2) + 4 * kh + ((8 * (s2 & 1) + j) & 3);
}

__device__ __forceinline__ f32x16 mfma32(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
typedef __bf16 tl_bf16x2 __attribute__((ext_vector_type(2)));
typedef float tl_f32x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (RNE) in ONE v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t tl_pack2(float a, float b) {
  const tl_f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, tl_bf16x2));
}
// LeakyReLU(0.1) in 2 VALU ops (fmaxf on a register hipcc cannot prove canonical costs a third,
// a v_max x, x canonicalisation)
__device__ __forceinline__ float tl_lrelu(float x) {
  float r;
  asm("v_mul_f32 %0, 0x3dcccccd, %1\n v_max_f32 %0, %1, %0" : "=&v"(r) : "v"(x));
  return r;
}
// 32-bit LDS address of a pointer into dynamic shared memory
__device__ __forceinline__ uint32_t tl_lds(const char* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ float tl_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float tl_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float tl_bf(const u32x4& v, int j) { return (j & 1) ? tl_hi(v[j >> 1]) : tl_lo(v[j >> 1]); }
// lane id produced afresh at each use (volatile: not CSE'd with earlier ones), so no lane-derived
// address stays live across the FFN and gets spilled
__device__ __forceinline__ int tl_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// x + x of the lane 32 apart (the row reductions over the two lane halves)
__device__ __forceinline__ float tl_xsum32(float x) {
  return x + __int_as_float(__builtin_amdgcn_ds_bpermute((tl_lane() ^ 32) << 2, __float_as_int(x)));
}

// 16 consecutive floats of an LDS table at byte address `addr` (this lane's features 16 hh .. +15
// of a 32-feature tile): reads and their wait in ONE asm statement, so the compiler can neither
// hoist them nor keep whole tables live in registers across a phase (tailp_kernel's epilogues)
__device__ __forceinline__ void tl_ld16(uint32_t addr, float (&v)[16]) {
  u32x4 r[4];
  asm volatile(
      "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
      " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "v"(addr));
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = __uint_as_float(r[i >> 2][i & 3]);
}

// wait until at most `younger` (<= MAXY) slabs of this wave (4 LDS-DMA instructions each) are in flight
template <int MAXY> __device__ __forceinline__ void tl_wait(int younger) {
  static_assert(4 * MAXY <= 63, "vmcnt range");
  if constexpr (MAXY <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (younger >= MAXY) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * MAXY) : "memory");
      return;
    }
    tl_wait<MAXY - 1>(younger);
  }
}

// calls body(std::integral_constant<int, I>{}) for I = 0 .. N-1: a forced full unroll (every
// register-array index in the body is a compile-time constant)
template <typename Body, int... Is>
__device__ __forceinline__ void tl_unroll(Body&& body, std::integer_sequence<int, Is...>) {
  (body(std::integral_constant<int, Is>{}), ...);
}

struct TailArgs {
  int M;
  const bf16* act;      // PRE: att [M, D]; else x1 [M, D]
  const bf16* resid;    // PRE: x (residual of LN1) [M, D]
  bf16* out;            // [M, D] (PRE: may alias resid)
  const char* ws;       // weight stream (snvrag_tail_pack)
  const float* vec;     // [b1 4D | b2' | c1 | g2 | be2]
  const float* b_o; const float* g1; const float* be1;
  float eps;
  unsigned long long* stamps;   // VAR 2 (diagnostics): [workgroup][wave][TL_NSTAMP] s_memtime stamps
  int desync;                   // > 0: first-round phase step in cycles (see tail_kernel)
};

// diagnostic stamp points of VAR 2 (slot 0: s_memrealtime at entry, 1..: s_memtime)
constexpr int TL_NSTAMP = 10;
enum { TS_REAL0 = 0, TS_START, TS_PROLOGUE, TS_PROJ, TS_LN1, TS_FFN, TS_EPI, TS_END, TS_REAL1 };

// VAR (diagnostics): 0 default; 1 = no weight DMA after the prologue (compute-side ceiling;
// results are garbage); 2 = the default kernel plus per-wave s_memtime stamps at the phase
// boundaries into p.stamps (a separate instantiation: no stamp executes in the real kernel);
// 3 = residual added early (see RR_G).  TL_SGB: shape each slab's schedule as MFMA f / read f + PF pairs.
// SNVRAG_TAIL_VARIANT (launch_tail): 1 = PF 8, 2 = VAR 1, 3 = no schedule groups, 4 = VAR 2
// (stamps), 5 = VAR 3.
// NC > 0: projection mode (snvrag_proj_forward): out[M, NC*D] = act W^T + b over NC output
// chunks of D features (the QKV projection: NC = 3), the same stream / ring / read machinery.
template <int D, bool PRE, int TL_PF = TL_PF4, int VAR = 0, bool TL_SGB = true, int NC = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void tail_kernel(TailArgs p) {
  using S = TailShape<D>;
  constexpr int NT = S::NT, KS = S::KS;
  constexpr bool PROJ = NC > 0;
  static_assert(!(PROJ && PRE), "modes");
  constexpr int NSLAB = (PRE ? S::NPRE : 0) + S::NCH * S::SPC;      // slabs consumed by this launch
  constexpr int RING = TL_NSLOT * TL_SLAB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* sv = reinterpret_cast<float*>(smem + RING);               // b1 [4D], g1, be1, b_o
  // wave index as a scalar: every LDS / stream offset below stays in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x, lane = tid & 63;
  const int ln = lane & 31, hh = lane >> 5;
  const long row = (long)blockIdx.x * TL_ROWS + wave * 32 + ln;
  const long rc = row < p.M ? row : (long)p.M - 1;
  // (VAR 2) stamp: every lane writes the same value to the same slot through a vector store
  // (branch-free: an exec-masked store splits the unrolled stream into blocks and changes the
  // register allocation being measured)
  auto stamp = [&](int slot, bool real = false) {
    if constexpr (VAR == 2) {
      const unsigned long long t = real ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
      __builtin_nontemporal_store(t, p.stamps + ((long)blockIdx.x * 4 + wave) * TL_NSTAMP + slot);
    }
  };
  stamp(TS_REAL0, true);
  // De-synchronised rounds: every workgroup runs the same weight stream for the same time, so
  // without this all 256 CUs start each round together and the prologue's activation + residual
  // loads (192 KB per CU) and the epilogue's stores hit HBM as one chip-wide burst (measured:
  // prologue 12 % of the wave, HBM-bound at ~4 TB/s, then idle HBM for the rest of the round).
  // The first round's workgroups start at 8 phase offsets of `desync` cycles (per XCD: dispatch
  // order blockIdx / 8), so later rounds stay spread and each CU's bursts overlap other CUs'
  // MFMA phases.  The delay is paid once per CU; with >= 17 blocks per CU it ends inside the
  // last partial round's slack.
  if (p.desync > 0 && blockIdx.x < 256) {
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }
  stamp(TS_START);

  // ---- vector tables to LDS first (their loads are waited on at once), then the activations
  // as B fragments (k-step s: features tail_in_feat(s, hh, 0..7)); the residual rows of PRE are
  // loaded after the weight prologue (below) and only needed at LN1, so their HBM burst runs
  // under the out-projection MFMAs
  for (int i = tid; i < (PROJ ? NC : 4) * D; i += 256) sv[i] = p.vec[i];
  if constexpr (PRE)
    for (int i = tid; i < D; i += 256) { sv[4 * D + i] = p.g1[i]; sv[5 * D + i] = p.be1[i]; sv[6 * D + i] = p.b_o[i]; }
  u32x4 xr[KS];                                      // x1 B fragments (PRE: produced by LN1)
  u32x4 xa[(PRE || PROJ) ? KS : 1];                  // PRE: att B fragments; PROJ: x
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    // (default cache policy: non-temporal activation loads/stores measured 8 % slower)
    const u32x4 v = *reinterpret_cast<const u32x4*>(p.act + rc * D + tail_in_feat(s, hh, 0));
    if constexpr (PRE || PROJ) xa[s] = v; else xr[s] = v;
  }

  // ---- weight stream: buffer_load ... lds with scalar offsets; chunks rotated per workgroup
  const int rot = (int)(blockIdx.x % (PROJ ? NC : S::NCH));
  constexpr int STREAM_SLABS = PROJ ? NC * S::NPRE : S::NSLAB;
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ws, (short)0, STREAM_SLABS * TL_SLAB, 0x00020000);
  const int voff = lane * 16;
  // FFN block order (software pipeline, see the chunk loop): with the stream's blocks
  // B(2c) = W1(c), B(2c+1) = W2'(c) (H slabs each) and r = rot, block s of the launch is
  //   s = 0: W1(r);  s = 2k-1 < 2N-1: W1(r+k) = B(2r+s+1);  s = 2k >= 2: W2'(r+k-1) = B(2r+s-1);
  //   s = 2N-1: W2'(r+N-1) = B(2r+s)   (block indices mod 2N)
  constexpr int H = S::FW1 / 16;                     // slabs per W1 (= per W2') block
  constexpr int NB2 = 2 * S::NCH;
  int is_slot = 0;                                   // ring slot (byte offset) of the next issue
  int is_i = 0;                                      // launch slab index of the next issue
  // stream byte offset of launch slab is_i, branch-free (selects only: a branch here splits the
  // unrolled MFMA stream into basic blocks and the register allocator then spills across them)
  auto src_of = [&](int i) -> int {
    if constexpr (PROJ) {                            // chunks rot, rot + 1, ... (mod NC), NPRE slabs each
      const int cc = i / S::NPRE, j = i - cc * S::NPRE;
      const int c = (rot + cc) % NC;
      return (c * S::NPRE + j) * TL_SLAB;
    }
    constexpr int NP = PRE ? S::NPRE : 0;
    const int q = i - NP > 0 ? i - NP : 0;
    const int s = q / H, j = q - s * H;              // FFN block, slab within it
    int m = 2 * rot + s + ((s == 0 || s == NB2 - 1) ? 0 : (s & 1) ? 1 : -1);
    m = m >= NB2 ? m - NB2 : m;
    m = m >= NB2 ? m - NB2 : m;                      // (overrun issues run past s = 2N - 1)
    const int ffn = (S::NPRE + m * H + j) * TL_SLAB;
    return i < NP ? i * TL_SLAB : ffn;
  };
  // Issues run NSLOT - 2 slabs past the end of the launch's stream (the wrapped stream
  // continues, so the addresses stay valid): every sync then has the same number of slabs in
  // flight behind the one it waits for — one constant vmcnt, no per-slab branches.  The
  // overrun lands in slots nobody reads; the epilogue drains it before reusing the ring.
  auto issue_next = [&]() {
    auto* dst = (__attribute__((address_space(3))) void*)(ring + is_slot + wave * 4 * TL_FRAG);
    const int src = src_of(is_i);
    ++is_i;
    tl_unroll([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      // (instruction offset 0: the slab offset rides in soffset, the LDS slot in M0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) char*)dst + j * TL_FRAG, 16,
                                               voff, src + (wave * 4 + j) * TL_FRAG, 0, 0);
    }, std::make_integer_sequence<int, 4>{});
    is_slot = is_slot + TL_SLAB == RING ? 0 : is_slot + TL_SLAB;
  };
#pragma unroll
  for (int g = 0; g < TL_NSLOT - 1; ++g) issue_next();
  // PRE: the residual rows x, behind the weight prologue in the vmcnt order (NRR loads)
  constexpr int NRR = PRE ? 2 * NT : 0;
  u32x4 rr[PRE ? 2 * NT : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        rr[2 * T + h2] = *reinterpret_cast<const u32x4*>(p.resid + rc * D + 32 * T + 16 * hh + 8 * h2);
  }
  static_assert(4 * (TL_NSLOT - 2) + NRR <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (TL_NSLOT - 2) + NRR) : "memory");
  __syncthreads();                                   // slab 0, the activations + the vector tables visible
  stamp(TS_PROLOGUE);

  // read side: rd_slot = ring slot of the current part's first slab
  int rd_slot = 0;
  auto rdA = [&](auto j_tag, auto fi_tag) -> u32x4 {   // fragment fi of the part's slab j
    constexpr int j = decltype(j_tag)::value, fi = decltype(fi_tag)::value;
    int so = rd_slot + j * TL_SLAB;
    so = so >= RING ? so - RING : so;
    return *reinterpret_cast<const u32x4*>(ring + so + lane * 16 + fi * TL_FRAG);
  };
  // sync before the first read of slab g (reached PF fragments before its boundary)
  // (g is a compile-time constant where it matters: PRE's first NSLOT - 2 slabs, issued before
  // the residual loads, have those NRR loads behind them in the vmcnt order)
  auto sync = [&](auto g_tag) {
    constexpr int g = decltype(g_tag)::value;
    if constexpr (VAR == 1) {
      __builtin_amdgcn_s_barrier();
      return;
    }
    if constexpr (PRE && g >= 0 && g <= TL_NSLOT - 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (TL_NSLOT - 3) + NRR) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (TL_NSLOT - 3)) : "memory");
    __builtin_amdgcn_s_barrier();
    issue_next();                                    // slab g - 2 + NSLOT into the slot of slab g - 2
  };

  u32x4 a[TL_PF];

  // consume NF fragments (whole slabs) of the part starting at ring slot rd_slot: mma(f, A) per
  // fragment, LDS reads PF ahead (into the next part), one sync per slab
  // G0: the part's first launch slab when known at compile time (PRE), else -1
  // STOP: no reads past the part (the caller re-primes a[] with prime() before the next part)
  auto run = [&](auto nf_tag, auto g0_tag, auto&& mma, auto stop_tag) {
    constexpr int NF = decltype(nf_tag)::value;
    constexpr int G0 = decltype(g0_tag)::value;
    constexpr bool STOP = decltype(stop_tag)::value;
    static_assert(NF % 16 == 0, "parts are whole slabs");
    tl_unroll([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      const u32x4 cur = a[f % TL_PF];
      if constexpr ((f & 15) == 16 - TL_PF) {
        // fence the scheduler at every slab sync: bounds the register live ranges of the
        // fully unrolled stream (hipcc otherwise hoists work across slabs and spills)
        __builtin_amdgcn_sched_barrier(0);
        sync(std::integral_constant<int, (G0 < 0 ? -1 : G0 + (f >> 4) + 1)>{});
      }
      mma(fc, cur);
      // (past the end of the stream this reads stale ring bytes that are never used)
      constexpr int qn = f + TL_PF;
      if constexpr (!STOP || qn < NF)
        a[f % TL_PF] = rdA(std::integral_constant<int, (qn >> 4)>{}, std::integral_constant<int, (qn & 15)>{});
      if constexpr (TL_SGB) {
        // pipeline shape for the scheduler: MFMA f, then the read PF fragments ahead
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }, std::make_integer_sequence<int, NF>{});
    rd_slot += (NF / 16) * TL_SLAB;
    rd_slot = rd_slot >= RING ? rd_slot - RING : rd_slot;
  };
  auto prime = [&]() {
    tl_unroll([&](auto ic) { a[decltype(ic)::value] = rdA(std::integral_constant<int, 0>{}, ic); },
              std::make_integer_sequence<int, TL_PF>{});
  };

  // (ao: out-projection accumulators; acc: FFN accumulators, born in the first chunk with a zero
  // C operand — explicit zero vectors here get materialised in VGPRs and spilled)
  f32x16 acc[NT];
  prime();
  if constexpr (PROJ) {
    // ---- per output chunk: acc = x W_c^T (zero C operand at k-step 0); + bias -> bf16 in yo.
    // The NT x 2 stores of chunk c go out PPS per slab during chunk c + 1's stream (bounds-
    // checked buffer stores: rows >= M fall outside the resource and are dropped): a burst of
    // stores right before a sync would hold that sync's vmcnt wait until they completed.
    const uint32_t sv_lane = tl_lds(reinterpret_cast<const char*>(sv)) + 64 * hh;   // &sv[16 hh]
    const long out_bytes = (long)p.M * NC * D * 2;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.out, (short)0, (int)(out_bytes < 0x7fffffffL ? out_bytes : 0x7fffffffL), 0x00020000);
    const int row_off = (int)(row * (NC * D) + 16 * hh) * 2;          // bytes; row < 2^31 / (2 NC D)
    constexpr int PPS = (NT + S::NPRE - 1) / S::NPRE;                 // store pairs per slab
    u32x4 yo[2 * NT];
    int yo_off = 0;                                                   // byte offset of yo's chunk
    auto store_pair = [&](auto t_tag) {
      constexpr int T = decltype(t_tag)::value;
      if constexpr (T < NT) {
        __builtin_amdgcn_raw_buffer_store_b128(yo[2 * T], ors, yo_off + 64 * T, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(yo[2 * T + 1], ors, yo_off + 64 * T + 16, 0, 0);
      }
    };
    auto chunk = [&](int c, auto stores_tag) {
      constexpr bool STORES = decltype(stores_tag)::value;
      tl_unroll([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        run(std::integral_constant<int, 4 * NT>{}, std::integral_constant<int, -1>{}, [&](auto fc, const u32x4& A) {
          constexpr int f = decltype(fc)::value;
          if constexpr (g == 0 && f < NT) acc[f] = mfma32(A, xa[f / NT], f32x16{});
          else acc[f % NT] = mfma32(A, xa[4 * g + f / NT], acc[f % NT]);
          if constexpr (STORES && (f & 15) == 16 - TL_PF) {
            constexpr int slab = g * (NT / 4) + (f >> 4);
            tl_unroll([&](auto pc) { store_pair(std::integral_constant<int, slab * PPS + decltype(pc)::value>{}); },
                      std::make_integer_sequence<int, PPS>{});
          }
        }, std::false_type{});
      }, std::make_integer_sequence<int, KS / 4>{});
#pragma unroll
      for (int T = 0; T < NT; ++T) {
        // bias of features c D + 32 T + 16 hh + 0..15 (reads + wait in one asm: a compiler LDS
        // read would wait for the whole in-flight weight stream, see the FFN bias)
        u32x4 bv[4];
        asm volatile(
            "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
            " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
            : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
            : "v"(sv_lane + 4 * (c * D + 32 * T)));
        float y[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = acc[T][i] + __uint_as_float(bv[i >> 2][i & 3]);
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          yo[2 * T + h2] = u32x4{tl_pack2(y[8 * h2], y[8 * h2 + 1]), tl_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                                 tl_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tl_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
      }
      yo_off = row_off + c * D * 2;
    };
    chunk(rot, std::false_type{});
#pragma unroll 1
    for (int cc = 1; cc < NC; ++cc) chunk((rot + cc) % NC, std::true_type{});
    tl_unroll([&](auto tc) { store_pair(tc); }, std::make_integer_sequence<int, NT>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stream overrun has landed before exit
    return;
  }
  if constexpr (PRE) {
    // PRE: the out-projection accumulates onto b_o; LN1 adds the residual x (loaded late, see rr)
    f32x16 ao[NT];
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int i = 0; i < 16; ++i) ao[T][i] = sv[6 * D + 32 * T + 16 * hh + i];
    // ---- ao += att W_o'^T;  fragment f: k-step f / NT, tile f % NT.  A runtime loop over
    // groups of 4 k-steps (4 NT fragments = whole slabs): the att fragments of the group are
    // xa[0..3], shifted down after each group (a straight-line 288-MFMA body makes hipcc
    // shuffle the accumulators between AGPRs)
    static_assert(KS % 4 == 0 && (4 * NT) % 16 == 0, "groups of 4 k-steps are whole slabs");
    // VAR 3 (diagnostics): the residual x added into ao at the start of group 3 instead of in
    // LN1's first pass (frees its registers before LN1, but waits for the residual burst earlier:
    // measured slower, tools/tail_micro.py)
    constexpr int RR_G = (VAR == 3 && KS / 4 > 3) ? 3 : -1;
    tl_unroll([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g == RR_G) {
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
          for (int i = 0; i < 16; ++i) ao[T][i] += tl_bf(rr[2 * T + (i >> 3)], i & 7);
      }
      run(std::integral_constant<int, 4 * NT>{}, std::integral_constant<int, g * (NT / 4)>{}, [&](auto fc, const u32x4& A) {
        constexpr int f = decltype(fc)::value;
        ao[f % NT] = mfma32(A, xa[4 * g + f / NT], ao[f % NT]);
      }, std::bool_constant<g == KS / 4 - 1>{});
    }, std::make_integer_sequence<int, KS / 4>{});
    stamp(TS_PROJ);
    // ---- x1 = LN1(ao) -> xr (B fragments): pass 1 sums v and v^2, pass 2 normalises
    // (v re-read from the AGPR accumulators, never all held in VGPRs)
    float sum = 0.f, sq = 0.f;
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float v = ao[T][i];
        if constexpr (RR_G < 0) {
          v += tl_bf(rr[2 * T + (i >> 3)], i & 7);
          ao[T][i] = v;
        }
        sum += v;
        sq = fmaf(v, v, sq);
      }
#pragma unroll
    for (int T = 0; T < NT; ++T) asm volatile("" : "+a"(ao[T]));
    asm volatile("" ::: "memory");
    sum = tl_xsum32(sum);
    sq = tl_xsum32(sq);
    const float mean = sum * (1.0f / D);
    const float rstd = 1.0f / sqrtf(fmaxf(sq * (1.0f / D) - mean * mean, 0.f) + p.eps);
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      float y[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ft = 32 * T + 16 * hh + i;
        y[i] = (ao[T][i] - mean) * rstd * sv[4 * D + ft] + sv[5 * D + ft];
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        xr[2 * T + h2] = u32x4{tl_pack2(y[8 * h2], y[8 * h2 + 1]), tl_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                               tl_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tl_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
    }
    // the FFN's first fragments are read only now: read ahead across LN1 they were live through
    // it and spilled, and their scratch reloads waited on vmcnt(0), i.e. drained the weight ring
    prime();
  }
  stamp(TS_LN1);
  // x1 opaque from here on: otherwise hipcc folds the epilogue's bf16 -> f32 unpacking of x1
  // into LN1 (it knows pack(y)) and carries 192 unpacked floats through the FFN loop
#pragma unroll
  for (int k = 0; k < KS; ++k) asm volatile("" : "+v"(xr[k]));

  // ---- FFN over 64-unit hidden chunks, software-pipelined: the MFMAs of phase 1 (W1) of
  // chunk k run while the VALU epilogue of chunk k-1 (LeakyReLU, LN_f sums, bf16 packing of
  // its hidden into phase-2 B fragments) is interleaved between them; then phase 2 (W2') of
  // chunk k-1.  Stream order: W1(0), W1(1), W2'(0), W1(2), W2'(1), ..., W2'(N-1).
  float st1 = 0.f, st2 = 0.f;
  const uint32_t sv_lane = tl_lds(reinterpret_cast<const char*>(sv)) + 16 * hh;
  f32x16 h0[2], h1[2];                               // hidden of even / odd chunks (ping-pong)
  u32x4 hf[4];                                       // phase-2 B fragments (k-step 2t + q)
  auto epi_pair = [&](const f32x16 (&hc)[2], int m) {   // hidden values 2m, 2m+1 of hc (m < 16)
    const int t = m >> 3, i = 2 * (m & 7);
    float x0 = hc[t][i], x1 = hc[t][i + 1];
    x0 = tl_lrelu(x0);
    x1 = tl_lrelu(x1);
    st1 += x0 + x1;
    st2 = fmaf(x0, x0, fmaf(x1, x1, st2));
    hf[2 * t + (i >> 3)][(i & 7) >> 1] = tl_pack2(x0, x1);
  };
  // phase 1 of chunk k into hn: h^T = W1_c x1^T + b1 (fragment f: k-step f / 2, tile f % 2; the
  // bias is the C operand of the first k-step, hidden unit of acc element i: 8(i/4) + 4hh + i%4),
  // with the epilogue of the previous chunk (hc) interleaved when EPI
  auto phase1 = [&](int k, f32x16 (&hn)[2], const f32x16 (&hc)[2], auto epi_tag) {
    constexpr bool EPI = decltype(epi_tag)::value;
    const int c = k + rot >= S::NCH ? k + rot - S::NCH : k + rot;
    const uint32_t b1 = sv_lane + 256 * c;          // &sv[64 c + 4 hh]
    u32x4 bv[8];
    // bv[r] = floats 32 (r / 4) + 8 (r % 4) .. + 3 of the chunk's bias: reads and their wait in ONE
    // asm statement (outputs early-clobber: the address stays intact until the last read)
    asm volatile(
        "ds_read_b128 %0, %8 offset:0\n ds_read_b128 %1, %8 offset:32\n ds_read_b128 %2, %8 offset:64\n"
        " ds_read_b128 %3, %8 offset:96\n ds_read_b128 %4, %8 offset:128\n ds_read_b128 %5, %8 offset:160\n"
        " ds_read_b128 %6, %8 offset:192\n ds_read_b128 %7, %8 offset:224\n s_waitcnt lgkmcnt(0)"
        : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3]), "=&v"(bv[4]), "=&v"(bv[5]), "=&v"(bv[6]), "=&v"(bv[7])
        : "v"(b1));
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) hn[t][4 * r + e] = __uint_as_float(bv[4 * t + r][e]);
    run(std::integral_constant<int, S::FW1>{}, std::integral_constant<int, -1>{}, [&](auto fc, const u32x4& A) {
      constexpr int f = decltype(fc)::value;
      hn[f & 1] = mfma32(A, xr[f >> 1], hn[f & 1]);
      constexpr int SP = S::FW1 / 16;                // 16 epilogue pairs spread over the MFMAs
      if constexpr (EPI && f % SP == 0) epi_pair(hc, f / SP);
    }, std::false_type{});
  };
  // phase 2 of the chunk whose hidden sits in hf: out^T += W2'_c h_c^T (fragment f: k-step
  // f / NT, output tile f % NT); the first one starts acc with a zero C operand
  auto phase2 = [&](auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    run(std::integral_constant<int, S::FW2>{}, std::integral_constant<int, -1>{}, [&](auto fc, const u32x4& A) {
      constexpr int f = decltype(fc)::value;
      if constexpr (FIRST && f < NT) acc[f] = mfma32(A, hf[0], f32x16{});
      else acc[f % NT] = mfma32(A, hf[f / NT], acc[f % NT]);
    }, std::false_type{});
  };
  // even chunks in h0, odd in h1: no hidden copies (a loop-carried copy makes hipcc shuffle
  // the accumulator registers at every back edge)
  static_assert(S::NCH % 2 == 0 && S::NCH >= 4, "chunk pairs");
  phase1(0, h0, h1, std::false_type{});
  phase1(1, h1, h0, std::true_type{});
  phase2(std::true_type{});
  phase1(2, h0, h1, std::true_type{});
  phase2(std::false_type{});
#pragma unroll 1
  for (int k = 3; k + 1 < S::NCH; k += 2) {
    phase1(k, h1, h0, std::true_type{});
    phase2(std::false_type{});
    phase1(k + 1, h0, h1, std::true_type{});
    phase2(std::false_type{});
  }
  phase1(S::NCH - 1, h1, h0, std::true_type{});
  phase2(std::false_type{});
#pragma unroll
  for (int m = 0; m < 16; ++m) epi_pair(h1, m);
  phase2(std::false_type{});

  stamp(TS_FFN);
  // ---- epilogue: out = LN2(x1 + lrelu(rstd_f acc - rstd_f mean_f c1 + b2'))
  st1 = tl_xsum32(st1);
  st2 = tl_xsum32(st2);
  const float hm = st1 * (1.0f / (4 * D));
  const float hr = 1.0f / sqrtf(fmaxf(st2 * (1.0f / (4 * D)) - hm * hm, 0.f) + p.eps);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the stream overrun has landed
  __syncthreads();                                   // every wave is done with the ring
  float* ev = reinterpret_cast<float*>(ring);        // [b2' | c1 | g2 | be2]
  for (int i = wave * 64 + tl_lane(); i < 4 * D; i += 256) ev[i] = p.vec[4 * D + i];   // fresh tid (no spill)
  __syncthreads();
  stamp(TS_EPI);
  const float* b2 = ev;
  const float* c1 = ev + D;
  const float* g2 = ev + 2 * D;
  const float* be2 = ev + 3 * D;
  // pass 1: v = x1 + lrelu(rstd_f (acc - mean_f c1) + b2') written back over acc, sums of v and
  // v^2; pass 2 normalises v in place of acc and stores
  float sum = 0.f, sq = 0.f;
#pragma unroll
  for (int T = 0; T < NT; ++T)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ft = 32 * T + 16 * hh + i;
      float u = hr * fmaf(-hm, c1[ft], acc[T][i]) + b2[ft];
      u = tl_lrelu(u);
      const float v = u + tl_bf(xr[2 * T + (i >> 3)], i & 7);
      acc[T][i] = v;
      sum += v;
      sq = fmaf(v, v, sq);
      // one tile's vector-table reads at a time: hoisted over all tiles they held ~30 registers
      // while x1 is still live, and x1 was spilled during the last chunk
      if (i == 15) asm volatile("" ::: "memory");
    }
#pragma unroll
  for (int T = 0; T < NT; ++T) asm volatile("" : "+a"(acc[T]));
  asm volatile("" ::: "memory");
  sum = tl_xsum32(sum);
  sq = tl_xsum32(sq);
  const float mean = sum * (1.0f / D);
  const float rstd = 1.0f / sqrtf(fmaxf(sq * (1.0f / D) - mean * mean, 0.f) + p.eps);
  const float nmr = -mean * rstd;
  auto v2 = [&](int T, int i) { return fmaf(acc[T][i], rstd, nmr); };
  // the row recomputed from a fresh lane id (kept live from the prologue it was spilled)
  const long row_e = (long)blockIdx.x * TL_ROWS + wave * 32 + (tl_lane() & 31);
  if (row_e < p.M) {
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      float y[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ft = 32 * T + 16 * hh + i;
        y[i] = fmaf(v2(T, i), g2[ft], be2[ft]);
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        *reinterpret_cast<u32x4*>(p.out + row_e * D + 32 * T + 16 * hh + 8 * h2) =
            u32x4{tl_pack2(y[8 * h2], y[8 * h2 + 1]), tl_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                  tl_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tl_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
    }
  }
  if constexpr (VAR == 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the row stores have left
    stamp(TS_END);
    stamp(TS_REAL1, true);
  }
}

// ---------------------------------------------------------------------------------------------
// PERSISTENT block tail (PRE mode, the engine's path): one workgroup per CU loops over 128-row
// tiles (tile = blockIdx.x, + gridDim.x, ...) with ONE continuous LDS-DMA ring across them.  Per
// tile the ring streams, in consumption order,
//   A  the tile's attention rows  (KS / 4 slabs; wave w's pieces = its 32 rows, 4 k-steps each)
//   Wo the W_o' fragments         (NPRE slabs)
//   R  the tile's residual rows x (KS / 4 slabs; features 32 T + 16 hh + 8 h2 per piece)
//   W1 / W2' chunk blocks         (NCH x SPC slabs, the per-workgroup rotation of tail_kernel)
// so the activations of tile t + 1 arrive by DMA while tile t finishes its FFN, instead of every
// workgroup waiting on a 192 KB HBM burst of its own before its first MFMA (tail_kernel: the
// prologue was 12 % of a wave's cycles, the ring drain + epilogue table loads another ~4 %).  The
// epilogue's vector tables stay in LDS for the whole launch (8-slot ring: 128 KiB + 11 D floats).
// The arithmetic is tail_kernel's, in the same order: outputs are bit-identical to it.
// LDS-DMA is issued by inline asm (dma_x4): the compiler sees no LDS stores, so its own LDS reads
// (vector tables, A / R pieces) get no waits on the weight stream; the ordering is this kernel's
// counted vmcnt + barrier.  The 2 NT epilogue stores of a tile are buffer stores (rows >= M fall
// outside the resource), so every tile issues the same vector-memory count and the first syncs of
// the next tile wait with that count added.
constexpr int TP_NSLOT = 8;

// STAMP (diagnostics, a separate instantiation): s_memtime at the phase boundaries of each tile,
// the last tile's kept in SGPRs and written out at exit: [workgroup][wave][TP_NSTAMP] u32
constexpr int TP_NSTAMP = 8;
template <int D, bool STAMP = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void tailp_kernel(TailArgs p) {
  using S = TailShape<D>;
  constexpr int NT = S::NT, KS = S::KS;
  constexpr int NA = KS / 4;                          // A (and R) slabs per tile
  // per tile, NA groups of GS slabs: [A_g, W_o' (NT / 4 slabs: k-steps 4 g .. 4 g + 3), R_g],
  // then the FFN: the activation slabs are consumed beside the out-projection's MFMAs, never
  // several in a row (a run of MFMA-free slabs would use up the ring's lookahead)
  constexpr int WPG = NT / 4;                         // W_o' slabs per group
  constexpr int GS = WPG + 2;
  constexpr int Q_FFN = NA * GS;
  static_assert(S::NPRE == NA * WPG, "W_o' groups");
  constexpr int NQ = Q_FFN + S::NCH * S::SPC;         // slabs per tile
  constexpr int AHEAD = TP_NSLOT - 2;                 // sync(g) issues slab g + AHEAD
  constexpr int RING = TP_NSLOT * TL_SLAB;
  constexpr int VM = 4 * (TP_NSLOT - 3);              // vmcnt at a sync: the younger slabs in flight
  constexpr int NST = 2 * NT;                         // epilogue stores per lane and tile
  constexpr int H = S::FW1 / 16;                      // slabs per W1 / W2' block
  constexpr int NB2 = 2 * S::NCH;                     // FFN blocks per tile
  static_assert(VM + NST <= 63, "vmcnt range");
  static_assert(KS % 4 == 0 && H == S::FW2 / 16, "whole A / R slabs, equal W1 / W2' blocks");
  // FFN block layout of a tile: phase1(0), phase1(1), phase2, phase1(2), phase2, then a runtime
  // loop of 4 blocks per iteration over chunks 3 .. NCH - 4, its last iteration peeled (compile-time
  // issue targets there: the last block W2'(N-1) breaks the loop's block pattern), then
  // phase1(NCH - 1), phase2, phase2
  // loop iterations (chunk pairs 3 .. NCH - 2): the runtime ones are those whose issue targets
  // (AHEAD slabs past their last part) stay inside plain blocks; the rest are unrolled
  constexpr int NIT = (S::NCH - 4) / 2;
  constexpr int LIT_MAX = ((NB2 - 1) * H - 1 - AHEAD - 9 * H);
  constexpr int LOOP_IT = LIT_MAX < 0 ? 0 : (LIT_MAX / (4 * H) + 1 < NIT ? LIT_MAX / (4 * H) + 1 : NIT);
  static_assert(S::NCH % 2 == 0 && S::NCH >= 6, "chunk pairs");
  constexpr int Q_LOOP = Q_FFN + 5 * H;               // first slab of the loop
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* sv = reinterpret_cast<float*>(smem + RING);  // [b1 4D | b2' | c1 | g2 | be2 | g1 | be1 | b_o]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x, lane = tid & 63;
  const int hh = lane >> 5;
  const int M = p.M;
  const int ntiles = (M + TL_ROWS - 1) / TL_ROWS;
  const int G = gridDim.x;

  for (int i = tid; i < 8 * D; i += 256) sv[i] = p.vec[i];
  for (int i = tid; i < D; i += 256) { sv[8 * D + i] = p.g1[i]; sv[9 * D + i] = p.be1[i]; sv[10 * D + i] = p.b_o[i]; }
  // first-tile stagger (tail_kernel's desync), only for the workgroups with one tile fewer: their
  // slack absorbs it
  if (p.desync > 0 && ntiles % G != 0 && (int)blockIdx.x >= ntiles % G && ntiles >= 8 * G) {
    const long wait = (long)p.desync * ((blockIdx.x >> 3) & 7);
    const long t0 = (long)__builtin_amdgcn_s_memtime();
    while ((long)__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  }

  // ---- issue side.  Every issue target is a compile-time tile-relative slab index (the loop's
  // are compile-time offsets from the iteration's runtime block base), so an issue is a few scalar
  // adds: the weight stream offset of an FFN block is (NPRE + H m) slabs with m = 2 rot + s + d(s)
  // mod 2 NCH (tail_kernel's rotated order), the activation pieces through a resource starting at
  // the tile's rows (rows >= M, and tiles >= ntiles, read as zeros).
  const int rot2 = 2 * (int)(blockIdx.x % S::NCH);
  const i32x4 wrs = dma_rsrc(p.ws, (long)S::NSLAB * TL_SLAB);
  const uint32_t ring_lds = lds_addr(ring) + wave * 4 * TL_FRAG;
  const int wave_off = wave * 4 * TL_FRAG;
  int is_slot = 0;                                    // ring slot (byte offset) of the next issue
  long tb = (long)blockIdx.x * TL_ROWS * D * 2;       // byte offset of the current tile's rows
  constexpr int TB_STEP = TL_ROWS * D * 2;
  // wave-uniform values made opaque at each use: otherwise hipcc precomputes every issue's
  // offset (each a loop-invariant scalar) before the tile loop and spills ~250 SGPRs
  auto opq = [](auto v) { asm volatile("" : "+s"(v)); return v; };
  // A / R piece j of this wave: 8 of its rows x the slab's 128 B of each (4 k-steps / 2 residual
  // tiles), i.e. 8 whole 128-B lines per DMA instruction; LDS image [32 rows][128 B] with the
  // 16-B chunks XOR-swizzled by row & 7 (conflict-free fragment reads): lane l fills row
  // 8 j + l / 8, slot l % 8, so it loads chunk (l % 8) ^ (row % 8).  From a fresh lane id.
  auto voff_act = [&](int j) {
    const int l = tl_lane();
    return (opq(wave) * 32 + 8 * j + (l >> 3)) * (D * 2) + 16 * ((l & 7) ^ ((l >> 3) & 7));
  };
  auto put = [&](const i32x4& rs, int soff, bool act) {
    const int lds = opq(ring_lds) + is_slot;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      dma_x4(rs, lds + j * TL_FRAG, act ? voff_act(j) : tl_lane() * 16, act ? soff : soff + j * TL_FRAG);
    is_slot = is_slot + TL_SLAB == RING ? 0 : is_slot + TL_SLAB;
  };
  auto ffn_off = [&](int m) {                         // m in [0, 2 NB2)
    m = m >= NB2 ? m - NB2 : m;
    return (S::NPRE * TL_SLAB) + m * (H * TL_SLAB);
  };
  // target QG: tile-relative slab (>= NQ: the next tile's); compile-time
  auto issue_ct = [&](auto q_tag) {
    constexpr int QG = decltype(q_tag)::value;
    constexpr bool NEXT = QG >= NQ;
    constexpr int q = NEXT ? QG - NQ : QG;
    constexpr int gq = q / GS, rq = q % GS;
    if constexpr (q < Q_FFN && (rq == 0 || rq == GS - 1)) {
      // A_g / R_g.  A resource over the tile's rows to the end of the array: the buffer range
      // check covers voffset, not soffset, so the tile offset goes into the base (rows >= M read
      // as zeros)
      const long tbl = NEXT ? opq(tb) + (long)G * TB_STEP : opq(tb);
      const long left = (long)M * D * 2 - tbl;
      const char* base = reinterpret_cast<const char*>(rq == 0 ? p.act : p.resid);
      put(dma_rsrc(base + (left > 0 ? tbl : 0), left > 0 ? left : 0), 128 * gq, true);
    } else if constexpr (q < Q_FFN) {
      put(wrs, (gq * WPG + rq - 1) * TL_SLAB + opq(wave_off), false);
    } else {
      constexpr int qq = q - Q_FFN, sb = qq / H, jb = qq % H;
      constexpr int d = (sb == 0 || sb == NB2 - 1) ? 0 : (sb & 1) ? 1 : -1;
      put(wrs, ffn_off(opq(rot2) + sb + d) + jb * TL_SLAB + opq(wave_off), false);
    }
  };
  // loop target: slab Q_LOOP + AHEAD + 4 H it + C; mloop = rot2 + 4 it (runtime)
  auto issue_loop = [&](auto c_tag, int mloop) {
    constexpr int C = decltype(c_tag)::value;
    constexpr int qq = Q_LOOP + AHEAD - Q_FFN + C, sb = qq / H, jb = qq % H;   // block of iteration 0
    constexpr int d = (sb & 1) ? 1 : -1;
    static_assert(sb > 0 && sb + 4 * (LOOP_IT - 1) < NB2 - 1, "loop targets are plain blocks");
    put(wrs, ffn_off(mloop + sb + d) + jb * TL_SLAB + opq(wave_off), false);
  };
  // the vector tables landed (plain loads), then the first AHEAD slabs
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  tl_unroll([&](auto gc) { issue_ct(gc); }, std::make_integer_sequence<int, AHEAD>{});

  // sync before reading slab g: it has landed (this wave's pieces: vmcnt; the others': barrier)
  auto wait_bar = [&](auto vm_tag) {
    constexpr int V = decltype(vm_tag)::value;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(V) : "memory");
    __builtin_amdgcn_s_barrier();
  };
  using VMc = std::integral_constant<int, VM>;
  using VMs = std::integral_constant<int, VM + NST>;
  // the syncs of a tile's slabs 1 .. AHEAD: issued before the previous tile's epilogue stores (the
  // first tile issues as many no-op stores at the same point), so those are among the younger
  auto vm_of = [](auto g_tag) {
    constexpr int g = decltype(g_tag)::value;
    return std::conditional_t<(g >= 1 && g <= AHEAD), VMs, VMc>{};
  };
  // sync of compile-time slab G (then slab G + AHEAD goes into the slot of slab G - 2)
  auto sync_ct = [&](auto g_tag, auto vm_tag) {
    wait_bar(vm_tag);
    issue_ct(std::integral_constant<int, decltype(g_tag)::value + AHEAD>{});
  };

  int rd_slot = 0;
  auto rdA = [&](auto j_tag, auto fi_tag) -> u32x4 {
    constexpr int j = decltype(j_tag)::value, fi = decltype(fi_tag)::value;
    int so = rd_slot + j * TL_SLAB;
    so = so >= RING ? so - RING : so;
    return *reinterpret_cast<const u32x4*>(ring + so + lane * 16 + fi * TL_FRAG);
  };
  // B fragment j of this wave's rows in the current A / R slab (features 64 slab + 32 (j / 2) +
  // 16 hh + 8 (j % 2) .. + 7 of row ln: 16-B chunk 4 (j / 2) + 2 hh + j % 2 of the row's 128 B)
  auto rdOwn = [&](int j) -> u32x4 {
    const int l = tl_lane(), ln = l & 31;
    const int c = 4 * (j >> 1) + 2 * (l >> 5) + (j & 1);
    return *reinterpret_cast<const u32x4*>(ring + rd_slot + opq(wave_off) + ln * 128 + 16 * (c ^ (ln & 7)));
  };
  auto advance = [&](int n) {
    rd_slot += n * TL_SLAB;
    rd_slot = rd_slot >= RING ? rd_slot - RING : rd_slot;
  };

  constexpr int PF = TL_PF4;
  u32x4 a[PF];
  // consume a part of NF fragments (whole slabs) starting at tile slab G0 (compile-time), or, with
  // G0 < 0, the loop part at block offset P of the iteration whose issue base is mloop
  auto run = [&](auto nf_tag, auto g0_tag, auto p_tag, int mloop, auto&& mma, auto stop_tag) {
    constexpr int NF = decltype(nf_tag)::value;
    constexpr int G0 = decltype(g0_tag)::value;
    constexpr int P = decltype(p_tag)::value;
    constexpr bool STOP = decltype(stop_tag)::value;
    static_assert(NF % 16 == 0, "parts are whole slabs");
    tl_unroll([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      const u32x4 cur = a[f % PF];
      if constexpr ((f & 15) == 16 - PF) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (G0 >= 0) {
          wait_bar(vm_of(std::integral_constant<int, G0 + (f >> 4) + 1>{}));
          issue_ct(std::integral_constant<int, G0 + (f >> 4) + 1 + AHEAD>{});
        } else {
          wait_bar(VMc{});
          issue_loop(std::integral_constant<int, P + (f >> 4) + 1>{}, mloop);
        }
      }
      mma(fc, cur);
      constexpr int qn = f + PF;
      if constexpr (!STOP || qn < NF)
        a[f % PF] = rdA(std::integral_constant<int, (qn >> 4)>{}, std::integral_constant<int, (qn & 15)>{});
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }, std::make_integer_sequence<int, NF>{});
    advance(NF / 16);
  };
  auto prime = [&]() {
    tl_unroll([&](auto ic) { a[decltype(ic)::value] = rdA(std::integral_constant<int, 0>{}, ic); },
              std::make_integer_sequence<int, PF>{});
  };
  using I0 = std::integral_constant<int, 0>;

  // table t, tile T: this lane's 16 floats (features 32 T + 16 hh + i)
  auto tab = [&](int t, int T, float (&v)[16]) {
    tl_ld16(opq(tl_lds(reinterpret_cast<const char*>(sv))) + 4 * (t * D + 32 * T) + 64 * (tl_lane() >> 5), v);
  };
  enum { TB_B2 = 4, TB_C1 = 5, TB_G2 = 6, TB_BE2 = 7, TB_G1 = 8, TB_BE1 = 9, TB_BO = 10 };
  const long out_bytes = (long)M * D * 2;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.out, (short)0, (int)(out_bytes < 0x7fffffffL ? out_bytes : 0x7fffffffL), 0x00020000);

  uint32_t st[TP_NSTAMP] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
  for (int t = blockIdx.x; t < ntiles; t += G, tb += (long)G * TB_STEP) {
    auto mark = [&](int i) {
      if constexpr (STAMP) st[i] = (uint32_t)__builtin_amdgcn_s_memtime();
    };
    mark(0);
    // ---- first tile: slab 0 and the stand-ins for the previous tile's epilogue stores
    if (t == (int)blockIdx.x) {
      sync_ct(std::integral_constant<int, 0>{}, VMc{});
      const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, 0, 0x00020000);
#pragma unroll
      for (int i = 0; i < NST; ++i) __builtin_amdgcn_raw_buffer_store_b128(a[0], nrs, 0, 0, 0);   // (dropped)
    }
    mark(1);
    // ---- ao = b_o + att W_o'^T, group by group: A_g (the attention rows' k-steps 4 g .. 4 g + 3 as
    // B fragments), the group's W_o' slabs, then R_g (residual tiles 2 g, 2 g + 1) into rr
    f32x16 ao[NT];
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      float bo[16];
      tab(TB_BO, T, bo);
#pragma unroll
      for (int i = 0; i < 16; ++i) ao[T][i] = bo[i];
    }
    u32x4 rr[2 * NT];
    tl_unroll([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      constexpr int QA = g * GS;
      if constexpr (g > 0) sync_ct(std::integral_constant<int, QA>{}, vm_of(std::integral_constant<int, QA>{}));
      u32x4 xa[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xa[j] = rdOwn(j);
      advance(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // in registers before the slot recycles
      sync_ct(std::integral_constant<int, QA + 1>{}, vm_of(std::integral_constant<int, QA + 1>{}));
      prime();
      run(std::integral_constant<int, 4 * NT>{}, std::integral_constant<int, QA + 1>{}, I0{}, 0,
          [&](auto fc, const u32x4& A) {
            constexpr int f = decltype(fc)::value;
            ao[f % NT] = mfma32(A, xa[f / NT], ao[f % NT]);
          }, std::true_type{});
#pragma unroll
      for (int j = 0; j < 4; ++j) rr[4 * g + j] = rdOwn(j);
      advance(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }, std::make_integer_sequence<int, NA>{});
    mark(2);
    sync_ct(std::integral_constant<int, Q_FFN>{}, vm_of(std::integral_constant<int, Q_FFN>{}));   // the first FFN slab
    mark(3);
    // ---- x1 = LN1(ao + x) -> xr
    u32x4 xr[KS];
    {
      float sum = 0.f, sq = 0.f;
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = ao[T][i] + tl_bf(rr[2 * T + (i >> 3)], i & 7);
          ao[T][i] = v;
          sum += v;
          sq = fmaf(v, v, sq);
        }
#pragma unroll
      for (int T = 0; T < NT; ++T) asm volatile("" : "+a"(ao[T]));
      asm volatile("" ::: "memory");
      sum = tl_xsum32(sum);
      sq = tl_xsum32(sq);
      const float mean = sum * (1.0f / D);
      const float rstd = 1.0f / sqrtf(fmaxf(sq * (1.0f / D) - mean * mean, 0.f) + p.eps);
#pragma unroll
      for (int T = 0; T < NT; ++T) {
        float y[16], g1v[16], be1v[16];
        tab(TB_G1, T, g1v);
        tab(TB_BE1, T, be1v);
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = (ao[T][i] - mean) * rstd * g1v[i] + be1v[i];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          xr[2 * T + h2] = u32x4{tl_pack2(y[8 * h2], y[8 * h2 + 1]), tl_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                                 tl_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tl_pack2(y[8 * h2 + 6], y[8 * h2 + 7])};
      }
    }
    prime();
#pragma unroll
    for (int k = 0; k < KS; ++k) asm volatile("" : "+v"(xr[k]));

    mark(4);
    // ---- FFN (tail_kernel's software pipeline)
    f32x16 acc[NT];
    float st1 = 0.f, st2 = 0.f;
    f32x16 h0[2], h1[2];
    u32x4 hf[4];
    auto epi_pair = [&](const f32x16 (&hc)[2], int m) {
      const int tt = m >> 3, i = 2 * (m & 7);
      float x0 = hc[tt][i], x1 = hc[tt][i + 1];
      x0 = tl_lrelu(x0);
      x1 = tl_lrelu(x1);
      st1 += x0 + x1;
      st2 = fmaf(x0, x0, fmaf(x1, x1, st2));
      hf[2 * tt + (i >> 3)][(i & 7) >> 1] = tl_pack2(x0, x1);
    };
    // G0: the part's first tile slab (compile-time) or < 0 for a loop part at block offset P
    auto phase1 = [&](int k, f32x16 (&hn)[2], const f32x16 (&hc)[2], auto epi_tag, auto g0_tag, auto p_tag,
                      int mloop) {
      constexpr bool EPI = decltype(epi_tag)::value;
      int c = k + (int)((unsigned)opq(rot2) >> 1);
      c = c >= S::NCH ? c - S::NCH : c;
      const uint32_t b1 = opq(tl_lds(reinterpret_cast<const char*>(sv))) + 16 * (tl_lane() >> 5) + 256 * c;
      u32x4 bv[8];
      asm volatile(
          "ds_read_b128 %0, %8 offset:0\n ds_read_b128 %1, %8 offset:32\n ds_read_b128 %2, %8 offset:64\n"
          " ds_read_b128 %3, %8 offset:96\n ds_read_b128 %4, %8 offset:128\n ds_read_b128 %5, %8 offset:160\n"
          " ds_read_b128 %6, %8 offset:192\n ds_read_b128 %7, %8 offset:224\n s_waitcnt lgkmcnt(0)"
          : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3]), "=&v"(bv[4]), "=&v"(bv[5]), "=&v"(bv[6]),
            "=&v"(bv[7])
          : "v"(b1));
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) hn[tt][4 * r + e] = __uint_as_float(bv[4 * tt + r][e]);
      run(std::integral_constant<int, S::FW1>{}, g0_tag, p_tag, mloop, [&](auto fc, const u32x4& A) {
        constexpr int f = decltype(fc)::value;
        hn[f & 1] = mfma32(A, xr[f >> 1], hn[f & 1]);
        constexpr int SP = S::FW1 / 16;
        if constexpr (EPI && f % SP == 0) epi_pair(hc, f / SP);
      }, std::false_type{});
    };
    auto phase2 = [&](auto first_tag, auto stop_tag, auto g0_tag, auto p_tag, int mloop) {
      constexpr bool FIRST = decltype(first_tag)::value;
      run(std::integral_constant<int, S::FW2>{}, g0_tag, p_tag, mloop, [&](auto fc, const u32x4& A) {
        constexpr int f = decltype(fc)::value;
        if constexpr (FIRST && f < NT) acc[f] = mfma32(A, hf[0], f32x16{});
        else acc[f % NT] = mfma32(A, hf[f / NT], acc[f % NT]);
      }, stop_tag);
    };
    using F_ = std::false_type;
    using T_ = std::true_type;
    auto at = [](auto blk) { return std::integral_constant<int, Q_FFN + decltype(blk)::value * H>{}; };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    using B2 = std::integral_constant<int, 2>;
    using B3 = std::integral_constant<int, 3>;
    using B4 = std::integral_constant<int, 4>;
    phase1(0, h0, h1, F_{}, at(B0{}), I0{}, 0);
    phase1(1, h1, h0, T_{}, at(B1{}), I0{}, 0);
    phase2(T_{}, F_{}, at(B2{}), I0{}, 0);
    phase1(2, h0, h1, T_{}, at(B3{}), I0{}, 0);
    phase2(F_{}, F_{}, at(B4{}), I0{}, 0);
    using LP = std::integral_constant<int, -1>;
    int mloop = rot2;
#pragma unroll 1
    for (int it = 0; it < LOOP_IT; ++it, mloop += 4) {
      const int k = 3 + 2 * it;
      phase1(k, h1, h0, T_{}, LP{}, std::integral_constant<int, 0>{}, mloop);
      phase2(F_{}, F_{}, LP{}, std::integral_constant<int, H>{}, mloop);
      phase1(k + 1, h0, h1, T_{}, LP{}, std::integral_constant<int, 2 * H>{}, mloop);
      phase2(F_{}, F_{}, LP{}, std::integral_constant<int, 3 * H>{}, mloop);
    }
    // the remaining iterations, unrolled: compile-time issue targets (they reach W2'(N-1) and
    // the next tile)
    tl_unroll([&](auto ic) {
      constexpr int it = LOOP_IT + decltype(ic)::value;
      constexpr int kb = 5 + 4 * it;                      // its first block
      constexpr int k = 3 + 2 * it;
      phase1(k, h1, h0, T_{}, at(std::integral_constant<int, kb>{}), I0{}, 0);
      phase2(F_{}, F_{}, at(std::integral_constant<int, kb + 1>{}), I0{}, 0);
      phase1(k + 1, h0, h1, T_{}, at(std::integral_constant<int, kb + 2>{}), I0{}, 0);
      phase2(F_{}, F_{}, at(std::integral_constant<int, kb + 3>{}), I0{}, 0);
    }, std::make_integer_sequence<int, NIT - LOOP_IT>{});
    static_assert(5 + 4 * NIT == NB2 - 3, "block schedule");
    phase1(S::NCH - 1, h1, h0, T_{}, at(std::integral_constant<int, NB2 - 3>{}), I0{}, 0);
    phase2(F_{}, F_{}, at(std::integral_constant<int, NB2 - 2>{}), I0{}, 0);
#pragma unroll
    for (int m = 0; m < 16; ++m) epi_pair(h1, m);
    // the last part syncs the next tile's slab 0 and stops reading there
    phase2(F_{}, T_{}, at(std::integral_constant<int, NB2 - 1>{}), I0{}, 0);

    mark(5);
    // ---- epilogue: out = LN2(x1 + lrelu(rstd_f acc - rstd_f mean_f c1 + b2'))
    st1 = tl_xsum32(st1);
    st2 = tl_xsum32(st2);
    const float hm = st1 * (1.0f / (4 * D));
    const float hr = 1.0f / sqrtf(fmaxf(st2 * (1.0f / (4 * D)) - hm * hm, 0.f) + p.eps);
    float sum = 0.f, sq = 0.f;
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      float c1v[16], b2v[16];
      tab(TB_C1, T, c1v);
      tab(TB_B2, T, b2v);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float u = hr * fmaf(-hm, c1v[i], acc[T][i]) + b2v[i];
        u = tl_lrelu(u);
        const float v = u + tl_bf(xr[2 * T + (i >> 3)], i & 7);
        acc[T][i] = v;
        sum += v;
        sq = fmaf(v, v, sq);
      }
    }
#pragma unroll
    for (int T = 0; T < NT; ++T) asm volatile("" : "+a"(acc[T]));
    asm volatile("" ::: "memory");
    sum = tl_xsum32(sum);
    sq = tl_xsum32(sq);
    const float mean = sum * (1.0f / D);
    const float rstd = 1.0f / sqrtf(fmaxf(sq * (1.0f / D) - mean * mean, 0.f) + p.eps);
    const float nmr = -mean * rstd;
    const int row_off = (int)(((long)t * TL_ROWS + wave * 32 + (tl_lane() & 31)) * D + 16 * (tl_lane() >> 5)) * 2;
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      float y[16], g2v[16], be2v[16];
      tab(TB_G2, T, g2v);
      tab(TB_BE2, T, be2v);
#pragma unroll
      for (int i = 0; i < 16; ++i) y[i] = fmaf(fmaf(acc[T][i], rstd, nmr), g2v[i], be2v[i]);
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{tl_pack2(y[8 * h2], y[8 * h2 + 1]), tl_pack2(y[8 * h2 + 2], y[8 * h2 + 3]),
                  tl_pack2(y[8 * h2 + 4], y[8 * h2 + 5]), tl_pack2(y[8 * h2 + 6], y[8 * h2 + 7])},
            ors, row_off + 64 * T + 16 * h2, 0, 0);
    }
    mark(6);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the ring overrun has landed before exit
  if constexpr (STAMP) {
    st[7] = (uint32_t)__builtin_amdgcn_s_memtime();
    uint32_t* o = reinterpret_cast<uint32_t*>(p.stamps) + ((long)blockIdx.x * 4 + wave) * TP_NSTAMP;
#pragma unroll
    for (int i = 0; i < TP_NSTAMP; ++i) o[i] = st[i];
  }
}

// One thread per 16-byte piece (8 bf16) of the stream: slab order = consumption order
// (W_o' fragments, then per 64-unit chunk: W1 then W2').  Fragment lane l = (m = l % 32,
// kh = l / 32) holds A[m][8 kh .. 8 kh + 7].
__global__ void tail_pack_kernel(int D, long n_pieces, const bf16* __restrict__ wo, const bf16* __restrict__ w1,
                                 const bf16* __restrict__ w2g, bf16* __restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pieces) return;
  const int NT = D / 32, KS = D / 16, FW1 = 2 * KS, FW2 = 4 * NT, FPC = FW1 + FW2, FPRE = NT * KS;
  const long F = p / 64;
  const int l = (int)(p % 64), m = l & 31, kh = l >> 5;
  bf16 v[8];
  if (F < FPRE) {
    const int s = (int)(F / NT), T = (int)(F % NT);
    const int n = tail_out_feat(T, m);
    for (int j = 0; j < 8; ++j) v[j] = wo[(long)n * D + tail_in_feat(s, kh, j)];
  } else {
    const long g = F - FPRE;
    const int c = (int)(g / FPC), f = (int)(g % FPC);
    if (f < FW1) {
      const int s = f >> 1, t = f & 1;
      const long hid = (long)c * 64 + 32 * t + m;
      for (int j = 0; j < 8; ++j) v[j] = w1[hid * D + tail_in_feat(s, kh, j)];
    } else {
      const int f2 = f - FW1, s2 = f2 / NT, T = f2 % NT;
      const int n = tail_out_feat(T, m);
      for (int j = 0; j < 8; ++j) v[j] = w2g[(long)n * 4 * D + (long)c * 64 + tail_hid(s2, kh, j)];
    }
  }
  for (int j = 0; j < 8; ++j) out[p * 8 + j] = v[j];
}

// Projection stream: per output chunk c (rows c D .. c D + D - 1 of W [NC D, D]), fragments
// F = s NT + T (k-step s, tile T) like the tail's W_o' part.
__global__ void proj_pack_kernel(int D, long n_pieces, const bf16* __restrict__ w, bf16* __restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pieces) return;
  const int NT = D / 32, KS = D / 16, FPRE = NT * KS;
  const long F = p / 64;
  const int l = (int)(p % 64), m = l & 31, kh = l >> 5;
  const int c = (int)(F / FPRE), f = (int)(F % FPRE);
  const int s = f / NT, T = f % NT;
  const long n = (long)c * D + tail_out_feat(T, m);
  for (int j = 0; j < 8; ++j) out[p * 8 + j] = w[n * D + tail_in_feat(s, kh, j)];
}

template <int D, int NC>
static int launch_proj(const TailArgs& a, hipStream_t s) {
  auto kern = tail_kernel<D, false, TL_PF4, 0, true, NC>;
  constexpr size_t lds = (size_t)TL_NSLOT * TL_SLAB + NC * D * 4;
  static_assert(NC * D * 4 <= TL_VEC_LDS && lds <= 160 * 1024, "LDS budget");
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(a.M, TL_ROWS)), dim3(256), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

static unsigned long long* g_tail_stamps = nullptr;   // snvrag_tail_stamps (diagnostics)
unsigned long long* diag_stamps() { return g_tail_stamps; }

static int cu_count() {
  static int n[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (n[dev] <= 0) {
    int v = 0;
    n[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return n[dev];
}

template <int D>
static int launch_tailp(TailArgs a, hipStream_t s) {
  const long ntiles = cdiv(a.M, TL_ROWS);
  const int grid = (int)std::min<long>(ntiles, cu_count());
  const int64_t dz = options().tail_desync;
  a.desync = ntiles >= 8L * grid ? (dz >= 0 ? (int)dz : 25000 * D / 384 * D / 384) : 0;
  constexpr size_t lds = (size_t)TP_NSLOT * TL_SLAB + 11 * D * 4;   // ring + [vec 8D | g1 | be1 | b_o]
  static_assert(lds <= 160 * 1024, "LDS budget");
  auto kern = tailp_kernel<D>;
  if (options().tail_variant == 7 && g_tail_stamps) {     // phase stamps (tools/tail_micro.py)
    kern = tailp_kernel<D, true>;
    a.stamps = g_tail_stamps;
  }
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

template <int D, bool PRE>
static int launch_tail(TailArgs a, hipStream_t s) {
  const int var = (int)options().tail_variant;
  // the wide-row form (tailw.hip): every weight fragment loaded once per workgroup into the
  // registers of the one wave that uses it
  if constexpr (PRE && D == 384)
    if (var == 0 && options().tail_wide) {
      const long nwg = cdiv(a.M, TL_ROWS);
      const int64_t dz = options().tail_desync;
      // (first-round stagger 10 k cycles: tools/tailw_desync.py, two boxes: 1.409 / 1.403 ms vs
      // 1.454 / 1.399 at tail_kernel's 25 k and 1.444 without; r6: 4 k was 1 % faster alone
      // (tools/tailw_desync_sweep.py) but 0.7 % slower inside the bench step, 1.363 vs 1.353 ms,
      // profiles/r6_tail_desync_bench_ab.txt — 10 k kept)
      const int desync = nwg >= 8 * 256 ? (dz >= 0 ? (int)dz : 10000) : 0;
      return tailw_launch(a.M, a.act, a.resid, a.out, a.ws, a.vec, a.b_o, a.g1, a.be1, a.eps, desync,
                          (int)options().tail_wide >= 2 ? (int)options().tail_wide - 1 : 0, s);
    }
  // the persistent kernel (option tail_persist; measured no faster, see tailp_kernel): 32-bit
  // byte offsets of the in-place rows
  if constexpr (PRE)
    if ((var == 0 || var == 7) && options().tail_persist && (long)a.M * D * 2 < 0x7fffffffL) return launch_tailp<D>(a, s);
  // default: 8 fragments read ahead (r5: 1.530 vs 1.553 ms at PF 4, mean of 5 sessions of
  // tools/tail_micro.py at M = 527 360; variant 1 = PF 4, the r4 default)
  auto kern = var == 1 ? tail_kernel<D, PRE, TL_PF4> : var == 2 ? tail_kernel<D, PRE, TL_PF4, 1>
              : var == 3 ? tail_kernel<D, PRE, TL_PF4, 0, false>
              : var == 5 ? tail_kernel<D, PRE, TL_PF4, 3> : tail_kernel<D, PRE, TL_PF_DEFAULT>;
  if (var == 4 && D == 384 && g_tail_stamps) {           // phase stamps (tools/tail_micro.py)
    kern = tail_kernel<D, PRE, TL_PF4, 2>;
    a.stamps = g_tail_stamps;
  }
  // first-round phase step: only when every CU runs several rounds (the delay is paid once).
  // Default 1/8 of a block's ~200 k cycles at D = 384 (tools/tail_micro.py, M = 527 360:
  // 1.668 ms without, 1.611 / 1.593 / 1.602 ms at 12 k / 25 k / 40 k), scaled with the D^2 work
  const long nwg = cdiv(a.M, TL_ROWS);
  const int64_t dz = options().tail_desync;
  a.desync = nwg >= 8 * 256 ? (dz >= 0 ? (int)dz : 25000 * D / 384 * D / 384) : 0;
  constexpr size_t lds = (size_t)TL_NSLOT * TL_SLAB + 7 * D * 4;     // ring + b1, g1, be1, b_o
  static_assert(7 * D * 4 <= TL_VEC_LDS && lds <= 160 * 1024, "LDS budget");
  SNV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(a.M, TL_ROWS)), dim3(256), lds, s, a);
  SNV_LAUNCH_CHECK();
  return 0;
}

static bool tail_d_ok(int D) { return D == 128 || D == 256 || D == 384; }

static size_t tail_bytes(int D) {
  switch (D) {
    case 128: return (size_t)TailShape<128>::NSLAB * TL_SLAB;
    case 256: return (size_t)TailShape<256>::NSLAB * TL_SLAB;
    case 384: return (size_t)TailShape<384>::NSLAB * TL_SLAB;
    default: return 0;
  }
}

}  // namespace snvrag

using namespace snvrag;

extern "C" size_t snvrag_tail_pack_bytes(int D) { return tail_bytes(D); }

extern "C" int snvrag_tail_stamps(void* buf) {
  g_tail_stamps = (unsigned long long*)buf;
  return 0;
}

extern "C" int snvrag_tail_pack(int D, const void* w_o, const void* w1, const void* w2g, void* out, void* stream) {
  SNV_CHECK_ARG(tail_d_ok(D), "block tail needs D in {128, 256, 384}");
  SNV_CHECK_ARG(w_o && w1 && w2g && out, "null pointer");
  const long pieces = (long)(tail_bytes(D) / 16);
  hipLaunchKernelGGL(tail_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), D, pieces,
                     (const bf16*)w_o, (const bf16*)w1, (const bf16*)w2g, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

static int tail_common(int64_t M, int D, bool pre, const TailArgs& a, void* stream) {
  hipStream_t s = as_stream(stream);
  evlog_begin(s);
  int rc;
  if (pre) {
    switch (D) {
      case 128: rc = launch_tail<128, true>(a, s); break;
      case 256: rc = launch_tail<256, true>(a, s); break;
      default: rc = launch_tail<384, true>(a, s); break;
    }
  } else {
    switch (D) {
      case 128: rc = launch_tail<128, false>(a, s); break;
      case 256: rc = launch_tail<256, false>(a, s); break;
      default: rc = launch_tail<384, false>(a, s); break;
    }
  }
  if (rc) return rc;
  evlog_end(s, EV_BLOCK, 2.0 * M * (double)D * D * (pre ? 9 : 8));
  return 0;
}

extern "C" int snvrag_tail_forward(int64_t M, int D, const void* att, void* x, const void* wstream, const float* b_o,
                                   const float* ln1_g, const float* ln1_b, const float* ffn_vec, float eps,
                                   void* stream) {
  SNV_CHECK_ARG(tail_d_ok(D), "block tail needs D in {128, 256, 384}");
  SNV_CHECK_ARG(att && x && wstream && b_o && ln1_g && ln1_b && ffn_vec, "null pointer");
  SNV_CHECK_ARG(att != x, "att and x must not alias");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)att % 16) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)wstream % 16) == 0 &&
                    ((uintptr_t)ffn_vec % 16) == 0,
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  const TailArgs a{(int)M, (const bf16*)att, (const bf16*)x, (bf16*)x, (const char*)wstream, ffn_vec, b_o, ln1_g,
                   ln1_b, eps, nullptr, 0};
  return tail_common(M, D, true, a, stream);
}

extern "C" int snvrag_tail_ffn_forward(int64_t M, int D, const void* x1, void* out, const void* wstream,
                                       const float* ffn_vec, float eps, void* stream) {
  SNV_CHECK_ARG(tail_d_ok(D), "block tail needs D in {128, 256, 384}");
  SNV_CHECK_ARG(x1 && out && wstream && ffn_vec, "null pointer");
  SNV_CHECK_ARG(x1 != out, "x1 and out must not alias");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)x1 % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)wstream % 16) == 0 &&
                    ((uintptr_t)ffn_vec % 16) == 0,
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  const TailArgs a{(int)M, (const bf16*)x1, nullptr, (bf16*)out, (const char*)wstream, ffn_vec, nullptr, nullptr,
                   nullptr, eps, nullptr, 0};
  return tail_common(M, D, false, a, stream);
}

static size_t proj_bytes(int D, int NC) {
  switch (D) {
    case 128: return (size_t)NC * TailShape<128>::NPRE * TL_SLAB;
    case 256: return (size_t)NC * TailShape<256>::NPRE * TL_SLAB;
    case 384: return (size_t)NC * TailShape<384>::NPRE * TL_SLAB;
    default: return 0;
  }
}

extern "C" size_t snvrag_proj_pack_bytes(int D, int NC) { return proj_bytes(D, NC); }

extern "C" int snvrag_proj_pack(int D, int NC, const void* w, void* out, void* stream) {
  SNV_CHECK_ARG(tail_d_ok(D) && (NC == 1 || NC == 3), "projection needs D in {128, 256, 384}, NC in {1, 3}");
  SNV_CHECK_ARG(w && out, "null pointer");
  const long pieces = (long)(proj_bytes(D, NC) / 16);
  hipLaunchKernelGGL(proj_pack_kernel, dim3((unsigned)cdiv(pieces, 256)), dim3(256), 0, as_stream(stream), D, pieces,
                     (const bf16*)w, (bf16*)out);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int snvrag_proj_forward(int64_t M, int D, int NC, const void* x, const void* wstream, const float* bias,
                                   void* out, void* stream) {
  SNV_CHECK_ARG(tail_d_ok(D) && (NC == 1 || NC == 3), "projection needs D in {128, 256, 384}, NC in {1, 3}");
  SNV_CHECK_ARG(x && wstream && bias && out, "null pointer");
  SNV_CHECK_ARG(x != out, "x and out must not alias");
  SNV_CHECK_ARG(M >= 0 && M < (1L << 31), "bad M");
  SNV_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)wstream % 16) == 0,
                "pointers must be 16-byte aligned");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const TailArgs a{(int)M, (const bf16*)x, nullptr, (bf16*)out, (const char*)wstream, bias, nullptr, nullptr,
                   nullptr, 0.f, nullptr, 0};
  evlog_begin(s);
  int rc;
  if (D == 384 && options().proj_wide && (long)M * NC * D * 2 < 0x7fffffffL) {
    // the wide-row projection (tailw.hip): first-round stagger as the block tail's
    const int64_t dz = options().sg_desync;
    const int desync = cdiv(M, TL_ROWS) >= 8 * 256 ? (dz >= 0 ? (int)dz : 8000) : 0;
    rc = projw_launch((int)M, NC, x, wstream, bias, out, desync, s);
    if (rc) return rc;
    evlog_end(s, EV_GEMM, 2.0 * M * (double)D * D * NC);
    return 0;
  }
  switch (D * 8 + NC) {
    case 128 * 8 + 1: rc = launch_proj<128, 1>(a, s); break;
    case 128 * 8 + 3: rc = launch_proj<128, 3>(a, s); break;
    case 256 * 8 + 1: rc = launch_proj<256, 1>(a, s); break;
    case 256 * 8 + 3: rc = launch_proj<256, 3>(a, s); break;
    case 384 * 8 + 1: rc = launch_proj<384, 1>(a, s); break;
    default: rc = launch_proj<384, 3>(a, s); break;
  }
  if (rc) return rc;
  evlog_end(s, EV_GEMM, 2.0 * M * (double)D * D * NC);
  return 0;
}
