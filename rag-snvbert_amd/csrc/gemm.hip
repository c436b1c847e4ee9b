// Dense layer  C = act(A W^T + bias + rank-1 terms) + resid   on gfx950 MFMA.
//
// Replaces every nn.Linear of the v18 model (see include/snvrag.h, snvrag_linear).
// Tile 128x128, 256 threads = 4 waves in a 2x2 grid, each wave 64x64 = 4x4
// MFMA 16x16 tiles.  One K-tile = 128 bytes of K per row (64 bf16 / 32 f32)
// staged global -> registers -> LDS (double buffered, one barrier per K-tile)
// with the st_16x32-style XOR swizzle `chunk ^ (row & 7)` so the 16-lane
// ds_read_b128 groups of the fragment reads are conflict-free.
//   bf16: v_mfma_f32_16x16x32_bf16 (one 16-B fragment = one MFMA K-step)
//   f32 : v_mfma_f32_16x16x4_f32  (exact f32; one 16-B fragment = 4 K-steps)
// Epilogue: accumulators -> LDS (f32, padded rows) -> coalesced 16-B output
// chunks with bias / rank-1 / activation / residual fused.
// Block -> tile mapping is XCD-aware: blocks that share an A row-panel are
// consecutive after the bijective remap, i.e. dispatched to the same XCD (L2).
#include "common.h"

namespace snvrag {

constexpr int GT_M = 128, GT_N = 128, G_ROWB = 128;        // tile rows, row bytes per K-tile
constexpr int G_TILE_BYTES = GT_M * G_ROWB;                 // 16 KB per operand tile
constexpr int G_STAGE_LD = 68;                              // f32 staging row stride (floats)
constexpr int G_SMEM = 4 * 64 * G_STAGE_LD * 4;             // 69,632 B >= 2 * 2 * 16 KB

struct EpiDev {
  const float* bias;
  const float* row1; long row1_stride; const float* col1;
  const float* row2; long row2_stride; const float* col2;
  long row_period;
  int act; float slope;
  const void* resid; long ld_resid;
};

__device__ __forceinline__ int swz(int row, int chunk) {      // byte offset inside a tile
  return row * G_ROWB + ((chunk ^ (row & 7)) << 4);
}

template <typename TI>
__device__ __forceinline__ void load_tile_regs(const TI* __restrict__ P, long ld, int rows_valid,
                                               int k0, int K, int tid, u32x4 (&r)[4]) {
  constexpr int EPC = 16 / sizeof(TI);                      // elements per 16-B chunk
  const int c = tid & 7;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    const int k = k0 + c * EPC;
    if (row < rows_valid && k < K) {
      r[i] = *reinterpret_cast<const u32x4*>(P + (long)row * ld + k);
    } else {
      r[i] = u32x4{0u, 0u, 0u, 0u};
    }
  }
}

__device__ __forceinline__ void store_tile_lds(char* tile, int tid, const u32x4 (&r)[4]) {
  const int c = tid & 7;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    *reinterpret_cast<u32x4*>(tile + swz(row, c)) = r[i];
  }
}

template <typename TI>
__device__ __forceinline__ void mma_tile(const char* At, const char* Bt, int wm, int wn, int lane,
                                         f32x4 (&acc)[4][4]) {
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int kc = 0; kc < 2; ++kc) {
    u32x4 a[4], b[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ra = wm + 16 * t + lr, rb = wn + 16 * t + lr;
      a[t] = *reinterpret_cast<const u32x4*>(At + swz(ra, 4 * kc + lg));
      b[t] = *reinterpret_cast<const u32x4*>(Bt + swz(rb, 4 * kc + lg));
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        if constexpr (sizeof(TI) == 2) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, a[mt]), __builtin_bit_cast(bf16x8, b[nt]), acc[mt][nt], 0, 0, 0);
        } else {
          const f32x4 av = __builtin_bit_cast(f32x4, a[mt]);
          const f32x4 bv = __builtin_bit_cast(f32x4, b[nt]);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc[mt][nt], 0, 0, 0);
        }
      }
    }
  }
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void linear_kernel(int M, int N, int K, const TI* __restrict__ A,
                                                     long lda, const TI* __restrict__ W, long ldw,
                                                     TO* __restrict__ C, long ldc, EpiDev epi,
                                                     int n_tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[G_SMEM];
  constexpr int EPT = G_ROWB / sizeof(TI);                  // K elements per K-tile

  // XCD-aware bijective remap of the 1-D grid (guide §5 "XCD swizzle must be bijective")
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tm = wg / n_tiles_n, tn = wg % n_tiles_n;
  const int m0 = tm * GT_M, n0 = tn * GT_N;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const TI* Ab = A + (long)m0 * lda;
  const TI* Wb = W + (long)n0 * ldw;
  const int mrows = min(GT_M, M - m0), nrows = min(GT_N, N - n0);
  const int nk = (K + EPT - 1) / EPT;

  u32x4 ra[4], rb[4];
  load_tile_regs<TI>(Ab, lda, mrows, 0, K, tid, ra);
  load_tile_regs<TI>(Wb, ldw, nrows, 0, K, tid, rb);
  store_tile_lds(smem, tid, ra);
  store_tile_lds(smem + G_TILE_BYTES, tid, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    char* At = smem + cur * 2 * G_TILE_BYTES;
    char* Bt = At + G_TILE_BYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile_regs<TI>(Ab, lda, mrows, (kt + 1) * EPT, K, tid, ra);
      load_tile_regs<TI>(Wb, ldw, nrows, (kt + 1) * EPT, K, tid, rb);
    }
    mma_tile<TI>(At, Bt, wm, wn, lane, acc);
    if (more) {
      char* An = smem + (cur ^ 1) * 2 * G_TILE_BYTES;
      store_tile_lds(An, tid, ra);
      store_tile_lds(An + G_TILE_BYTES, tid, rb);
    }
    __syncthreads();
  }

  // ---- epilogue: stage f32 accumulators per wave, then coalesced 16-B output chunks ----
  float* stage = reinterpret_cast<float*>(smem) + wave * 64 * G_STAGE_LD;
  {
    const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          stage[(16 * mt + 4 * lg + i) * G_STAGE_LD + 16 * nt + lr] = acc[mt][nt][i];
  }
  __syncthreads();

  constexpr int OPC = 16 / sizeof(TO);                      // outputs per 16-B chunk
  constexpr int CPR = 64 / OPC;                             // chunks per wave row
  for (int id = lane; id < 64 * CPR; id += 64) {
    const int rr = id / CPR, cc = (id % CPR) * OPC;
    const int m = m0 + wm + rr, n = n0 + wn + cc;
    if (m >= M || n >= N) continue;
    float v[OPC];
#pragma unroll
    for (int j = 0; j < OPC; ++j) v[j] = stage[rr * G_STAGE_LD + cc + j];
    const long mr = epi.row_period > 0 ? (m % epi.row_period) : m;
    const float r1 = epi.row1 ? epi.row1[mr * epi.row1_stride] : 0.f;
    const float r2 = epi.row2 ? epi.row2[mr * epi.row2_stride] : 0.f;
#pragma unroll
    for (int j = 0; j < OPC; ++j) {
      float x = v[j];
      if (epi.bias) x += epi.bias[n + j];
      if (epi.row1) x += r1 * epi.col1[n + j];
      if (epi.row2) x += r2 * epi.col2[n + j];
      v[j] = apply_act(epi.act, x, epi.slope);
    }
    if (epi.resid) {
      const TO* R = reinterpret_cast<const TO*>(epi.resid) + (long)m * epi.ld_resid + n;
#pragma unroll
      for (int j = 0; j < OPC; ++j) v[j] += to_f32(R[j]);
    }
    TO o[OPC];
#pragma unroll
    for (int j = 0; j < OPC; ++j) o[j] = from_f32<TO>(v[j]);
    *reinterpret_cast<u32x4*>(C + (long)m * ldc + n) = *reinterpret_cast<u32x4*>(o);
  }
}

template <typename TI, typename TO>
static int launch_linear(long M, long N, long K, const void* A, long lda, const void* W, long ldw,
                         void* C, long ldc, const EpiDev& e, hipStream_t s) {
  const int tn = cdiv(N, GT_N), tm = cdiv(M, GT_M);
  const long nb = (long)tn * tm;
  SNV_CHECK_ARG(nb < (1L << 31), "grid too large");
  evlog_begin(s);
  hipLaunchKernelGGL((linear_kernel<TI, TO>), dim3((unsigned)nb), dim3(256), 0, s, (int)M, (int)N,
                     (int)K, (const TI*)A, lda, (const TI*)W, ldw, (TO*)C, ldc, e, tn);
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_GEMM, 2.0 * M * N * K);
  return 0;
}

int rows_linear(int din, int dout, long M, long N, long K, const void* A, long lda, const void* W, long ldw,
                void* C, long ldc, const snvrag_epilogue_t* epi, const snvrag_rownorm_t* anorm, hipStream_t s);

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_linear(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K,
                             const void* A, int64_t lda, const void* W, int64_t ldw, void* C,
                             int64_t ldc, const snvrag_epilogue_t* epi, void* stream) {
  return snvrag_linear_ex(dtype_in, dtype_out, M, N, K, A, lda, W, ldw, C, ldc, epi, nullptr, stream);
}

extern "C" int snvrag_linear_ex(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K,
                                const void* A, int64_t lda, const void* W, int64_t ldw, void* C,
                                int64_t ldc, const snvrag_epilogue_t* epi, const snvrag_rownorm_t* anorm,
                                void* stream) {
  SNV_CHECK_ARG(M >= 0 && N > 0 && K > 0, "bad shape");
  SNV_CHECK_ARG(A && W && C, "null pointer");
  SNV_CHECK_ARG(dtype_in == SNVRAG_F32 || dtype_in == SNVRAG_BF16, "dtype_in");
  SNV_CHECK_ARG(dtype_out == SNVRAG_F32 || dtype_out == SNVRAG_BF16, "dtype_out");
  const int ein = dtype_in == SNVRAG_BF16 ? 8 : 4, eout = dtype_out == SNVRAG_BF16 ? 8 : 4;
  SNV_CHECK_ARG(K % 8 == 0, "K must be a multiple of 8");
  SNV_CHECK_ARG(lda % ein == 0 && ldw % ein == 0, "lda/ldw must keep 16-byte row alignment");
  SNV_CHECK_ARG(N % eout == 0 && ldc % eout == 0, "N/ldc must keep 16-byte output chunks");
  SNV_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)C % 16) == 0,
                "A/W/C must be 16-byte aligned");
  if (M == 0) return 0;
  const int ept = dtype_in == SNVRAG_BF16 ? 64 : 32;
  const bool fused = anorm || (epi && (epi->ln_g || epi->stats_out));
  const bool rows_ok = N % 64 == 0 && K % ept == 0 && !options().gemm_tile128;
  if (fused || rows_ok) {               // row-panel GEMM (checks its own shape constraints)
    hipStream_t s = as_stream(stream);
    evlog_begin(s);
    const int rc = rows_linear(dtype_in, dtype_out, M, N, K, A, lda, W, ldw, C, ldc, epi, anorm, s);
    if (rc) return rc;
    evlog_end(s, EV_GEMM, 2.0 * M * N * K);
    return 0;
  }
  EpiDev e{};
  if (epi) {
    e.bias = epi->bias; e.row1 = epi->row1; e.row1_stride = epi->row1_stride; e.col1 = epi->col1;
    e.row2 = epi->row2; e.row2_stride = epi->row2_stride; e.col2 = epi->col2;
    e.row_period = epi->row_period; e.act = epi->act; e.slope = epi->slope;
    e.resid = epi->resid; e.ld_resid = epi->ld_resid;
    SNV_CHECK_ARG(!e.row1 || e.col1, "row1 without col1");
    SNV_CHECK_ARG(!e.row2 || e.col2, "row2 without col2");
    if (e.resid) SNV_CHECK_ARG(e.ld_resid % eout == 0 && ((uintptr_t)e.resid % 16) == 0, "resid alignment");
  }
  hipStream_t s = as_stream(stream);
  if (dtype_in == SNVRAG_BF16 && dtype_out == SNVRAG_BF16)
    return launch_linear<bf16, bf16>(M, N, K, A, lda, W, ldw, C, ldc, e, s);
  if (dtype_in == SNVRAG_BF16 && dtype_out == SNVRAG_F32)
    return launch_linear<bf16, float>(M, N, K, A, lda, W, ldw, C, ldc, e, s);
  if (dtype_in == SNVRAG_F32 && dtype_out == SNVRAG_F32)
    return launch_linear<float, float>(M, N, K, A, lda, W, ldw, C, ldc, e, s);
  return launch_linear<float, bf16>(M, N, K, A, lda, W, ldw, C, ldc, e, s);
}
