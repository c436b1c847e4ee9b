// Weight gradient of a Linear layer on 32x32x16 bf16 MFMAs (gfx950), f32 result:
//
//   dW[N, K] = sum_m dY[m, n] X[m, k]        (optionally db[N] = sum_m dY[m, n])
//
// the backward of every nn.Linear of the training graph (multi_head_attention.py:44-51,
// feed_forward.py:18-21, fusion.py, foundation_model.py; pretrain_with_val_optimized.py:235
// backward).  The reduction runs over the M = 2 B L token rows (~5e4 at B = 24), the output is
// small (<= 1536 x 1536), so the launch splits M into S chunks (enough workgroups to fill 256
// CUs) and every chunk's 128 x 128 tile is added into the f32 output with no-return float atomics
// (one add per element per chunk: <= 17 M adds per layer, well inside the chip's atomic rate).
//
// Both operands are K-major for the MFMA (the reduction index m is the ROW of dY and X), so a
// 32-row stage of each is staged row-major in LDS and read back TRANSPOSED with
// ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3; lane i
// receives column i of the 4 rows): two such reads are one 8-k MFMA fragment, A[n][m] = dY[m][n]
// and B[m][k] = X[m][k].  Rows are 256 B; the 32-B column blocks are XOR-swizzled by (row & 7)
// so the four rows of a transposed read fall in different banks.
#include "common.h"

#include <cstdlib>

namespace snvrag {

constexpr int DW_T = 128;                 // output tile (n and k)
constexpr int DW_R = 32;                  // m rows per stage
constexpr int DW_STAGE = 2 * DW_R * DW_T * 2;   // dY tile + X tile, bf16

__device__ __forceinline__ int dw_swz(int row, int colbyte) {   // byte offset in a [32][256 B] tile
  return row * 256 + ((((colbyte >> 5) ^ (row & 7))) << 5) + (colbyte & 31);
}

__device__ __forceinline__ bf16x4 dw_tr(const char* p) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  return __builtin_bit_cast(bf16x4, v);
}

// grid: (N / 128) (K / 128) S blocks (tile, chunk: see the kernel); 256 threads = 4 waves,
// wave (wn, wk) owns the 64 x 64 sub-tile
// n0 + 64 wn, k0 + 64 wk (2 x 2 MFMA tiles of 32 x 32).
// Output of the launch: dW rows (and db entries) n live in part n / seg of up to 4 separately
// allocated buffers (the q/k/v weights of one fused N = 3D output), each [seg, K] / [seg].
struct DwOut {
  float* w[4];
  float* b[4];
  int seg;
};

// dw_dma_kernel: the 32-row stages brought in by LDS-DMA (buffer_load ... lds, 1 KiB = 4 rows of
// one operand per wave instruction) through a 4-slot ring, 3 stages in flight, one barrier per
// stage (r3: replaced a register-staged kernel that moved every operand byte through VGPRs and a
// ds_write_b128 with one stage of look-ahead).  The XOR swizzle of dw_swz is applied to the SOURCE column of each
// lane (the LDS side of a DMA piece is contiguous) and rows past the chunk read the buffer's zeros.
constexpr int DWD_NS = 4;

__global__ __launch_bounds__(256) void dw_dma_kernel(int M, int N, int K, const bf16* __restrict__ dy, long ldy,
                                                     const bf16* __restrict__ x, long ldx, DwOut out, int chunk,
                                                     int xcd_map) {
  // one __shared__ object per ring slot, filled by the inline-asm DMA (dma_x4): the compiler's
  // waitcnt pass does not track LDS-DMA across the loop back-edge (with the builtin it still put a
  // vmcnt(0) before the first slot's reads of every ring cycle, draining the ring once per cycle);
  // the counted vmcnt waits below are the only ones
  __shared__ __attribute__((aligned(16))) char sl0[DW_STAGE], sl1[DW_STAGE], sl2[DW_STAGE], sl3[DW_STAGE];
  static_assert(DWD_NS == 4, "four slot objects");
  auto slot_ptr = [&](int i) -> char* { return i == 0 ? sl0 : i == 1 ? sl1 : i == 2 ? sl2 : sl3; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  // 1-D grid of tiles x chunks.  Blocks b and b + 8 share an XCD (round-robin dealing,
  // MI355X_MICROARCH.md "Workgroup dispatch"): with xcd_map the work items (chunk-major, tiles
  // inner) are cut into 8 contiguous ranges, one per XCD, so all tiles of an M chunk run on one
  // XCD and read its rows from HBM once (L2 serves the other tiles); in plain order the tiles of
  // a chunk are spread over all 8 XCDs and each XCD fetches the chunk's rows again.
  const int nx = N / DW_T, ntile = nx * (K / DW_T);
  int w = blockIdx.x;
  if (xcd_map) {
    const int xcd = blockIdx.x & 7, per = gridDim.x >> 3, rem = gridDim.x & 7;
    w = xcd * per + min(xcd, rem) + (blockIdx.x >> 3);
  }
  const int tile = w % ntile, zc = w / ntile;
  const int n0 = (tile % nx) * DW_T, k0 = (tile / nx) * DW_T;
  const int part = n0 / out.seg;
  const int nbase = part * out.seg;
  float* __restrict__ dw = out.w[part];
  float* __restrict__ db = out.b[part];
  const int m_begin = zc * chunk;
  const int m_end = min(M, m_begin + chunk);
  if (m_begin >= m_end) return;                      // whole workgroup, before any barrier
  const int nst = (m_end - m_begin + DW_R - 1) / DW_R;

  // sources: this chunk's rows only (the resource ends at m_end: later rows read zeros)
  const long rows = m_end - m_begin;
  const long by = (rows - 1) * ldy * 2 + (long)DW_T * 2, bx = (rows - 1) * ldx * 2 + (long)DW_T * 2;
  const i32x4 ry = dma_rsrc(dy + (long)m_begin * ldy + n0, by);
  const i32x4 rx = dma_rsrc(x + (long)m_begin * ldx + k0, bx);
  // piece j (0..7) of an operand = rows 4 j .. 4 j + 3; wave w issues pieces 2 w, 2 w + 1 of dY and
  // of X.  Lane l lands at byte 16 l of the piece: row 4 j + l / 16, 16-B unit u = l % 16 of the
  // 256-B row, i.e. 32-B block u / 2 which dw_swz fills from column block (u / 2) ^ (row & 7)
  int voy[2], vox[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = 2 * wave + i, row = 4 * j + (lane >> 4), u = lane & 15;
    const int cb = (((u >> 1) ^ (row & 7)) << 5) + ((u & 1) << 4);     // source byte within the row
    voy[i] = (int)(row * ldy * 2) + cb;
    vox[i] = (int)(row * ldx * 2) + cb;
  }
  const int sty = (int)(DW_R * ldy * 2), stx = (int)(DW_R * ldx * 2);
  auto issue = [&](int st, int slot) __attribute__((always_inline)) {
    const uint32_t s = lds_addr(slot_ptr(slot));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 2 * wave + i;
      dma_x4(ry, s + j * 1024, voy[i], st * sty);
      dma_x4(rx, s + DW_R * 256 + j * 1024, vox[i], st * stx);
    }
  };
  auto wait = [&](int y) {                           // 4 DMA per stage per wave
    if (y >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (y == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int rowb = 8 * (g >> 1) + q;
  const int colb = 2 * (16 * (g & 1) + 4 * p);
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  const bool do_db = db != nullptr && k0 == 0 && wk == 0;
  float dbs[2] = {0.f, 0.f};
  auto compute = [&](const char* s) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r0 = 16 * ks + rowb;
        const int ca = 128 * wn + 64 * t + colb;
        const int cb = 128 * wk + 64 * t + colb;
        const bf16x4 a0 = dw_tr(s + dw_swz(r0, ca)), a1 = dw_tr(s + dw_swz(r0 + 4, ca));
        const bf16x4 b0 = dw_tr(s + DW_R * 256 + dw_swz(r0, cb)), b1 = dw_tr(s + DW_R * 256 + dw_swz(r0 + 4, cb));
        fa[t] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
        fb[t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
      if (do_db) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int j = 0; j < 8; ++j) dbs[a] += (float)fa[a][j];
      }
    }
  };
#pragma unroll
  for (int j = 0; j < DWD_NS - 1; ++j)
    if (j < nst) issue(j, j);
  int st = 0;
  for (; st + DWD_NS <= nst; st += DWD_NS) {
#pragma unroll
    for (int u = 0; u < DWD_NS; ++u) {
      wait(min(DWD_NS - 2, nst - 1 - (st + u)));
      __builtin_amdgcn_s_barrier();
      if (st + u + DWD_NS - 1 < nst) issue(st + u + DWD_NS - 1, (u + DWD_NS - 1) % DWD_NS);
      compute(slot_ptr(u));
    }
  }
  for (; st < nst; ++st) {
    wait(min(DWD_NS - 2, nst - 1 - st));
    __builtin_amdgcn_s_barrier();
    if (st + DWD_NS - 1 < nst) issue(st + DWD_NS - 1, (st + DWD_NS - 1) % DWD_NS);
    switch (st % DWD_NS) {                           // compile-time slot objects
      case 0: compute(sl0); break;
      case 1: compute(sl1); break;
      case 2: compute(sl2); break;
      default: compute(sl3); break;
    }
  }

#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int kk = k0 + 64 * wk + 32 * b + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int nn = n0 + 64 * wn + 32 * a + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
        unsafeAtomicAdd(dw + (long)(nn - nbase) * K + kk, acc[a][b][e]);
      }
    }
  if (do_db) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const float v = dbs[a] + __shfl_xor(dbs[a], 32, 64);
      if (lane < 32) unsafeAtomicAdd(db + (n0 - nbase) + 64 * wn + 32 * a + lane, v);
    }
  }
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_dw_splits(int64_t M, int64_t N, int64_t K) {
  // Every split adds one f32 partial per output element (no-return atomics): the atomic volume
  // is splits x N x K, comparable to the MFMA time at these shapes, so the split count targets
  // ~2 workgroups per CU (~1 when there are few output tiles), not a full 4-deep occupancy.
  // Measured at M = 49 440 (tools/dw_micro.py): 1536 x 384 104.8 us at 14 splits vs 132.2 at 29,
  // 384 x 384 48.7 us at 28 vs 73.0 at 114; 15 splits of 36 tiles (540 > 512 workgroups) 120.1 us.
  const long tiles = (N / DW_T) * (K / DW_T);
  const long target = tiles >= 16 ? 512 : 256;
  long s = target / std::max<long>(tiles, 1);                         // whole rounds: <= target workgroups
  const long max_s = (M + 8 * DW_R - 1) / (8 * DW_R);                // >= 8 stages per chunk
  s = std::min(std::max(s, 1L), std::max(max_s, 1L));
  return (int)s;
}

static int launch_dw(int64_t M, int64_t N, int64_t K, const void* dy, int64_t ldy, const void* x, int64_t ldx,
                     const DwOut& out, int splits, hipStream_t s) {
  if (M == 0) return 0;
  if (splits <= 0) splits = snvrag_dw_splits(M, N, K);
  const int chunk = (int)((((M + splits - 1) / splits) + DW_R - 1) / DW_R * DW_R);
  const int S = (int)((M + chunk - 1) / chunk);
  evlog_begin(s);
  hipLaunchKernelGGL(dw_dma_kernel, dim3((unsigned)((N / DW_T) * (K / DW_T) * S)), dim3(256), 0, s, (int)M, (int)N,
                     (int)K, (const bf16*)dy, (long)ldy, (const bf16*)x, (long)ldx, out, chunk,
                     (int)options().dw_xcd);
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_TRAIN, 2.0 * M * (double)N * K);
  return 0;
}

static int dw_check(int64_t M, int64_t N, int64_t K, const void* dy, int64_t ldy, const void* x, int64_t ldx) {
  SNV_CHECK_ARG(dy && x, "null pointer");
  SNV_CHECK_ARG(M >= 0 && N % DW_T == 0 && K % DW_T == 0 && N > 0 && K > 0, "N and K must be multiples of 128");
  SNV_CHECK_ARG(ldy >= N && ldx >= K && ldy % 8 == 0 && ldx % 8 == 0, "leading dims: >= N / K, multiples of 8");
  SNV_CHECK_ARG(((uintptr_t)dy % 16) == 0 && ((uintptr_t)x % 16) == 0, "operands must be 16-byte aligned");
  return 0;
}

extern "C" int snvrag_linear_dw(int64_t M, int64_t N, int64_t K, const void* dy, int64_t ldy, const void* x,
                                int64_t ldx, float* dw, float* db, int splits, void* stream) {
  if (int rc = dw_check(M, N, K, dy, ldy, x, ldx)) return rc;
  SNV_CHECK_ARG(dw, "null pointer");
  // dw / db are accumulated: the caller zeroes them (or passes a running sum)
  DwOut out{{dw, nullptr, nullptr, nullptr}, {db, nullptr, nullptr, nullptr}, (int)N};
  return launch_dw(M, N, K, dy, ldy, x, ldx, out, splits, as_stream(stream));
}

extern "C" int snvrag_linear_dw_parts(int64_t M, int64_t N, int64_t K, const void* dy, int64_t ldy, const void* x,
                                      int64_t ldx, int n_parts, float* const* dw_parts, float* const* db_parts,
                                      int splits, void* stream) {
  if (int rc = dw_check(M, N, K, dy, ldy, x, ldx)) return rc;
  SNV_CHECK_ARG(n_parts >= 1 && n_parts <= 4 && N % n_parts == 0 && (N / n_parts) % DW_T == 0,
                "1-4 equal parts of N, each a multiple of 128");
  SNV_CHECK_ARG(dw_parts, "null pointer");
  DwOut out{{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}, (int)(N / n_parts)};
  for (int i = 0; i < n_parts; ++i) {
    SNV_CHECK_ARG(dw_parts[i], "null dW part");
    out.w[i] = dw_parts[i];
    out.b[i] = db_parts ? db_parts[i] : nullptr;
    SNV_CHECK_ARG(!db_parts || db_parts[i], "null db part");
  }
  return launch_dw(M, N, K, dy, ldy, x, ldx, out, splits, as_stream(stream));
}
