// Embedding-space exact-L2 kNN scan — the reference's literal retrieval, as a cross-check of the
// token-resident index (SURVEY §8d "C2 embedding-space mode"): the reference ranks panel
// haplotypes by ||E(q) - E(r)||^2 over the flattened [L * D] embeddings (torch.cdist + topk,
// embedding_rag_dataset.py:390-402; FAISS IndexFlatL2, embedding_rag_infer_dataset.py:176-177).
// With stored squared norms that is qn + rn - 2 q . r, so the scan is one distance GEMM
// dot[q][r] = Q[q] . E[r] over K = L * D — HBM-bound: every panel byte read once per launch
// (N * K * 2 B), the queries (Bq * K * 2 B) re-read from L2.
//
// Index layout in HBM (snvrag_knn_emb_pack, once at index build): 32-row x 64-k TILES, each 4 KiB
// contiguous, tile-major over k then rows: tile (T, b) holds rows 32 T .. + 31, k = 64 b .. + 63,
// ordered [k-step s 4][half kh 2][row m 32][8 k] — so the 16 B a lane (m, kh) needs for k-step s
// of an MFMA A operand sit at byte 1024 s + 16 (m + 32 kh) and every wave load instruction reads
// one contiguous KiB.  (Row-major [N, K] rows put each instruction's 64 lanes on 32 rows 791 KB
// apart, 32 B each: 39-46 % of HBM peak against 55-64 % tiled at the C2 shape, tools/knn_emb_micro.py.)
// Rows past N are zero-padded to a whole tile.
//
// A workgroup owns 4 x 32 RT panel rows (each wave RT 32-row MFMA tiles) and one of `splits`
// slices of K.  Each wave streams its tiles' bf16 values straight into VGPRs as the A operand of
// v_mfma_f32_32x32x16_bf16 (PF batches of 64 k in flight in a register ring).  The queries are the
// B operand, shared by the 4 waves: each batch's query fragments are DMA'd global -> LDS
// (buffer_load ... lds, 1 KiB per wave instruction, already in B-fragment order) into a ring of
// PF + 1 slots with one barrier per batch, so a workgroup fetches QT KiB of queries per k-step
// from L2 instead of 4 QT KiB (one copy per wave: measured 45-50 % of HBM peak vs 59 %).  The
// workgroup writes dot partials [split][Bq][N] (f32) that snvrag_knn_emb_finish sums into
// squared distances.
#include "common.h"

#include <utility>

namespace snvrag {

// f(integral_constant<int, J>) for each J of the sequence, in order
template <int... J, class F>
__device__ __forceinline__ void for_slots(std::integer_sequence<int, J...>, F&& f) {
  (f(std::integral_constant<int, J>{}), ...);
}

template <int RT, int QT, int PF>
__global__ __launch_bounds__(256) void knn_emb_dot_kernel(const bf16* __restrict__ E, long N, long K,
                                                          const bf16* __restrict__ Q, int Bq, int splits,
                                                          float* __restrict__ part) {
  constexpr int S = 4, KB = 16 * S;                 // k per batch
  constexpr int FR = QT * S;                        // query fragments (1 KiB) per batch
  constexpr int SLOT = FR * 1024;
  static_assert(FR % 4 == 0, "fragments split evenly over the 4 waves");
  constexpr int FPW = FR / 4;                       // DMA instructions per wave per batch
  extern __shared__ __attribute__((aligned(16))) char qring[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 31, kh = lane >> 5;
  const long rb = ((long)blockIdx.x * 4 + wave) * 32 * RT;
  const int split = blockIdx.y;
  // 32-bit batch counters: 64-bit compares run on the VALU, and the compiler's temporaries for
  // them landed on a register of an in-flight row load (a write-after-write vmcnt(0) draining the
  // whole load ring every PF + 1 batches)
  const int nb = (int)(K / KB);
  const int b0 = (int)((long)nb * split / splits), b1 = (int)((long)nb * (split + 1) / splits);   // may be empty
  const bf16* er[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    long r = rb + 32 * t + m;
    r = r < N ? r : N - 1;
    er[t] = E + (r >> 5) * 32 * K + 8 * lane;        // this lane's 16 B in k-step 0 of tile (r / 32, 0)
  }
  // fragment f = u S + s of a batch: lane (n, kh) <- Q[32 u + n][k0 + 16 s + 8 kh .. + 7]
  const i32x4 qrs = dma_rsrc(Q, (long)Bq * K * 2);
  int qoff[FPW];
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    const int f = wave * FPW + i, u = f / S, sidx = f % S;
    int q = 32 * u + m;
    q = q < Bq ? q : Bq - 1;
    qoff[i] = (int)(((long)q * K + 16 * sidx + 8 * kh) * 2);
  }
  f32x16 acc[RT][QT];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int u = 0; u < QT; ++u) acc[t][u] = f32x16{};
  u32x4 ev[PF + 1][RT][S];
  auto issue = [&](int b, int slot) {
    const int bb = b < b1 ? b : b1 - 1;             // past the range: re-read the last batch
    const int kbyte = bb * KB * 2;
    const uint32_t dst = lds_addr(qring + slot * SLOT + wave * FPW * 1024);
#pragma unroll
    for (int i = 0; i < FPW; ++i) dma_x4(qrs, dst + i * 1024, qoff[i], kbyte);
#pragma unroll
    for (int s2 = 0; s2 < S; ++s2)
#pragma unroll
      for (int t = 0; t < RT; ++t) ev[slot][t][s2] = *reinterpret_cast<const u32x4*>(er[t] + (long)bb * 32 * KB + 512 * s2);
  };
  if (b0 < b1) {
#pragma unroll
    for (int j = 0; j < PF; ++j) issue(b0 + j, j);
  }
  constexpr int AFTER = RT * S + (PF - 1) * (RT * S + FPW);   // loads issued after a batch's DMA
  static_assert(AFTER <= 63, "vmcnt range");
  auto batch = [&](int b, auto j_tag) __attribute__((always_inline)) {
    constexpr int j = decltype(j_tag)::value;     // ring slot: a compile-time register / LDS index
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AFTER) : "memory");   // my DMA of batch b landed
    __builtin_amdgcn_s_barrier();                                    // everyone's; slot j-1 free
    issue(b + PF, (j + PF) % (PF + 1));
    const char* qs = qring + j * SLOT + lane * 16;
#pragma unroll
    for (int s2 = 0; s2 < S; ++s2) {
      u32x4 qf[QT];
#pragma unroll
      for (int u = 0; u < QT; ++u) qf[u] = *reinterpret_cast<const u32x4*>(qs + (u * S + s2) * 1024);
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int u = 0; u < QT; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ev[j][t][s2]),
                                                              __builtin_bit_cast(bf16x8, qf[u]), acc[t][u], 0, 0, 0);
    }
  };
  // whole ring cycles without conditions (a conditional body made the compiler shuffle the ring
  // registers at the back-edge and drain the loads), then the < PF + 1 remaining batches
  int b = b0;
  for (; b + PF + 1 <= b1; b += PF + 1)
    for_slots(std::make_integer_sequence<int, PF + 1>{}, [&](auto j) { batch(b + j, j); });
  for_slots(std::make_integer_sequence<int, PF + 1>{}, [&](auto j) {
    if (b + j < b1) batch(b + j, j);
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the overrun DMAs have landed before exit
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      const int q = 32 * u + m;
      if (q >= Bq) continue;
      float* dst = part + ((long)split * Bq + q) * N;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const long r = rb + 32 * t + 8 * (i >> 2) + 4 * kh + (i & 3);
        if (r < N) dst[r] = acc[t][u][i];
      }
    }
}

// row-major [N, K] -> the tiled layout above; one 16-B unit per thread, coalesced stores
__global__ void knn_emb_pack_kernel(const bf16* __restrict__ E, long N, long K, bf16* __restrict__ Et, long units) {
  const long u = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= units) return;
  const int lane = (int)(u & 63), s = (int)((u >> 6) & 3);
  const long tb = u >> 8;                          // (tile, batch) = 4 KiB blocks
  const long nbk = K / 64, tile = tb / nbk, b = tb % nbk;
  const long row = tile * 32 + (lane & 31);
  const long k = b * 64 + 16 * s + 8 * (lane >> 5);
  u32x4 v = {0u, 0u, 0u, 0u};
  if (row < N) v = *reinterpret_cast<const u32x4*>(E + row * K + k);
  *reinterpret_cast<u32x4*>(Et + u * 8) = v;
}

__global__ void knn_emb_finish_kernel(const float* __restrict__ part, int splits, int Bq, long N,
                                      const float* __restrict__ qn, const float* __restrict__ rn,
                                      float* __restrict__ dist) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Bq * N) return;
  float d = 0.f;
  for (int s = 0; s < splits; ++s) d += part[(long)s * Bq * N + i];
  const int q = (int)(i / N);
  const long r = i % N;
  dist[i] = qn[q] + rn[r] - 2.f * d;
}

}  // namespace snvrag

using namespace snvrag;

constexpr int KE_RT = 2, KE_PF = 2, KE_KB = 64;   // rows tiles per wave, batches in flight, k per batch

extern "C" size_t snvrag_knn_emb_packed_bytes(int64_t N, int64_t K) {
  return (size_t)((N + 31) / 32) * 32 * (size_t)K * 2;
}

extern "C" int snvrag_knn_emb_pack(const void* E, int64_t N, int64_t K, void* Et, void* stream) {
  SNV_CHECK_ARG(E && Et, "null pointer");
  SNV_CHECK_ARG(N > 0 && K > 0 && K % KE_KB == 0, "K must be a positive multiple of 64");
  SNV_CHECK_ARG(((uintptr_t)E % 16) == 0 && ((uintptr_t)Et % 16) == 0, "pointers must be 16-byte aligned");
  const long units = (long)snvrag_knn_emb_packed_bytes(N, K) / 16;
  hipLaunchKernelGGL(knn_emb_pack_kernel, dim3((unsigned)cdiv(units, 256)), dim3(256), 0, as_stream(stream),
                     (const bf16*)E, (long)N, (long)K, (bf16*)Et, units);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t snvrag_knn_emb_ws_bytes(int64_t N, int Bq, int splits) {
  return (size_t)splits * Bq * N * 4;
}


extern "C" int snvrag_knn_emb_splits(int64_t N, int64_t K, int Bq) {
  // ~1280 workgroups (measured best at the C2 shape: 59 % of HBM peak at Bq 48 vs 51-56 % at
  // 16/24/48/64 splits), each keeping >= 32 batches of K; more splits add partial-sum traffic
  // (splits * Bq * N * 4 B written and re-read)
  (void)Bq;
  const int64_t rows = 4 * 32 * KE_RT;
  const int64_t blocks = (N + rows - 1) / rows;
  const int64_t nb = K / KE_KB;
  int s = 1;
  while (s < 256 && blocks * s < 1280 && nb / (s + 1) >= 32) ++s;
  return s;
}

extern "C" int snvrag_knn_emb_scan(const void* E, int64_t N, int64_t K, const void* Q, int Bq, int splits, float* ws,
                                   void* stream) {
  SNV_CHECK_ARG(E && Q && ws, "null pointer");
  SNV_CHECK_ARG(N > 0 && K > 0 && K % KE_KB == 0, "K must be a positive multiple of 64");
  SNV_CHECK_ARG(Bq > 0 && Bq <= 128 && splits >= 1 && splits <= 256, "Bq in [1, 128], splits in [1, 256]");
  SNV_CHECK_ARG(((uintptr_t)E % 16) == 0 && ((uintptr_t)Q % 16) == 0, "pointers must be 16-byte aligned");
  SNV_CHECK_ARG((long)Bq * K * 2 < (1L << 31), "query block must stay below 2 GiB (32-bit buffer offsets)");
  hipStream_t s = as_stream(stream);
  const int qt = (Bq + 31) / 32;
  const dim3 grid((unsigned)cdiv(N, 4 * 32 * KE_RT), (unsigned)splits);
  const size_t lds = (size_t)(KE_PF + 1) * qt * 4 * 1024;
  evlog_begin(s);
  switch (qt) {
#define KE_CASE(T)                                                                                         \
  case T:                                                                                                  \
    SNV_HIP(hipFuncSetAttribute((const void*)knn_emb_dot_kernel<KE_RT, T, KE_PF>,                         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                    \
    hipLaunchKernelGGL((knn_emb_dot_kernel<KE_RT, T, KE_PF>), grid, dim3(256), lds, s, (const bf16*)E,      \
                       (long)N, (long)K, (const bf16*)Q, Bq, splits, ws);                                  \
    break;
    KE_CASE(1)
    KE_CASE(2)
    KE_CASE(3)
    KE_CASE(4)
#undef KE_CASE
  }
  SNV_LAUNCH_CHECK();
  evlog_end(s, EV_KNN_SCAN, (double)N * K * 2 + (double)Bq * K * 2);
  return 0;
}

extern "C" int snvrag_knn_emb_finish(const float* ws, int splits, int Bq, int64_t N, const float* qn, const float* rn,
                                     float* dist, void* stream) {
  SNV_CHECK_ARG(ws && qn && rn && dist && splits >= 1 && Bq > 0 && N > 0, "bad arguments");
  const long n = (long)Bq * N;
  hipLaunchKernelGGL(knn_emb_finish_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream), ws, splits,
                     Bq, (long)N, qn, rn, dist);
  SNV_LAUNCH_CHECK();
  return 0;
}
