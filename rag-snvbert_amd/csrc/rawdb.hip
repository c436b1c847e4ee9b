// Raw-genotype window index search (reference: build_ref_db_l2.py:15-98 builds one
// faiss.IndexFlatL2 per window over the samples' flattened (window_len, 2) 0/1 genotypes;
// test_faiss_intersect.py:171-181 the IndexBinaryFlat / Hamming twin).  On 0/1 vectors
// the squared L2 distance IS the Hamming distance, so the index is bit-packed (32 genotype
// bits per word, stored word-major [nw][N] so a wave's 64 rows load one coalesced line) and
// the distance of a query to a row is sum_w popcount(q_w ^ r_w) — exact integers.
//
// hamming_lists_kernel: one workgroup per query; each of its 256 threads keeps a sorted
// top-k of (distance, row) keys over the rows tid, tid + 256, ... in LDS (insertion only
// below the thread's current k-th, rare after the first k rows), then writes its list;
// the 256 lists per query go through the shared topk_merge kernel (knn.hip).  Keys use the
// kNN's packing ((d + 2^30) << 32 | row), so ties order by row id like the (D, idx) oracle.
#include "common.h"

namespace snvrag {

constexpr int HL_THREADS = 256;
constexpr int HL_KMAX = 32;

__global__ __launch_bounds__(HL_THREADS) void hamming_lists_kernel(int nq, long N, int nw, int k,
                                                                   const uint32_t* __restrict__ codes_wm,
                                                                   const uint32_t* __restrict__ q,
                                                                   uint64_t* __restrict__ lists) {
  __shared__ uint64_t top[HL_KMAX][HL_THREADS];       // [slot][thread]: conflict-free per thread
  __shared__ uint32_t qs[2048];                       // query words (nw <= 2048: 65536 genotype bits)
  const int qi = blockIdx.x, tid = threadIdx.x;
  for (int w = tid; w < nw; w += HL_THREADS) qs[w] = q[(long)qi * nw + w];
  for (int j = 0; j < k; ++j) top[j][tid] = ~0ull;
  __syncthreads();
  uint64_t kth = ~0ull;
  for (long r = tid; r < N; r += HL_THREADS) {
    int d = 0;
    for (int w = 0; w < nw; ++w) d += __popc(qs[w] ^ codes_wm[(long)w * N + r]);
    const uint64_t key = ((uint64_t)(uint32_t)(d + (1 << 30)) << 32) | (uint64_t)(uint32_t)r;
    if (key < kth) {
      int j = k - 1;
      while (j > 0 && top[j - 1][tid] > key) {         // shift the larger keys down one slot
        top[j][tid] = top[j - 1][tid];
        --j;
      }
      top[j][tid] = key;
      kth = top[k - 1][tid];
    }
  }
  for (int j = 0; j < k; ++j) lists[((long)tid * nq + qi) * k + j] = top[j][tid];
}

}  // namespace snvrag

using namespace snvrag;

extern "C" int snvrag_hamming_lists(int64_t nq, int64_t N, int32_t nw, int k, const uint32_t* codes_wm,
                                    const uint32_t* queries, uint64_t* lists, void* stream) {
  SNV_CHECK_ARG(codes_wm && queries && lists, "null pointer");
  SNV_CHECK_ARG(k >= 1 && k <= HL_KMAX, "k must be in [1, 32]");
  SNV_CHECK_ARG(nw >= 1 && nw <= 2048, "1 .. 2048 words (65536 genotype bits) per row");
  SNV_CHECK_ARG(N >= 0 && N < (1LL << 32), "row index must fit 32 bits");
  if (nq == 0) return 0;
  hipLaunchKernelGGL(hamming_lists_kernel, dim3((unsigned)nq), dim3(HL_THREADS), 0, as_stream(stream), (int)nq,
                     (long)N, nw, k, codes_wm, queries, lists);
  SNV_LAUNCH_CHECK();
  return 0;
}

extern "C" int32_t snvrag_hamming_list_count(void) { return HL_THREADS; }
