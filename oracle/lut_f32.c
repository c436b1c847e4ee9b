/* ORACLE (test infrastructure, not product code): the token-index LUT Delta_q[s] restated in
 * the device's f32 arithmetic, so the oracle's quantised LUT equals the device's bit for bit.
 *
 * What it restates.  The reference ranks panel haplotypes by the squared L2 distance of the
 * flattened [L*D] embeddings (torch.cdist + topk, src/dataset/embedding_rag_dataset.py:390-402;
 * FAISS IndexFlatL2, src/dataset/embedding_rag_infer_dataset.py:176-177, :279-285).  With the
 * position-wise embedding (src/model/embedding/bert.py:53-75) the per-site term of
 * dist^2(q, r) = C_q + sum_s Delta_q[s] a_r[s] is
 *
 *     Delta_q[s] = || u - Wp[tok1] ||^2 - || u - Wp[tok0] ||^2,   u = W[tok_q,l] (+ A_q,l) (- A_r,l)
 *
 * at token position l = s + 1 (oracle/knn_np.py ``lut_delta`` computes it in float64).  The
 * canonical kNN order of this repo quantises Delta to a per-query power-of-two
 * grid; for that grid to be the same on both sides, this file computes Delta with the same f32
 * operations in the same order as csrc/knn.hip:
 *
 *   no offsets (lut_kernel, the token-table path and its per-position loop):  lane i of a
 *     64-lane wave accumulates d = i, i + 64, ... with fmaf(a, a, acc), a = W[t][d] - Wp[c][d];
 *     the 64 partials are summed by the xor butterfly 32, 16, 8, 4, 2, 1 (wave_sum);
 *   offsets A_q and/or A_r (lut_delta_kernel):  16 lanes per position; lane j accumulates
 *     d = 4j + 64m + e (m outer, e = 0..3 inner) with u = (W + A_q) - A_r in f32, then the
 *     xor butterfly 8, 4, 2, 1 inside the 16 lanes;
 *
 * and Delta = t1 - t0 in f32; masked index sites give 0.  fmaf() is C99's correctly rounded
 * fused multiply-add (built with -ffp-contract=off: no other contraction). */
#include <math.h>
#include <stdint.h>
#include <string.h>

static float butterfly(float* v, int n) {
  float t[64];
  for (int o = n / 2; o >= 1; o >>= 1) {
    for (int i = 0; i < n; ++i) t[i] = v[i] + v[i ^ o];
    memcpy(v, t, sizeof(float) * (size_t)n);
  }
  return v[0];
}

int oracle_lut_delta_f32(int64_t nq, int64_t L, int64_t D, const int64_t* tok, const float* W, const float* Wp,
                         const float* Aq, int64_t aq_period, const float* Ar, const uint8_t* site_mask,
                         int64_t n_sites, int tok0, int tok1, float* delta) {
  if (D % 4 || n_sites + 1 > L) return 1;
  const float* w0 = Wp + (int64_t)tok0 * D;
  const float* w1 = Wp + (int64_t)tok1 * D;
  float p0[64], p1[64];
  for (int64_t q = 0; q < nq; ++q) {
    const int64_t arow = Aq ? ((aq_period > 0 ? q % aq_period : q) * L) : 0;
    for (int64_t s = 0; s < n_sites; ++s) {
      const int64_t l = s + 1;
      float* out = delta + q * n_sites + s;
      if (site_mask[s]) { *out = 0.f; continue; }
      const float* wt = W + tok[q * L + l] * D;
      float t0, t1;
      if (!Aq && !Ar) {
        for (int lane = 0; lane < 64; ++lane) {
          float a0 = 0.f, a1 = 0.f;
          for (int64_t d = lane; d < D; d += 64) {
            const float a = wt[d] - w0[d], b = wt[d] - w1[d];
            a0 = fmaf(a, a, a0);
            a1 = fmaf(b, b, a1);
          }
          p0[lane] = a0;
          p1[lane] = a1;
        }
        t0 = butterfly(p0, 64);
        t1 = butterfly(p1, 64);
      } else {
        for (int j = 0; j < 16; ++j) {
          float a0 = 0.f, a1 = 0.f;
          for (int64_t d = 4 * j; d < D; d += 64)
            for (int e = 0; e < 4; ++e) {
              float u = wt[d + e];
              if (Aq) u = u + Aq[(arow + l) * D + d + e];
              if (Ar) u = u - Ar[l * D + d + e];
              const float a = u - w0[d + e], b = u - w1[d + e];
              a0 = fmaf(a, a, a0);
              a1 = fmaf(b, b, a1);
            }
          p0[j] = a0;
          p1[j] = a1;
        }
        t0 = butterfly(p0, 16);
        t1 = butterfly(p1, 16);
      }
      *out = t1 - t0;
    }
  }
  return 0;
}
