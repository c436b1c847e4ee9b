// Encoder stack orchestration: every launch of the n_layers transformer blocks issued
// from C++ (one C-ABI call per forward, capturable in a hipGraph).  bf16 at D in {128,
// 256, 384}: 3 launches per layer (QKV stream GEMM, attention, block tail); otherwise (f32
// parity path, other D) the row-panel GEMM form below with LN fused into the epilogues
// (SNVRAG_UNFUSED_LN=1: the 8-launch unfused form, test-only).
//
// Per block (model/transformer.py:27-30, sublayer.py:15-16, feed_forward.py:18-21,
// multi_head_attention.py:44-51), eval:
//   qkv = x Wqkv^T + b                      (one GEMM, N = 3D: q;k;v rows packed)
//   a   = attention(qkv)                    (flash, unmasked)
//   x1  = LN1(x + a Wo^T + bo)              (residual fused in the GEMM epilogue)
//   h   = LN_f(lrelu(x1 W1^T + b1))         (LN in place)
//   x   = LN2(x1 + lrelu(h W2^T + b2))      (residual fused after the activation)
// Sequences are processed in chunks so a chunk's activations (9 D per token)
// stay resident in the 256 MiB Infinity Cache across the 12 layers.
#include "common.h"

#include <cmath>

namespace snvrag {

static int64_t chunk_seqs(int64_t nseq, int64_t L, int D, int esz) {
  if (options().encoder_chunk > 0) return std::min<int64_t>(options().encoder_chunk, nseq);
  // The row-panel GEMMs tile M by 128 rows with whole output rows per tile, so a chunk
  // must hold >= ~4 tiles per CU (1024 tiles = 131k rows) to fill 256 CUs; cap the
  // per-chunk workspace (10 D / token) at ~16 GB of the 288 GB HBM; chunks are balanced
  // (a 505 + 7 split would run the 7-sequence chunk at a fraction of the chip).
  const double per_seq = (double)L * D * 10.0 * esz;
  int64_t c = (int64_t)(16.0e9 / per_seq);
  if (c < 1) c = 1;
  if (c >= nseq) return nseq;
  const int64_t nchunks = (nseq + c - 1) / c;
  return (nseq + nchunks - 1) / nchunks;
}

}  // namespace snvrag

using namespace snvrag;

extern "C" size_t snvrag_encoder_ws_bytes(int dtype, int64_t nseq, int64_t L, int D, int heads) {
  (void)heads;
  const int esz = dtype == SNVRAG_BF16 ? 2 : 4;
  const int64_t c = chunk_seqs(nseq, L, D, esz);
  const size_t M = (size_t)c * L;
  return M * (size_t)D * 9 * esz + M * 64 * 8 + 8192;
}

extern "C" int snvrag_encoder_forward(int dtype, int64_t nseq, int64_t L, int D, int heads, int n_layers,
                                      const snvrag_layer_t* layers, void* x, void* ws, size_t ws_bytes,
                                      void* stream) {
  SNV_CHECK_ARG(layers && x && ws, "null pointer");
  SNV_CHECK_ARG(D % heads == 0, "D % heads");
  SNV_CHECK_ARG(ws_bytes >= snvrag_encoder_ws_bytes(dtype, nseq, L, D, heads), "encoder workspace too small");
  const int esz = dtype == SNVRAG_BF16 ? 2 : 4;
  const int64_t cs = chunk_seqs(nseq, L, D, esz);
  const size_t Mc = (size_t)cs * L;
  char* w = (char*)ws;
  auto carve = [&](size_t elems) { char* p = w; w += ((elems * esz + 255) / 256) * 256; return (void*)p; };
  void* qkv = carve(Mc * 3 * D);
  void* att = carve(Mc * D);
  void* x1 = carve(Mc * D);
  void* h = carve(Mc * 4 * D);
  // FFN LayerNorm statistics: [N-tiles of the 4D GEMM][Mc] float2
  const int n_stat_parts = (4 * D) % 384 == 0 ? (4 * D) / 384 : (4 * D) % 256 == 0 ? (4 * D) / 256
                           : (4 * D) % 128 == 0 ? (4 * D) / 128 : (4 * D) / 64;
  w = (char*)(((uintptr_t)w + 255) & ~(uintptr_t)255);
  void* stats = w; w += ((Mc * n_stat_parts * 8 + 255) / 256) * 256;
  const int dh = D / heads;
  const float scale = 1.0f / sqrtf((float)dh);

  const bool fused = (D == 64 || D == 128 || D == 256 || D == 384) && !options().unfused_ln &&
                     layers[0].w2g && layers[0].b2g && layers[0].c2g;
  for (int64_t s0 = 0; s0 < nseq; s0 += cs) {
    const int64_t ns = std::min<int64_t>(cs, nseq - s0);
    const int64_t M = ns * L;
    char* xc = (char*)x + (size_t)s0 * L * D * esz;
    for (int i = 0; i < n_layers; ++i) {
      const snvrag_layer_t& ly = layers[i];
      snvrag_epilogue_t e{};
      int rc;
      e.bias = ly.b_qkv;
      // QKV: the 8-wave stream GEMM (csrc/sgemm.hip); its 32-bit output offsets cap one launch
      // at 2 GiB, beyond that the 32x32 projection stream (csrc/tail.hip PROJ mode)
      // (the wide-row projection, csrc/tailw.hip, measured 0.62-0.70 vs 0.54 ms for the 8-wave stream
      // GEMM at M = 527 360: the stream GEMM stays; tools/proj_micro.py)
      if (dtype == SNVRAG_BF16 && ly.qkv_sg && M * 3 * D * 2 < (1L << 31))
        rc = snvrag_sgemm_forward(M, (int)D, (int)(3 * D), 0, SNVRAG_ACT_NONE, 0.f, xc, ly.qkv_sg, ly.b_qkv, nullptr,
                                  nullptr, 0, 0.f, qkv, nullptr, nullptr, stream);
      else if (dtype == SNVRAG_BF16 && ly.qkv_pw)
        rc = snvrag_proj_forward(M, D, 3, xc, ly.qkv_pw, ly.b_qkv, qkv, stream);
      else
        rc = snvrag_linear(dtype, dtype, M, 3 * D, D, xc, D, ly.w_qkv, D, qkv, 3 * D, &e, stream);
      if (rc) return rc;
      // q rows may carry a folded factor (the bf16 engine folds log2(e)/sqrt(dh))
      const float sc = ly.q_scale > 0.f ? scale / ly.q_scale : scale;
      rc = snvrag_attention(dtype, ns, L, heads, dh, qkv, 3 * D, att, D, sc, stream);
      if (rc) return rc;
      if (fused && dtype == SNVRAG_BF16 && ly.tail_w && ly.ffn_v) {
        // the whole block tail on 32x32 MFMAs (csrc/tail.hip): one launch
        rc = snvrag_tail_forward(M, D, att, xc, ly.tail_w, ly.b_o, ly.ln1_g, ly.ln1_b, ly.ffn_v, 1e-5f, stream);
        if (rc) return rc;
        continue;
      }
      if (fused) {
        // x1 = LN1(x + attn Wo^T + bo)                       (one launch)
        e = snvrag_epilogue_t{};
        e.bias = ly.b_o; e.resid = xc; e.ld_resid = D; e.ln_g = ly.ln1_g; e.ln_b = ly.ln1_b; e.ln_eps = 1e-5f;
        rc = snvrag_linear(dtype, dtype, M, D, D, att, D, ly.w_o, D, x1, D, &e, stream);
        if (rc) return rc;
        // h = lrelu(x1 W1^T + b1), row stats of h for the FFN LayerNorm (one launch)
        e = snvrag_epilogue_t{};
        e.bias = ly.b1; e.act = SNVRAG_ACT_LRELU; e.slope = 0.1f; e.stats_out = (float*)stats;
        rc = snvrag_linear(dtype, dtype, M, 4 * D, D, x1, D, ly.w1, D, h, 4 * D, &e, stream);
        if (rc) return rc;
        // x = LN2(x1 + lrelu(LN_f(h) W2^T + b2)); LN_f folded into W2 and the epilogue (one launch)
        snvrag_rownorm_t rn{(const float*)stats, n_stat_parts, 4 * D, 1e-5f, ly.c2g};
        e = snvrag_epilogue_t{};
        e.bias = ly.b2g; e.act = SNVRAG_ACT_LRELU; e.slope = 0.1f; e.resid = x1; e.ld_resid = D;
        e.ln_g = ly.ln2_g; e.ln_b = ly.ln2_b; e.ln_eps = 1e-5f;
        rc = snvrag_linear_ex(dtype, dtype, M, D, 4 * D, h, 4 * D, ly.w2g, 4 * D, xc, D, &e, &rn, stream);
        if (rc) return rc;
        continue;
      }
      e = snvrag_epilogue_t{};
      e.bias = ly.b_o; e.resid = xc; e.ld_resid = D;
      rc = snvrag_linear(dtype, dtype, M, D, D, att, D, ly.w_o, D, x1, D, &e, stream);
      if (rc) return rc;
      rc = snvrag_layernorm(dtype, dtype, M, D, x1, D, nullptr, 0, ly.ln1_g, ly.ln1_b, 1e-5f, x1, D, nullptr, stream);
      if (rc) return rc;
      e = snvrag_epilogue_t{};
      e.bias = ly.b1; e.act = SNVRAG_ACT_LRELU; e.slope = 0.1f;
      rc = snvrag_linear(dtype, dtype, M, 4 * D, D, x1, D, ly.w1, D, h, 4 * D, &e, stream);
      if (rc) return rc;
      rc = snvrag_layernorm(dtype, dtype, M, 4 * D, h, 4 * D, nullptr, 0, ly.lnf_g, ly.lnf_b, 1e-5f, h, 4 * D,
                            nullptr, stream);
      if (rc) return rc;
      e = snvrag_epilogue_t{};
      e.bias = ly.b2; e.act = SNVRAG_ACT_LRELU; e.slope = 0.1f; e.resid = x1; e.ld_resid = D;
      rc = snvrag_linear(dtype, dtype, M, D, 4 * D, h, 4 * D, ly.w2, 4 * D, xc, D, &e, stream);
      if (rc) return rc;
      rc = snvrag_layernorm(dtype, dtype, M, D, xc, D, nullptr, 0, ly.ln2_g, ly.ln2_b, 1e-5f, xc, D, nullptr, stream);
      if (rc) return rc;
    }
  }
  return 0;
}
