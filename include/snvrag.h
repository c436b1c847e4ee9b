/*
 * snvrag.h — C ABI of libsnvrag.so, the MI355X (gfx950) hot path of the v18
 * embedding-RAG SNV-imputation model (wangbaonan/RAG-SNVBERT).
 *
 * Conventions (all entry points):
 *   - plain device pointers + sizes, row-major, leading dimensions in ELEMENTS;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - caller owns every buffer (outputs and workspaces); no hidden device state;
 *   - return 0 on success, non-zero on error; snvrag_last_error() has the text
 *     (thread-local).  The Python host layer maps non-zero to RuntimeError.
 *   - dtypes: SNVRAG_F32 (exact-f32 parity path) or SNVRAG_BF16 (throughput
 *     path; f32 accumulation, f32 LayerNorm/softmax statistics).
 *
 * Each group names the reference interface it replaces (paths relative to
 * /root/reference/src).
 */
#ifndef SNVRAG_H
#define SNVRAG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNVRAG_ABI_VERSION 28

enum { SNVRAG_F32 = 0, SNVRAG_BF16 = 1 };
enum { SNVRAG_ACT_NONE = 0, SNVRAG_ACT_GELU = 1, SNVRAG_ACT_LRELU = 2, SNVRAG_ACT_SIGMOID = 3 };

int snvrag_abi_version(void);
const char* snvrag_last_error(void);
/* fills name (>= 64 bytes) with the device name of `device`; returns the CU count */
int snvrag_device_info(int device, char* name, int name_len);
/* Library options — tuning switches of the micro-benchmarks and test hooks, no reference
 * counterpart: knn_no_reduce, scan_mode, scan_nt, unfused_ln, encoder_chunk, gemm_tile128,
 * gemm_nw, tail_variant, tail_desync, sg_desync, sg_waves4, ln_bwd_nopf, attn_variant.  Each
 * starts from the environment variable SNVRAG_<NAME> (read once, at first use); launches read
 * the table. */
int snvrag_set_option(const char* name, int64_t value);
int snvrag_get_option(const char* name, int64_t* value);

/* ------------------------------------------------------------------------
 * Dense layers  (replaces torch.nn.Linear calls of model/attention/
 * multi_head_attention.py:44-51, model/utils/feed_forward.py:18-21,
 * model/fusion.py:96-117,346, model/foundation_model.py:72-80,
 * model/embedding/af_embedding.py:131-137)
 *   C[m,n] = act( sum_k A[m,k] W[n,k] + bias[n]
 *                 + row1[(m % row_period)*row1_stride] * col1[n]
 *                 + row2[(m % row_period)*row2_stride] * col2[n] )
 *            + resid[m,n]
 * The rank-1 terms fold the reference's torch.cat([x, af, af_p]) / cat([emb,
 * pos_feat, af]) input columns into the epilogue.
 * A and W share dtype_in; C/resid use dtype_out.  K must be a multiple of 8.
 * ---------------------------------------------------------------------- */
typedef struct {
  const float* bias;
  const float* row1; int64_t row1_stride; const float* col1;
  const float* row2; int64_t row2_stride; const float* col2;
  int64_t row_period;          /* 0 = no wrap */
  int act; float slope;
  const void* resid; int64_t ld_resid;
  /* LayerNorm over the whole output row, fused (needs N in {64,128,256,384}):
   *   y = ln_act(LN(v) * ln_g + ln_b);  optional y = post_base + post_scale * y * maf(post_af[m])  */
  const float* ln_g; const float* ln_b; float ln_eps; int ln_act;
  const void* post_base; int64_t ld_post; float post_scale;
  const float* post_af; int64_t post_af_period; int post_maf;
  /* per-(column tile, row) float2 (sum, sumsq) of the output: [N/tile][M] (tile = 384 when N % 384 == 0) */
  float* stats_out;
} snvrag_epilogue_t;

/* LayerNorm of the A operand folded into the epilogue (stats from a previous stats_out):
 * LN(A) W^T = rstd_m * (A W'^T) - rstd_m * mean_m * c1[n] + beta W^T, with the caller passing
 * W' = W diag(gamma), c1 = W gamma, and beta W^T added into the bias.  mean/var of row m
 * from the n_parts (sum, sumsq) partials over `dim` columns. */
typedef struct {
  const float* stats; int n_parts; int64_t dim; float eps; const float* c1;
} snvrag_rownorm_t;

int snvrag_linear(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K,
                  const void* A, int64_t lda, const void* W, int64_t ldw,
                  void* C, int64_t ldc, const snvrag_epilogue_t* epi, void* stream);
int snvrag_linear_ex(int dtype_in, int dtype_out, int64_t M, int64_t N, int64_t K,
                     const void* A, int64_t lda, const void* W, int64_t ldw,
                     void* C, int64_t ldc, const snvrag_epilogue_t* epi,
                     const snvrag_rownorm_t* rownorm, void* stream);

/* LayerNorm over the last dim, eps as given (torch default 1e-5):
 *   y = LN(x + r) * gamma + beta                  (r optional: residual of sublayer.py:15-16)
 *   post (optional): y = act(y); y = base + scale * y * w(m)   w = maf weight of af[m % period]
 *   (EnhancedRareVariantFusion tail, model/fusion.py:155-162) or w = 1.            */
typedef struct {
  const void* base; int64_t ld_base;  /* dtype_out */
  float scale;
  const float* af; int64_t af_period; int maf_weight;
  int act;                            /* applied to LN output before the base/scale step */
} snvrag_ln_post_t;

int snvrag_layernorm(int dtype_in, int dtype_out, int64_t M, int64_t N,
                     const void* X, int64_t ldx, const void* R, int64_t ldr,
                     const float* gamma, const float* beta, float eps,
                     void* Y, int64_t ldy, const snvrag_ln_post_t* post, void* stream);

/* ------------------------------------------------------------------------
 * Attention without mask (model/attention/attention.py:21-31 with
 * multi_head_attention.py head split/merge).  qkv row = [q | k | v], each
 * heads*dh wide, row stride ld_qkv; out row stride ld_out (heads*dh used).
 * softmax(q k^T * scale) v per (sequence, head).  dh in {16,32,48,64}.
 * ---------------------------------------------------------------------- */
int snvrag_attention(int dtype, int64_t nseq, int64_t L, int heads, int dh,
                     const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out,
                     float scale, void* stream);
/* Waves (32 queries each) of the bf16 dh=32 kernel that overflowed the fixed-shift
 * softmax and were recomputed with the exact online-max path since the last reset. */
int snvrag_attention_fallbacks(int reset);

/* ------------------------------------------------------------------------
 * Embedding  (model/embedding/bert.py:66-77, af_embedding.py:79-91,
 * position.py:37-38)
 * ---------------------------------------------------------------------- */
/* feat[m, j] = sin(2*pi*af[m]*f[j]), feat[m, nb+j] = cos(..), j < nb   */
int snvrag_af_features(int dtype_out, int64_t M, const float* af, const float* freqs, int nb,
                       void* feat, void* stream);
/* out[s,l,:] = W[tok[s,l]] + pe[l,:] + afemb[(s % af_period)*L + l, :]  (afemb may be NULL) */
int snvrag_embed_tokens(int dtype_out, int64_t nseq, int64_t L, int64_t D, const int64_t* tok,
                        const float* W, int64_t vocab, const float* pe, const void* afemb,
                        int afemb_dtype, int64_t af_period, void* out, void* stream);

/* PositionFeatModule (model/fusion.py:317-332), eval BatchNorm */
typedef struct {
  const float* c1_w; const float* c1_b;   /* [4,1,9], [4] */
  const float* c2_w; const float* c2_b;   /* [4,4,9], [4] */
  const float* c3_w; const float* c3_b;   /* [1,4,9], [1] */
  const float* bn1_w; const float* bn1_b; const float* bn1_rm; const float* bn1_rv;
  const float* bn2_w; const float* bn2_b; const float* bn2_rm; const float* bn2_rv;
  float bn_eps;
} snvrag_posfeat_w_t;
int snvrag_posfeat(int64_t B, int64_t L, const float* pos, const snvrag_posfeat_w_t* w,
                   float* out, void* stream);

/* CrossAFInteraction (model/fusion.py:82-86): fused_af[m,:] = af + rs*(gate*enc) */
typedef struct {
  const float* g1_w; const float* g1_b;   /* [32,2], [32] */
  const float* g2_w; const float* g2_b;   /* [D,32], [D]  */
  const float* j_w; const float* j_b;     /* [D,2],  [D]  */
  const float* ln_w; const float* ln_b;   /* [D] */
  float res_scale;
} snvrag_afgate_w_t;
int snvrag_af_gate(int dtype_out, int64_t M, int64_t D, const float* af, const float* af_p,
                   const snvrag_afgate_w_t* w, void* out, void* stream);

/* out[m, 0:D] = q[m,:];  out[m, D:2D] = rag[m,:] * wgt[m % period, :]
 * (torch.cat([orig_feat, pooled_ref]) with K=1 pooling weight 1, model/fusion.py:141-152) */
int snvrag_rag_weighted_concat(int dtype, int64_t M, int64_t D, const void* q, const void* rag,
                               const void* wgt, int64_t period, void* out, void* stream);

/* heads (model/foundation_model.py:64-80, :156-176) */
int snvrag_hap_head_out(int dtype_in, int64_t M, int64_t K, const void* H, int64_t ldh,
                        const float* w /*[2,K]*/, const float* b /*[2]*/,
                        float* logits /*[M,2] or NULL*/, float* probs /*[M,2]*/, void* stream);
typedef struct {
  const float* f_w; const float* f_b;       /* gf_fusion [16,7] */
  const float* n_w; const float* n_b;       /* gf_norm [16] */
  const float* w1; const float* b1;         /* layer.w_1 [16,16] */
  const float* ln_w; const float* ln_b;     /* layer.norm [16] */
  const float* w2; const float* b2;         /* layer.w_2 [16,16] */
  const float* c_w; const float* c_b;       /* classifier [4,16] */
} snvrag_gt_w_t;
int snvrag_gt_head(int64_t M, const float* p1, const float* p2, const float* ref,
                   const float* het, const float* hom, int64_t period,
                   const snvrag_gt_w_t* w, float* out /*[M,4]*/, void* stream);

/* ------------------------------------------------------------------------
 * Reference-panel kNN on the HBM-resident token index
 * (replaces embedding_rag_dataset.py:334-402 JIT embedding index + cdist/topk
 *  and embedding_rag_infer_dataset.py:71-224,279-285 FAISS IndexFlatL2)
 *
 * Index: codes u8 [n_ref, ld_codes], allele (0/1) of each panel haplotype at
 * each window site (ld_codes >= n_sites_pad = round_up(n_sites, 64), zero pad).
 * Distances are exact integers on a per-query power-of-two fixed-point LUT;
 * results are ordered by (distance, index) — see DESIGN.md §3.
 * ---------------------------------------------------------------------- */
/* LUT: Delta_q[s] = ||u - W[tok1]||^2 - ||u - W[tok0]||^2, u = W[tok_q[s+1]] + Aq - Ar,
 * 0 where site_mask[s]; quantised to `limbs` int8 limbs (1 or 2) in scan-fragment
 * order.  Aq: [nq_period rows of L x D] (query q uses (q % aq_period)); Aq/Ar may be NULL.
 * lut_out: knn_lut_bytes(nq, n_sites_pad, limbs); exp_out [nq] int32 scale exponents;
 * const_out [nq] f32 (distance offset; dist^2 = const + D * 2^-exp) may be NULL.      */
size_t snvrag_knn_lut_bytes(int64_t nq, int32_t n_sites_pad, int limbs);
int snvrag_knn_lut(int64_t nq, int64_t L, int64_t D, const int64_t* tok_q, const float* W,
                   const float* Aq, int64_t aq_period, const float* Ar,
                   const uint8_t* site_mask, int32_t n_sites, int32_t n_sites_pad,
                   int tok0, int tok1, int mask_tok, int limbs,
                   void* lut_out, int32_t* exp_out, float* const_out, void* stream);
/* The same LUT with the PANEL side's token table Wp separate from the query side's W:
 * Delta_q[s] = ||u - Wp[tok1]||^2 - ||u - Wp[tok0]||^2, u = W[tok_q[s+1]] + Aq - Ar.  The
 * reference caches a window's panel embeddings once per window visit and keeps searching them
 * while the weights train (embedding_rag_dataset.py:334-377, jit_cache_win_idx); Wp / Ar are
 * then the snapshot taken when that window's cache was built, W / Aq the current weights. */
int snvrag_knn_lut_panel(int64_t nq, int64_t L, int64_t D, const int64_t* tok_q, const float* W,
                         const float* Wp, const float* Aq, int64_t aq_period, const float* Ar,
                         const uint8_t* site_mask, int32_t n_sites, int32_t n_sites_pad,
                         int tok0, int tok1, int mask_tok, int limbs,
                         void* lut_out, int32_t* exp_out, float* const_out, void* stream);

/* Scan: every block scans a contiguous range of the panel and keeps an exact
 * per-query top-k (k <= 32) of its range; partial lists (ascending uint64 keys
 * ((D + 2^30) << 32 | ref_index), UINT64_MAX padding) -> part_keys [n_parts, nq, k].
 * ref_offset is added to ref indices (panel shards).  th_init (nullable, [nq]) is a per-query
 * strict upper bound on the distances worth keeping (e.g. from snvrag_knn_threshold over a
 * sample of the panel: any bound >= the true k-th distance + 1 leaves the result exact). */
int snvrag_knn_scan_parts(int64_t n_ref, int32_t nq);
int snvrag_knn_scan(const uint8_t* codes, int64_t n_ref, int64_t ld_codes, int32_t n_sites_pad,
                    const void* lut, int32_t nq, int limbs, int k, int64_t ref_offset,
                    uint64_t* part_keys, int32_t n_parts, const int32_t* th_init, void* stream);
/* th_out[q] = D of keys[q][k-1] + 1 (INT32_MAX when that slot is padding): the strict
 * threshold a second scan may start from. */
int snvrag_knn_threshold(const uint64_t* keys, int32_t nq, int k, int32_t* th_out, void* stream);
/* Merge n_lists sorted lists per query into the global top-k (exact (D, idx) order). */
size_t snvrag_topk_merge_ws_bytes(int32_t n_lists, int32_t nq, int k);
int snvrag_topk_merge(const uint64_t* keys, int32_t n_lists, int32_t nq, int k,
                      uint64_t* out_keys, void* ws, size_t ws_bytes, void* stream);
/* keys -> int64 indices (-1 for padding) and f32 squared-L2 (const + D*2^-exp) */
int snvrag_knn_decode(const uint64_t* keys, int32_t nq, int k, const int32_t* exps,
                      const float* consts, int64_t* idx_out, float* dist_out, void* stream);

/* Embedding-space exact-L2 scan (cross-check mode): the reference's literal
 * retrieval over flattened window embeddings (embedding_rag_dataset.py:390-402 torch.cdist +
 * topk; embedding_rag_infer_dataset.py:176-177 IndexFlatL2 over [N, L*D]).
 * E bf16 [N, K] panel embeddings, Q bf16 [Bq, K] queries, K % 64 == 0, Bq <= 128.
 * pack: E row-major -> Et (knn_emb_packed_bytes), the scan's index layout: 4 KiB tiles of
 *   32 rows x 64 k, tile-major over k then rows, each ordered [k-step 4][half 2][row 32][8 k],
 *   rows past N zero (done once when the index is built);
 * scan: ws (f32, knn_emb_ws_bytes) <- per-split partial dots Q Et^T;
 * finish: dist [Bq, N] f32 = qn[q] + rn[r] - 2 sum_split ws (qn, rn: squared norms).
 * splits: 1..256 (snvrag_knn_emb_splits picks one that fills the chip). */
int snvrag_knn_emb_splits(int64_t N, int64_t K, int Bq);
size_t snvrag_knn_emb_ws_bytes(int64_t N, int Bq, int splits);
size_t snvrag_knn_emb_packed_bytes(int64_t N, int64_t K);
int snvrag_knn_emb_pack(const void* E, int64_t N, int64_t K, void* Et, void* stream);
int snvrag_knn_emb_scan(const void* Et, int64_t N, int64_t K, const void* Q, int Bq, int splits, float* ws,
                        void* stream);
int snvrag_knn_emb_finish(const float* ws, int splits, int Bq, int64_t N, const float* qn, const float* rn,
                          float* dist, void* stream);

/* Mean of the k retrieved neighbours' COMPLETE-token embeddings
 * (embedding_rag_dataset.py:406-438 re-encode + bert.py:176-179 K-mean), eval:
 * out[q,l,:] = mean_j W[tok_j(l)] + pe[l] + Ar[l]; tokens: <sos>, alleles, <eos>, <pad>.
 * 1 <= k <= 128 (negative indices = no neighbour, excluded from the mean). */
int snvrag_rag_mean(int dtype_out, int64_t nq, int64_t L, int64_t D, int k, const int64_t* idx,
                    const uint8_t* codes, int64_t ld_codes, int32_t n_sites,
                    const float* W, const float* pe, const float* Ar,
                    int tok0, int tok1, int sos, int eos, int pad, void* out, void* stream);

/* Sharded panel (replaces the reference's single-process gather of the
 * neighbours' complete tokens, embedding_rag_dataset.py:404-442 / _infer_dataset.py:287-322):
 * the neighbour mean needs only the per-site alt-allele COUNT over the k neighbours.
 * snvrag_neighbor_counts: counts[q][s] = sum_j codes[idx[q][j] - row0][s] over the
 *   neighbours a shard owns (global idx in [row0, row0 + n_rows)); u8 [nq][ld_out],
 *   ld and ld_out multiples of 16, ld_out >= ld.  The shards' partials add up (all-reduce).
 * snvrag_rag_mean_counts: snvrag_rag_mean with those counts ([nq][ld_counts]) in place of
 *   the panel rows; idx gives the valid-neighbour count per query. */
int snvrag_neighbor_counts(int64_t nq, int k, const int64_t* idx, const uint8_t* codes, int64_t ld,
                           int64_t row0, int64_t n_rows, uint8_t* counts, int64_t ld_out, void* stream);
int snvrag_rag_mean_counts(int dtype_out, int64_t nq, int64_t L, int64_t D, int k, const int64_t* idx,
                           const uint8_t* counts, int64_t ld_counts, int32_t n_sites,
                           const float* W, const float* pe, const float* Ar,
                           int tok0, int tok1, int sos, int eos, int pad, void* out, void* stream);

/* Raw-genotype window index (build_ref_db_l2.py:15-98: faiss.IndexFlatL2 over each
 * sample's flattened (window_len, 2) 0/1 genotypes; test_faiss_intersect.py:171-181 the
 * Hamming twin).  Squared L2 on 0/1 vectors = Hamming distance: rows bit-packed 32
 * genotypes per word, word-major codes_wm[nw][N]; queries [nq][nw].  Writes
 * snvrag_hamming_list_count() sorted top-k key lists per query, lists[n_lists][nq][k]
 * (key = (d + 2^30) << 32 | row), to be merged by snvrag_topk_merge.  k <= 32, nw <= 2048. */
int snvrag_hamming_lists(int64_t nq, int64_t N, int32_t nw, int k, const uint32_t* codes_wm,
                         const uint32_t* queries, uint64_t* lists, void* stream);
int32_t snvrag_hamming_list_count(void);

/* Deterministic synthetic panel on device: code = (u(seed,r,s) < af[s]), u = splitmix64
 * hash (src/dataset/synthetic.py hash_uniform), zero padding to ld.  _rows: rows
 * [row0, row0 + n_rows) of that panel (a shard). */
int snvrag_panel_synth(uint8_t* codes, int64_t n_ref, int64_t ld, int32_t n_sites,
                       const float* af, uint64_t seed, void* stream);
int snvrag_panel_synth_rows(uint8_t* codes, int64_t row0, int64_t n_rows, int64_t ld, int32_t n_sites,
                            const float* af, uint64_t seed, void* stream);

/* ------------------------------------------------------------------------
 * Encoder stack (model/transformer.py:27-30 x n_layers, model/bert.py:213-217),
 * eval: x <- LN2(x1 + FFN(x1)), x1 = LN1(x + MHA(x)).  x is [nseq*L, D] in place.
 * ---------------------------------------------------------------------- */
typedef struct {
  const void* w_qkv; const float* b_qkv;   /* [3D, D] rows q;k;v (dtype), [3D] */
  const void* w_o; const float* b_o;       /* [D, D], [D] */
  const float* ln1_g; const float* ln1_b;  /* input_sublayer.norm */
  const void* w1; const float* b1;         /* [4D, D], [4D] */
  const float* lnf_g; const float* lnf_b;  /* feed_forward.norm [4D] */
  const void* w2; const float* b2;         /* [D, 4D], [D] */
  const float* ln2_g; const float* ln2_b;  /* output_sublayer.norm */
  /* feed_forward.norm folded into w_2 (fused path): w2g = w2 diag(lnf_g),
   * b2g = b2 + w2 lnf_b, c2g = w2 lnf_g */
  const void* w2g; const float* b2g; const float* c2g;
  /* factor already folded into the q rows of w_qkv / b_qkv (0 = none); the bf16 engine
   * folds log2(e)/sqrt(dh) so attention's exp2 needs no per-score scaling */
  float q_scale;
  /* optional (bf16, D in {128,256,384}): the block tail's vector table (ffn_vec of
   * snvrag_tail_forward) and snvrag_tail_pack of (w_o, w1, w2g) -> the whole block tail runs
   * on the 32x32-MFMA kernel (snvrag_tail_forward); NULL = the row-panel GEMM path */
  const float* ffn_v;
  const void* tail_w;
  /* optional (bf16, D in {128,256,384}): snvrag_proj_pack of w_qkv (NC = 3) -> the QKV
   * projection runs on snvrag_proj_forward when it is too large for the stream GEMM */
  const void* qkv_pw;
  /* optional (bf16, D in {128,256,384}): snvrag_sgemm_pack of w_qkv -> the QKV projection runs on
   * the stream GEMM (snvrag_sgemm_forward, epi 0); takes precedence over qkv_pw while
   * M * 3D * 2 bytes < 2^31 */
  const void* qkv_sg;
} snvrag_layer_t;

/* Block tail on 32x32x16 MFMAs (csrc/tail.hip), bf16, eval — same math as
 * x1 = LN1(x + att W_o^T + b_o); x = LN2(x1 + FFN(x1)), in place
 * on x.  128 token rows per workgroup (4 waves x 32 rows), activations in registers, the
 * LDS a 9-slot ring of 16 KiB weight slabs.  ONE weight stream of snvrag_tail_pack_bytes(D)
 * bytes packed by snvrag_tail_pack(D, w_o [D,D], w1 [4D,D], w2g [D,4D], out, stream)
 * with w2g = w2 diag(lnf_g) (the FFN LayerNorm's gamma folded in).  ffn_vec is an f32
 * table of 8*D floats (16-byte aligned): [b1 4D | b2' D | c1 D | ln2_g D | ln2_b D] with
 * b2' = b2 + w2 lnf_b and c1[n] = sum_k w2g[n,k] (of the bf16 values).  att and x must not
 * alias; pointers 16-byte aligned; D in {128, 256, 384}.
 * snvrag_tail_ffn_forward: the FFN sublayer alone (out = LN2(x1 + FFN(x1))), same stream. */
size_t snvrag_tail_pack_bytes(int D);
int snvrag_tail_pack(int D, const void* w_o, const void* w1, const void* w2g, void* out, void* stream);
int snvrag_tail_forward(int64_t M, int D, const void* att, void* x, const void* wstream, const float* b_o,
                        const float* ln1_g, const float* ln1_b, const float* ffn_vec, float eps, void* stream);
int snvrag_tail_ffn_forward(int64_t M, int D, const void* x1, void* out, const void* wstream,
                            const float* ffn_vec, float eps, void* stream);
/* Diagnostics: buffer of [workgroups][4 waves][10] uint64 phase stamps filled by the block tail at
 * D = 384 when SNVRAG_TAIL_VARIANT=4 (a separate stamped instantiation; NULL turns it off). */
int snvrag_tail_stamps(void* buf);
/* Projection on the same 32x32-MFMA stream machinery (the QKV projection of
 * multi_head_attention.py:44-46, bf16): out[M, NC*D] = x[M, D] W^T + bias with W [NC*D, D]
 * packed once by snvrag_proj_pack (snvrag_proj_pack_bytes(D, NC) bytes); D in {128, 256,
 * 384}, NC in {1, 3}; bias f32 [NC*D]. */
size_t snvrag_proj_pack_bytes(int D, int NC);
int snvrag_proj_pack(int D, int NC, const void* w, void* out, void* stream);
int snvrag_proj_forward(int64_t M, int D, int NC, const void* x, const void* wstream, const float* bias,
                        void* out, void* stream);

/* Stream GEMM on 32x32x16 MFMAs (csrc/sgemm.hip), bf16, eval: x [M, D] W^T with W [N, D]
 * packed once by snvrag_sgemm_pack (snvrag_sgemm_pack_bytes(D, N) bytes; D in {128, 256,
 * 384}, or 768 for epi 0 with GELU (fusion.py:157 over cat(h, g r)); N % 64 == 0), output tiles streamed outermost so each tile's epilogue runs under the
 * next tiles' MFMAs.  vec (f32) = [bias N | c1 N, c2 N when r1 | LN: g N, be N | head: w_out
 * [2, N], b_out 2]; rank terms r1[m % period] c1 + r2[m % period] c2 join the bias (the
 * cat(x, pos, af) / cat(x, af, af_p) Linear inputs of fusion.py:355-360 and
 * foundation_model.py:25-33 without widening K); r1 = NULL: none.  epi:
 *   0  out[M, N] = act(.)                      bf16 (act: NONE / GELU)
 *   1  probs[M, 2] = softmax(act(.) w_out^T + b_out), logits (nullable) [M, 2] f32
 *      (foundation_model.py:77-80; N = 4D, act GELU, no rank terms)
 *   2  out[M, D] = LN(act(.) + x) g + be       bf16 (N = D, act LeakyReLU(slope);
 *      fusion.py:355-360) */
/* The same with a concatenated input built in registers (fusion.py:157, rag_fusion's
 * cat(h, aw * h_rag) -> Linear(2D, 4D) -> GELU, without materialising the [M, 2D] cat):
 * out[M, N] = GELU([q | bf16(x2 * g2[m % period2])] W^T + b), q and x2 [M, Dh], g2 [period2, Dh]
 * (bf16), W [N, 2 Dh] packed with snvrag_sgemm_pack(2 Dh, N, ...), vec = bias [N]; Dh = 384. */
int snvrag_sgemm_cat_forward(int64_t M, int Dh, int N, const void* q, const void* x2, const void* g2,
                             int64_t period2, const void* wstream, const float* vec, void* out, void* stream);
/* Two projections in one launch with the [M, 4D] hidden on chip (fusion.py:131-141 af_adapter,
 * foundation_model.py:25-33 af_fusion), bf16, eval, D = 384:
 *   out[M, D] = EPI2(GELU(x W1^T + b1 [+ r1[m % period] c1 + r2[m % period] c2]) W2^T + b2)
 * epi2: 0 sigmoid, 1 LayerNorm (g, be).  W1 [4D, D], W2 [D, 4D] packed once by snvrag_mlp_pack
 * (snvrag_mlp_pack_bytes(D) bytes); vec (f32) = [b1 4D | c1 4D, c2 4D when r1 | b2 D | g D, be D
 * when epi2 = 1]. */
size_t snvrag_mlp_pack_bytes(int D);
int snvrag_mlp_pack(int D, const void* w1, const void* w2, void* out, void* stream);
int snvrag_mlp_forward(int64_t M, int D, int epi2, const void* x, const void* wstream, const float* vec,
                       const float* r1, const float* r2, int64_t period, float eps, void* out, void* stream);
/* The af_adapter chain with its input computed in the prologue (fusion.py:135-138: fused_af =
 * CrossAFInteraction(af, af_p), then af_adapter = Linear(D, 4D) -> GELU -> Linear(4D, D) -> Sigmoid):
 * out bf16 [M, D] from af, af_p f32 [M] in ONE launch (snvrag_af_gate + snvrag_mlp_forward epi2 0).
 * D = 384.  wstream: snvrag_mlp_pack of (a0, a3); vec (f32) = [b1 4D | b2 D | g2_b D | j_w[:, 0] D |
 * j_w[:, 1] D | j_b D | ln_w D | ln_b D | g1_w 64 (row-major [32, 2]) | g1_b 32 | m0 m1 mb S00 S11 S01
 * S0b S1b Sbb] with m the column means of (j_w[:, 0], j_w[:, 1], j_b) and S their centred second
 * moments (1 / D); gate_frags: the gate GEMV's W2 [D, 32] as 12 tiles x 2 k16 steps x (bf16 hi,
 * bf16 lo = bf16(W2 - hi)) 1 KiB MFMA fragments, lane l = (m = l % 32, h = l / 32) of fragment
 * (T, s, part) holding W2[32 T + 16 ((m / 4) % 2) + 4 (m / 8) + m % 4][16 h + 8 s + 0 .. 7]
 * (src/kernels.py mlp_afgate_pack). */
int snvrag_mlp_afgate_forward(int64_t M, int D, const float* af, const float* af_p, const void* gate_frags,
                              float res_scale, const void* wstream, const float* vec, void* out, void* stream);
size_t snvrag_sgemm_pack_bytes(int D, int N);
int snvrag_sgemm_pack(int D, int N, const void* w, void* out, void* stream);

/* Derived weight tensors of the training graph, all refreshed from the f32 master parameters
 * in ONE launch after each optimizer step (the bf16 GEMM operands the kernels read: stream-GEMM
 * packs, transposed / concatenated bf16 copies, f32 bias tables).  A job reads a source matrix
 * of `rows` x `cols` f32 elements made of up to 4 parts stacked along the rows, part i being
 * the strided view src[i][r * rs[i] + c * cs[i]] of part_rows[i] rows, and writes
 *   kind 0: f32   dst[r * dst_ld + c]
 *   kind 1: bf16  dst[r * dst_ld + c]   (round to nearest even, as the optimizer's bf16 mirror)
 *   kind 2: bf16  snvrag_sgemm_pack of the (rows = N) x (cols = D) matrix (dst_ld unused),
 *   kind 3: bf16  snvrag_gemm256_pack of the (rows = N) x (cols = K) matrix (dst_ld unused).
 * Job j owns the output pieces (8 elements) [piece0, piece0 + pieces); jobs sorted by piece0,
 * piece0[0] = 0, total = the last job's piece0 + pieces.  `jobs` is a DEVICE pointer. */
typedef struct {
  int32_t kind, nparts;
  int64_t rows, cols, dst_ld, piece0, pieces;
  int64_t part_rows[4], rs[4], cs[4];
  const float* src[4];
  void* dst;
} snvrag_derive_job_t;
int snvrag_derive(const snvrag_derive_job_t* jobs, int njobs, int64_t total_pieces, void* stream);

/* Wide-row GEMM (gemm256.hip) for the large-K projections onto N = 384 features of training:
 * FeedForward's w_2 forward (feed_forward.py:20, K = 4D) and the dX GEMMs with K = 3D / 4D of the
 * backward of the attention projections and of w_1 (the autograd of pretrain_with_val_optimized.py:
 * 235).  out bf16 [M, N] (ldo) = A bf16 [M, K] (lda) W^T (+ bias f32 [N]) (+ resid bf16 [M, N]),
 * f32 accumulation, one rounding.  W bf16 [N, K] (ldw) is packed once into
 * snvrag_gemm256_pack_bytes(N, K) bytes (or by snvrag_derive kind 3).  N = 384, K % 64 == 0, rows
 * and pointers 16-byte aligned. */
size_t snvrag_gemm256_pack_bytes(int N, int K);
int snvrag_gemm256_pack(int N, int K, const void* w, int64_t ldw, void* out, void* stream);
int snvrag_gemm256_forward(int64_t M, int N, int K, const void* A, int64_t lda, const void* wpacked, const float* bias,
                           const void* resid, int64_t ld_resid, void* out, int64_t ldo, void* stream);
/* The same GEMM with the rag fusion's tail as its epilogue (fusion.py:152-162: fusion[3] Linear(4D, D)
 * -> fusion[4] LayerNorm -> MAF weighting -> residual, replacing the row-panel GEMM's LN/post epilogue
 * of snvrag_linear for this call): y = A W^T + bias (f32); v = LN(y) * ln_g + ln_b over the N = 384
 * outputs of a row (two-pass mean / variance, eps); out = base + post_scale * v * w(af[m % period])
 * with w(a) = min(log1p(1 / (min(a, 1 - a) + 1e-6)), 3) (post_af null: w = 1; base null: out = v).
 * Inference / eval only (no saved statistics). */
int snvrag_gemm256_ln_forward(int64_t M, int N, int K, const void* A, int64_t lda, const void* wpacked,
                              const float* bias, const float* ln_g, const float* ln_b, float eps, const void* base,
                              int64_t ld_base, float post_scale, const float* post_af, int64_t post_af_period,
                              void* out, int64_t ldo, void* stream);

/* The hap head's Linear(K, 2) (foundation_model.py:25-33 net[2]) in training: x bf16 [M, K],
 * w f32 [2, K], b f32 [2] -> out f32 [M, 2] = x w^T + b.  Backward: dx bf16 [M, K] = g w (optional),
 * dw f32 [2, K] = g^T x (written, or added when accumulate; optional), g f32 [M, 2];
 * ws: snvrag_head2_ws_bytes(M, K).  K % 8 == 0. */
int snvrag_head2_fwd(int64_t M, int K, const void* x, const float* w, const float* b, float* out, void* stream);
size_t snvrag_head2_ws_bytes(int64_t M, int K);
/* Weight gradient of a V-row token table (embedding/bert.py:63-75 TokenEmbedding under autograd):
 * dw f32 [V, D] = sum over m of onehot(tok[m]) g[m] (rows with tok = padding_idx skipped; pass -1
 * for none); tok int64 [M], g f32 [M, D]; V <= 16, D even; deterministic; written, not added.
 * ws: snvrag_tokgrad_ws_bytes(M, V, D). */
size_t snvrag_tokgrad_ws_bytes(int64_t M, int V, int D);
int snvrag_tokgrad(int64_t M, int V, int D, int padding_idx, const int64_t* tok, const float* g, float* dw,
                   void* ws, size_t ws_bytes, void* stream);
int snvrag_head2_bwd(int64_t M, int K, const float* g, const void* x, const float* w, void* dx, float* dw,
                     int accumulate, void* ws, size_t ws_bytes, void* stream);
int snvrag_sgemm_forward(int64_t M, int D, int N, int epi, int act, float slope, const void* x,
                         const void* wstream, const float* vec, const float* r1, const float* r2,
                         int64_t period, float eps, void* out, float* probs, float* logits, void* stream);

size_t snvrag_encoder_ws_bytes(int dtype, int64_t nseq, int64_t L, int D, int heads);
int snvrag_encoder_forward(int dtype, int64_t nseq, int64_t L, int D, int heads, int n_layers,
                           const snvrag_layer_t* layers, void* x, void* ws, size_t ws_bytes,
                           void* stream);

/* Event log for live per-kernel timing (bench.py): when enabled, GEMM / attention /
 * LayerNorm / kNN-scan launches record a HIP event pair on their stream plus their
 * algorithmic work (FLOPs, or bytes for LN / kNN scan).  kinds: 1 GEMM, 2 attention,
 * 3 LayerNorm, 4 kNN scan.  enable(capacity<=0) frees the log. */
int snvrag_evlog_enable(int capacity);
int snvrag_evlog_pause(int paused);
int snvrag_evlog_reset(void);
int snvrag_evlog_read(int* kinds, float* ms, double* work, int max);

/* ---------------------------------------------------------------- training --
 * Replaces the autograd backward of model/attention/attention.py:21-31 (via
 * multi_head_attention.py:44-51) and the trainer step of
 * main/pretrain_with_val_optimized.py:210-245 (FocalLoss optim_schedule.py:64-96,
 * clip_grad_norm_, fused torch.optim.Adam, cal_pr optim_schedule.py:167-203).
 *
 * attention_train_fwd: bf16 qkv [nseq*L, ld_qkv] (q | k | v column blocks) -> out
 *   [nseq*L, ld_out] and lse [nseq][heads][L] f32 (log2 domain: P = exp2(c s - lse),
 *   c = scale*log2 e).  attention_bwd: dout [nseq*L, ld_dout] -> dqkv (same layout as
 *   qkv, bf16); d_ws f32 [nseq*heads*L] scratch (rowsum(dO o O)).  dh in {32, 64}.
 *   dropout_p > 0: attention-probability dropout (attention.py:28-29) with the counter-based
 *   keep mask of csrc/attn_common.h (seed; the backward must get the forward's p and seed). */
int snvrag_attention_train_fwd(int64_t nseq, int64_t L, int heads, int dh, const void* qkv, int64_t ld_qkv,
                               void* out, int64_t ld_out, float* lse, float scale, float dropout_p,
                               uint64_t seed, void* stream);
int snvrag_attention_bwd(int64_t nseq, int64_t L, int heads, int dh, const void* qkv, int64_t ld_qkv,
                         const void* out, int64_t ld_out, const void* dout, int64_t ld_dout,
                         const float* lse, float* d_ws, void* dqkv, int64_t ld_dqkv, float scale,
                         float dropout_p, uint64_t seed, void* stream);
/* focal loss over rows with mask[m] != 0: probs [M, C] f32 (the heads' softmax output),
 * labels int64 [M]; loss_sum += weight * sum_m FL_m (caller zeroes it); grad [M, C] =
 * weight * dFL/dprobs (0 on unmasked rows). */
int snvrag_focal_loss(int64_t M, int C, const float* probs, const int64_t* labels, const uint8_t* mask,
                      float gamma, float weight, float* loss_sum, float* grad, void* stream);
/* acc = sum x^2 in a fixed reduction order (bit-identical for identical x). x 16-byte aligned.
 * snvrag_sqnorm keeps its per-block partials in one process-wide device buffer: one call in flight
 * per device (stream-ordered); snvrag_sqnorm_ws takes a caller-owned workspace of
 * snvrag_sqnorm_ws_bytes() bytes instead, so calls on different streams may overlap. */
int snvrag_sqnorm(int64_t n, const float* x, float* acc, void* stream);
size_t snvrag_sqnorm_ws_bytes(void);
int snvrag_sqnorm_ws(int64_t n, const float* x, float* acc, float* ws, size_t ws_bytes, void* stream);
typedef struct {
  float lr, beta1, beta2, eps, weight_decay;
  float grad_scale;     /* g <- g * grad_scale (1/world for summed DDP gradients) */
  float max_norm;       /* > 0: clip the scaled gradient to this L2 norm using *sqnorm */
  int step;             /* 1-based */
} snvrag_adam_t;
/* One Adam step over a flat f32 buffer; p_bf16 (nullable) receives bf16(p_new);
 * sqnorm (nullable) = snvrag_sqnorm of g (unscaled). */
int snvrag_adam_step(int64_t n, float* p, const float* g, float* m, float* v, void* p_bf16,
                     const float* sqnorm, const snvrag_adam_t* a, void* stream);
/* counts [3][C] uint64 (tp, fp, fn) += over rows with mask[m] (and mask2[m] when given). */
int snvrag_confusion(int64_t M, int C, const float* probs, const int64_t* labels, const uint8_t* mask,
                     const uint8_t* mask2, uint64_t* counts, void* stream);

/* Training LayerNorm (sublayer.py:15-16, feed_forward.py:20, nn.LayerNorm under autograd):
 * y = drop_o(LN(x + drop_r(r)) g + b), bf16 [M, N] in/out (r nullable), f32 statistics; writes
 * s = bf16(x + drop_r(r)) (when r is given) and stats [M] = (mean, rstd) for the backward.  The
 * dropouts around the norms (sublayer.py / transformer.py: nn.Dropout) are fused: p_r on the
 * residual operand, p_out on the output, counter-based keep masks of (seed, row, column)
 * (attn_common.h's hash; streams 0 / 1), regenerated by the backward.  The backward returns
 * ds (= dx; = dr when p_r == 0), dres = the masked ds (the gradient of r when p_r > 0), and
 * dg, db (f32 [N]) written, or added to their contents when accumulate != 0 (the parameters'
 * .grad buffers).  N % 8 == 0, N <= 2048. */
int snvrag_ln_fwd_train(int64_t M, int N, const void* x, const void* r, const float* g, const float* b,
                        float eps, void* y, void* s_out, float* stats, float p_r, float p_out, uint64_t seed,
                        void* stream);
/* The same with FeedForward's LeakyReLUs fused (feed_forward.py:20-21): slope_x != 0 (no
 * residual): y = LN(lrelu(x)), s_out unused (the backward's s is x itself); slope_r != 0:
 * s = x + drop(lrelu(r)).  Backward: slope_x: s = the pre-activation x, ds = d/dx through the
 * activation; slope_r: r_pre = the pre-activation r, dres = d/dr (always written). */
int snvrag_ln_fwd_train_act(int64_t M, int N, const void* x, const void* r, const float* g, const float* b,
                            float eps, void* y, void* s_out, float* stats, float p_r, float p_out, uint64_t seed,
                            float slope_x, float slope_r, void* stream);
int snvrag_ln_bwd_act(int64_t M, int N, const void* dy, const void* s, const float* stats, const float* g,
                      void* ds, void* dres, const void* r_pre, float* dg, float* db, int accumulate, float p_r,
                      float p_out, uint64_t seed, float slope_x, float slope_r, void* ws, size_t ws_bytes,
                      void* stream);
/* Train-mode neighbour mean with the reference's dropout semantics (embedding_rag_dataset.py:
 * 404-417, bert.py:176-179): out[q, l] = mean over q's valid neighbours j of
 * drop(W[tok(u, l)] + pe[l] + Ar[l]), u = inv[q, j] (< 0: none) indexing the window's unique
 * neighbours (their allele codes [U, ld_codes]); one dropout mask per unique neighbour (counter-
 * based hash of seed, u, l, feature pair), never materialising the [U, L, D] embeddings.  The
 * backward ACCUMULATES dW [V, D] (not the <pad> row) and dAr [L, D]. */
int snvrag_nbr_mean_drop_fwd(int64_t nq, int k, int64_t L, int D, int n_sites, int64_t ld_codes, int V,
                             const int32_t* inv, const uint8_t* codes, const float* W, const float* pe,
                             const float* Ar, float p, uint64_t seed, int tok0, int sos, int eos, int pad,
                             float* out, void* stream);
int snvrag_nbr_mean_drop_bwd(int64_t nq, int k, int64_t L, int D, int n_sites, int64_t ld_codes, int V,
                             const int32_t* inv, const uint8_t* codes, const float* W, const float* pe,
                             const float* Ar, float p, uint64_t seed, int tok0, int sos, int eos, int pad,
                             const float* dout, float* dW, float* dAr, void* stream);
size_t snvrag_ln_bwd_ws_bytes(int64_t M, int N);
int snvrag_ln_bwd(int64_t M, int N, const void* dy, const void* s, const float* stats, const float* g,
                  void* ds, void* dres, float* dg, float* db, int accumulate, float p_r, float p_out,
                  uint64_t seed, void* ws, size_t ws_bytes, void* stream);
/* out[n] = sum_m x[m, n] for a bf16 [M, N] matrix (Linear bias gradients), f32 out. */
size_t snvrag_colsum_ws_bytes(int64_t M, int N);
int snvrag_colsum_bf16(int64_t M, int N, const void* x, float* out, void* ws, size_t ws_bytes, void* stream);

/* Weight (and bias) gradient of a Linear layer (the backward of pretrain_with_val_optimized.py:235
 * through every nn.Linear of multi_head_attention.py:44-51, feed_forward.py:18-21, fusion.py,
 * foundation_model.py), csrc/dw.hip: dw[N, K] += sum_m dy[m, n] x[m, k] and, db != NULL,
 * db[N] += sum_m dy[m, n]; dy [M, N], x [M, K] bf16 row-major, f32 results ACCUMULATED (zero them
 * first; a parameter's f32 .grad can be passed directly), rows of dy / x ldy / ldx elements apart
 * (a column slice of a fused N: the q/k/v parts).  32x32x16 MFMAs on LDS-transposed tiles, M split into `splits` chunks (0: enough to fill
 * the chip, snvrag_dw_splits) whose 128 x 128 tiles are added with float atomics (the summation
 * order across chunks is not fixed).  N, K multiples of 128. */
int snvrag_dw_splits(int64_t M, int64_t N, int64_t K);
int snvrag_linear_dw(int64_t M, int64_t N, int64_t K, const void* dy, int64_t ldy, const void* x, int64_t ldx,
                     float* dw, float* db, int splits, void* stream);
/* The same over a fused output of n_parts equal parts (the q/k/v Linear layers of one N = 3D
 * GEMM, multi_head_attention.py:44): part i's dW rows / db entries accumulate into
 * dw_parts[i] [N / n_parts, K] / db_parts[i] (host arrays of device pointers; db_parts nullable).
 * 1 <= n_parts <= 4, (N / n_parts) % 128 == 0. */
int snvrag_linear_dw_parts(int64_t M, int64_t N, int64_t K, const void* dy, int64_t ldy, const void* x,
                           int64_t ldx, int n_parts, float* const* dw_parts, float* const* db_parts, int splits,
                           void* stream);

/* Inference post-processing (replaces infer_embedding_rag.py:145-152): probs_h1/h2 [M, 2]
 * f32 head probabilities -> p1, p2 [M] = softmax(probs)[..., 1] (the reference's second
 * softmax) and gt [M, 4] = (p00, p01, p10, p11).  gt 16-byte aligned. */
int snvrag_infer_post(int64_t M, const float* probs_h1, const float* probs_h2, float* p1, float* p2,
                      float* gt, void* stream);

/* self tests of MFMA operand/accumulator layouts used by the kernels (GPU only):
 * returns 0 when the i8 / bf16 / f32 MFMA maps match the CPU product. */
int snvrag_selftest_mfma(void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SNVRAG_H */
