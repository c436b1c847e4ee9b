"""Embedding-space panel index (the reference's literal cdist/IndexFlatL2 retrieval, kept as a
cross-check of the token-resident index; SURVEY.md §8d C2 mode).

CPU: the panel tokenisation equals WordVocab.tokenize of the same alleles + window mask.
GPU: the distance-GEMM kernel (csrc/knn_emb.hip) against float64 on the same bf16 values, and the
embedding-space top-k against the token index's exact distances.
"""

import numpy as np
import pytest
import torch

from knn_helpers import rand_case


def test_panel_tokens_match_vocab_tokenize():
    from src.dataset import synthetic
    from src.dataset import utils as U
    from src.dataset.vocab import WordVocab
    from src.retrieval import panel_tokens
    rng = np.random.default_rng(3)
    vocab = WordVocab(synthetic.POPS)
    n_sites = 300
    alle = rng.integers(0, 2, (17, n_sites)).astype(np.uint8)
    raw_mask = (rng.random(n_sites) < 0.3).astype(np.int64)
    mask = U.sequence_padding(raw_mask, "int")
    ref = vocab.tokenize(alle, mask)
    codes = torch.zeros(17, 512, dtype=torch.uint8)
    codes[:, :n_sites] = torch.from_numpy(alle)
    got = panel_tokens(codes, n_sites, mask, ref.shape[1])
    np.testing.assert_array_equal(got.numpy(), ref)


def _f64_dist(Q, E):
    q, e = Q.double(), E.double()
    return (q * q).sum(1)[:, None] + (e * e).sum(1)[None] - 2 * q @ e.T


@pytest.mark.gpu
@pytest.mark.parametrize("N,Kd,Bq,splits", [(1000, 64 * 7, 1, None), (333, 1030 * 32, 33, None), (2049, 4096, 64, 5),
                                            (700, 64 * 101, 96, None), (129, 640, 128, 1), (64, 64, 48, 3),
                                            (1500, 1030 * 384, 96, None)])   # the bench's K (C2: L*D)
def test_knn_emb_distance_kernel_vs_f64(N, Kd, Bq, splits):
    from src import kernels as K
    g = torch.Generator(device="cuda").manual_seed(N + Kd)
    E = torch.randn(N, Kd, device="cuda", generator=g).bfloat16()
    Q = torch.randn(Bq, Kd, device="cuda", generator=g).bfloat16()
    rn = K.knn_emb_norms(E)
    torch.testing.assert_close(rn.double(), (E.double() ** 2).sum(1), rtol=1e-5, atol=1e-3)
    Et = K.knn_emb_pack(E)
    # the packed layout: 4 KiB tiles [k-step 4][half 2][row 32][8 k], padding rows zero
    assert Et.shape[0] == (N + 31) // 32 * 32
    t = Et.view(-1, Kd // 64, 4, 2, 32, 8).permute(0, 4, 1, 2, 3, 5).reshape(-1, Kd)
    assert torch.equal(t[:N], E) and not t[N:].any()
    d = K.knn_emb_dist(Et, Q, rn, splits=splits)
    ref = _f64_dist(Q, E)
    # f32 accumulation over K terms of |q e| ~ 1: error ~ sqrt(K) * 2^-24 * scale; the norms
    # are ~K, so bound relative to them
    tol = 2e-5 * Kd + 1e-3
    assert (d.double() - ref).abs().max().item() <= tol


@pytest.mark.gpu
def test_embedding_space_search_agrees_with_token_index():
    """The literal embedding-space search (bf16 E, f32 norms) returns neighbours whose EXACT
    distance (float64 sums of ||W[a] - W[b]||^2 over positions) is within noise of the token
    index's exact k-th distance, and its distances match the exact ones to bf16-rounding
    level; the token index's own neighbours are bit-exact (tests/test_gpu_kernels.py)."""
    from src.retrieval import EmbeddingIndex, PanelIndex, panel_tokens
    n_ref, n_sites, nq, k = 3000, 300, 40, 16
    W, panel, site_mask, tok = rand_case(n_ref, n_sites, nq, 21)
    L, D = tok.shape[1], W.shape[1]
    rng = np.random.default_rng(5)
    pe = torch.from_numpy(rng.standard_normal((L, D)).astype(np.float32)).cuda()
    Ar = torch.from_numpy(rng.standard_normal((L, D)).astype(np.float32)).cuda()
    Wt = torch.from_numpy(W).cuda()
    pidx = PanelIndex.from_alleles(panel, np.zeros(L, np.float32), "cuda")
    tq = torch.from_numpy(tok).cuda()
    idx_t, _ = pidx.search(tq, Wt, torch.from_numpy(site_mask).cuda(), k)
    mask_tok = np.zeros(L, np.int64)
    mask_tok[1:1 + n_sites] = site_mask
    tr = panel_tokens(pidx.codes, n_sites, mask_tok, L)
    eidx = EmbeddingIndex.build(tr, Wt, pe, Ar)
    d_e, idx_e = eidx.search(eidx.embed_queries(tq, Wt, pe, Ar), k)
    # exact distances: T[a, b] = ||W[a] - W[b]||^2 summed over token positions
    W64 = W.astype(np.float64)
    T = ((W64[:, None] - W64[None]) ** 2).sum(-1)
    trn = tr.cpu().numpy()
    exact = np.zeros((nq, n_ref))
    for l in range(L):
        exact += T[tok[:, l]][:, trn[:, l]]
    ie, it = idx_e.cpu().numpy(), idx_t.cpu().numpy()
    de_exact = np.take_along_axis(exact, ie, 1)
    kth = np.take_along_axis(exact, it, 1)[:, -1]
    assert (de_exact <= kth[:, None] + 1.0).all()
    np.testing.assert_allclose(d_e.cpu().numpy(), de_exact, rtol=2e-3, atol=1.0)
    # same multiset of exact distances as the token index's top-k
    np.testing.assert_allclose(np.sort(de_exact, 1), np.take_along_axis(exact, it, 1), rtol=0, atol=1.0)
