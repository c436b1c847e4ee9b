"""kNN parity at the launch shapes the benchmark and large batches actually run.

The bench (configs[2]) searches 512 query haplotypes against a 1,000,000-haplotype,
1024-site panel: 32 query tiles -> G = 4 co-scheduled query groups sharing each panel
range (csrc/knn.hip scan2_kernel slot/group/part mapping), the n_parts >= 256 branch of
``scan_parts`` and the threshold pre-pass over a 1/64 panel prefix.  Every case here
compares the device top-k keys with the ORACLE (``oracle/knn_np.knn``, float64-exact
(distance, index) order) run on the host copy of the same panel and the same integer LUT
the device quantised; sampled queries cover every query group.

Cases:
  * bench shape:   N = 1,000,000, 1024 sites, 512 queries (G = 4), aligned masks (the
                   one-limb reduced scan), the bench's own workload generator;
  * ragged:        N = 600,000, 1000 sites, 200 queries (G = 2, last tile half full),
                   misaligned query masks (two-limb scan);
  * Aq != Ar:      N = 200,000, 96 queries whose AF embedding differs from the panel's
                   (the exact-LUT path of embedding_rag_dataset.py:193-196), checked LUT
                   and keys.
Reference behaviour: src/dataset/embedding_rag_dataset.py:390-402 (cdist + topk).
"""

from types import SimpleNamespace

import numpy as np
import pytest
import torch

from knn_helpers import decode_lut, lut_wide_flag
from oracle import knn_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _sample_queries(nq, per_group=8, seed=0):
    """Queries spread over every 128-query group (and both ends of the last tile)."""
    rng = np.random.default_rng(seed)
    out = []
    for g0 in range(0, nq, 128):
        g1 = min(nq, g0 + 128)
        pick = rng.choice(np.arange(g0, g1), size=min(per_group, g1 - g0), replace=False)
        out += sorted(set(pick.tolist()) | {g0, g1 - 1})
    return np.array(sorted(set(out)))


def _check_sampled(index, lut, nq, limbs, keys, idx, sample, k):
    """Device keys/indices of the sampled queries == oracle top-k on the host panel copy, using
    the integer LUT the device itself quantised."""
    n_sites = index.n_sites
    codes = index.codes.cpu().numpy()[:, :n_sites]
    dq = decode_lut(lut, nq, index.n_sites_pad, limbs)[sample, :n_sites]
    oi, od = knn_np.knn(codes, dq, k)
    np.testing.assert_array_equal(idx.cpu().numpy()[sample], oi)
    kk = keys.cpu().numpy().view(np.uint64)[sample]
    np.testing.assert_array_equal(kk, knn_np.pack_key(od, oi))
    return oi, od


def test_knn_bench_launch_shape_1m_512q():
    import bench
    from src.dataset import synthetic
    from src.dataset.vocab import WordVocab
    from src.engine import engine_for
    from src.model import build_model
    args = SimpleNamespace(batch=256, n_ref=1_000_000, window=1024, level=4)
    vocab = WordVocab(synthetic.POPS)
    torch.manual_seed(0)
    m = build_model(len(vocab), 384, 1, 12).to(DEV).eval()
    P = engine_for(m).packed()
    wl = bench.build_workload(args, torch.device(DEV), vocab)
    nq, k = wl.tok.shape[0], 32
    assert nq == 512 and ((nq + 15) // 16 + 7) // 8 == 4          # four co-scheduled query groups
    idx, dist, keys, lut, exps = wl.index.search(wl.tok, P.W, wl.site_mask, k, return_keys=True)
    # aligned masks + equal AF: binary Delta -> the device took the reduced one-limb scan
    assert lut_wide_flag(lut, nq, wl.index.n_sites_pad) == 0
    sample = _sample_queries(nq)
    assert len(sample) >= 32 and len({q // 128 for q in sample}) == 4
    oi, od = _check_sampled(wl.index, lut, nq, 2, keys, idx, sample, k)
    # each query's own source haplotype (2 % flips) is among its nearest neighbours
    src = np.concatenate([wl.src[:, 0], wl.src[:, 1]])[sample]
    assert np.mean([s in row for s, row in zip(src, oi)]) > 0.9
    # the search is deterministic across launches
    idx2, _ = wl.index.search(wl.tok, P.W, wl.site_mask, k)
    torch.testing.assert_close(idx2, idx, rtol=0, atol=0)


def test_knn_ragged_600k_200q_two_limb():
    from src.retrieval import PanelIndex
    n_ref, n_sites, nq, k = 600_000, 1000, 200, 32
    rng = np.random.default_rng(21)
    af = torch.from_numpy(rng.beta(0.3, 3.0, n_sites).astype(np.float32)).to(DEV)
    index = PanelIndex.synthetic(n_ref, n_sites, af, torch.zeros(1030, device=DEV), seed=5)
    assert index.n_sites_pad == 1024
    codes_h = index.codes[:, :n_sites].cpu().numpy()
    W = torch.from_numpy(rng.standard_normal((12, 64)).astype(np.float32)).to(DEV)
    site_mask = (rng.random(n_sites) < 0.4).astype(np.uint8)
    q_alle = codes_h[rng.integers(0, n_ref, nq)] ^ (rng.random((nq, n_sites)) < 0.03)
    tok = np.zeros((nq, 1030), np.int64)
    tok[:, 0] = 2
    tok[:, 1:1 + n_sites] = np.where(site_mask[None] == 1, 4, 5 + q_alle)
    tok[:, 1 + n_sites] = 3
    tok[:, 1:1 + n_sites][:, rng.random(n_sites) < 0.05] = 4     # query-only masked sites
    smask = torch.from_numpy(site_mask).to(DEV)
    idx, dist, keys, lut, exps = index.search(torch.from_numpy(tok).to(DEV), W, smask, k, return_keys=True)
    assert ((nq + 15) // 16 + 7) // 8 == 2 and nq % 16 == 8
    # the device LUT equals the oracle's quantisation of the fp64 Delta (<= 1 quantum)
    delta = knn_np.lut_delta(W.cpu().numpy(), tok, None, site_mask)
    dq_o, e_o = knn_np.quantize_lut(delta, 2)
    np.testing.assert_array_equal(exps.cpu().numpy(), e_o)
    dq_g = decode_lut(lut, nq, index.n_sites_pad, 2)
    assert np.abs(dq_g[:, :n_sites] - dq_o).max() <= 1
    sample = _sample_queries(nq, per_group=12, seed=1)
    assert {q // 128 for q in sample} == {0, 1} and nq - 1 in sample
    _check_sampled(index, lut, nq, 2, keys, idx, sample, k)


def test_knn_aq_ne_ar_exact_lut():
    """Query AF embedding != panel AF embedding: u = W[tok] + A_q - A_r per position."""
    from src.retrieval import PanelIndex
    n_ref, n_sites, nq, k, D, L = 200_000, 512, 96, 16, 64, 1030
    rng = np.random.default_rng(4)
    af = torch.from_numpy(rng.beta(0.3, 3.0, n_sites).astype(np.float32)).to(DEV)
    index = PanelIndex.synthetic(n_ref, n_sites, af, torch.zeros(L, device=DEV), seed=9)
    codes_h = index.codes[:, :n_sites].cpu().numpy()
    W = rng.standard_normal((12, D)).astype(np.float32)
    period = nq // 2                                               # A_q rows repeat (h1 | h2 of a sample)
    Aq = (0.3 * rng.standard_normal((period, L, D))).astype(np.float32)
    Ar = (0.3 * rng.standard_normal((L, D))).astype(np.float32)
    site_mask = (rng.random(n_sites) < 0.3).astype(np.uint8)
    q_alle = codes_h[rng.integers(0, n_ref, nq)] ^ (rng.random((nq, n_sites)) < 0.05)
    tok = np.zeros((nq, L), np.int64)
    tok[:, 0], tok[:, 1 + n_sites] = 2, 3
    tok[:, 1:1 + n_sites] = np.where(site_mask[None] == 1, 4, 5 + q_alle)
    T = lambda a: torch.from_numpy(a).to(DEV)
    idx, dist, keys, lut, exps = index.search(T(tok), T(W), T(site_mask), k, Aq=T(Aq), aq_period=period, Ar=T(Ar),
                                              return_keys=True)
    dA = Aq[np.arange(nq) % period] - Ar[None]
    delta = knn_np.lut_delta(W, tok, dA, site_mask)
    dq_o, e_o = knn_np.quantize_lut(delta, 2)
    np.testing.assert_array_equal(exps.cpu().numpy(), e_o)
    dq_g = decode_lut(lut, nq, index.n_sites_pad, 2)
    assert np.abs(dq_g[:, :n_sites] - dq_o).max() <= 1
    assert lut_wide_flag(lut, nq, index.n_sites_pad) == 1           # real-valued Delta: two limbs
    sample = np.arange(nq)
    _check_sampled(index, lut, nq, 2, keys, idx, sample, k)
