"""Pin the ORACLE against fixtures produced by running the reference (tests/golden/make_golden.py)."""

import numpy as np
import pytest

from conftest import golden_state_dict, load_golden
from oracle import data_np, knn_np, model_np

CASES = ["fwd_tiny", "fwd_small", "fwd_full"]


def _inputs(g, which="ref"):
    I1, I2 = (g["Iref_h1"], g["Iref_h2"]) if which == "ref" else (g["Ican_h1"], g["Ican_h2"])
    return I1, I2


@pytest.mark.parametrize("case", CASES)
def test_oracle_forward_matches_reference(case):
    g = load_golden(case)
    cfg = g["cfg"]
    sd = golden_state_dict(cfg)
    x = {k: g[k] for k in ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom")}
    for which, pre in (("ref", ""), ("can", "can_")):
        I1, I2 = _inputs(g, which)
        x["rag_mean_h1"] = model_np.rag_mean(g["ref_complete"], I1, g["ref_af"], sd)
        x["rag_mean_h2"] = model_np.rag_mean(g["ref_complete"], I2, g["ref_af"], sd)
        o = model_np.forward(x, sd, cfg["layers"], cfg["heads"])
        for key in ("logits_h1", "logits_h2"):
            np.testing.assert_allclose(o[key], g[pre + key], rtol=1e-4, atol=1e-4)
        for key in ("probs_h1", "probs_h2", "gt"):
            np.testing.assert_allclose(o[key], g[pre + key], rtol=1e-4, atol=1e-5)


def test_oracle_norag_forward_matches_reference():
    """configs[0] path: no retrieved embeddings in the batch (bert.py:207-210)."""
    g = load_golden("fwd_norag")
    cfg = g["cfg"]
    sd = golden_state_dict(cfg)
    x = {k: g[k] for k in ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom")}
    o = model_np.forward(x, sd, cfg["layers"], cfg["heads"])
    for key in ("logits_h1", "logits_h2"):
        np.testing.assert_allclose(o[key], g[key], rtol=1e-4, atol=1e-4)
    for key in ("probs_h1", "probs_h2", "gt"):
        np.testing.assert_allclose(o[key], g[key], rtol=1e-4, atol=1e-5)


def test_oracle_intermediates_tiny():
    g = load_golden("fwd_tiny")
    sd = golden_state_dict(g["cfg"])
    np.testing.assert_allclose(model_np.af_embedding(g["af"], sd), g["af_emb"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(model_np.embed(g["hap_1"], g["af"], sd), g["emb_h1"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(model_np.pos_feat(g["pos"], sd), g["posfeat"], rtol=1e-5, atol=1e-6)
    rm = model_np.rag_mean(g["ref_complete"], g["Iref_h1"], g["ref_af"], sd)
    np.testing.assert_allclose(rm, g["rag_mean_h1"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", CASES)
def test_oracle_knn_canonical_and_tie_equivalent(case):
    """Canonical (dist, idx) kNN on the quantised LUT == fixture canonical order; the reference's
    fp32 cdist picks are the same multiset of exact distances (tie-equivalent)."""
    g = load_golden(case)
    cfg = g["cfg"]
    sd = golden_state_dict(cfg)
    W = sd["bert.embedding.tokenizer.weight"]
    k = cfg["k"]
    site_mask = g["raw_mask"].astype(np.uint8)
    codes = g["panel"].astype(np.uint8)
    for h in ("h1", "h2"):
        tok = g["hap_1" if h == "h1" else "hap_2"]
        delta = knn_np.lut_delta(W, tok, None, site_mask)
        # the device-arithmetic restatement (f32, csrc/knn.hip order) agrees with the fp64 Delta
        d32 = knn_np.lut_delta_f32(W, tok, site_mask)
        np.testing.assert_allclose(d32, delta, rtol=1e-5, atol=1e-5 * np.abs(delta).max())
        for limbs in (1, 2):
            dq, e = knn_np.quantize_lut(delta, limbs)
            idx, d = knn_np.knn(codes, dq, k)
            np.testing.assert_array_equal(idx, g[f"Ican_{h}"])
            idx32, _ = knn_np.knn(codes, knn_np.quantize_lut(d32, limbs)[0], k)
            np.testing.assert_array_equal(idx32, g[f"Ican_{h}"])
        # tie-equivalence of the reference's own choice (exact fp64 distances)
        full = knn_np.distances(codes, np.rint(delta * 1.0).astype(np.int64))  # any linear map of delta
        ref_sorted = np.sort(np.take_along_axis(full, g[f"Iref_{h}"], 1), 1)
        can_sorted = np.sort(np.take_along_axis(full, g[f"Ican_{h}"], 1), 1)
        np.testing.assert_array_equal(ref_sorted, can_sorted)


def test_oracle_lut_f32_restatement_offsets_and_exponent():
    """oracle/lut_f32.c with query / panel AF offsets (the device's 16-lane lut_delta_kernel
    order) and a separate panel token table stays within f32 rounding of the fp64 Delta, and
    quantize_lut's exponent is the largest e with max|Delta| 2^e <= qmax (also at exact powers
    of two, where floor(log2) alone is on the edge)."""
    rng = np.random.default_rng(8)
    nq, L, S, D = 6, 1030, 257, 48
    W = rng.standard_normal((12, D)).astype(np.float32)
    Wp = (W + 0.1 * rng.standard_normal(W.shape)).astype(np.float32)
    tok = np.zeros((nq, L), np.int64)
    tok[:, 0], tok[:, S + 1] = 2, 3
    tok[:, 1:S + 1] = 5 + (rng.random((nq, S)) < 0.3)
    sm = (rng.random(S) < 0.25).astype(np.uint8)
    Aq = (0.3 * rng.standard_normal((3, L, D))).astype(np.float32)
    Ar = (0.3 * rng.standard_normal((L, D))).astype(np.float32)
    d32 = knn_np.lut_delta_f32(W, tok, sm, Aq=Aq, aq_period=3, Ar=Ar, Wp=Wp)
    u = W.astype(np.float64)[tok[:, 1:S + 1]] + (Aq[np.arange(nq) % 3] - Ar[None])[:, 1:S + 1]
    d64 = ((u - Wp[6].astype(np.float64)) ** 2).sum(-1) - ((u - Wp[5].astype(np.float64)) ** 2).sum(-1)
    d64[:, sm.astype(bool)] = 0
    np.testing.assert_allclose(d32, d64, rtol=1e-5, atol=1e-5 * np.abs(d64).max())
    assert (d32[:, sm.astype(bool)] == 0).all()
    for limbs in (1, 2):
        qmax = (1 << (7 * limbs)) - 1
        for m in (1.0, 0.5, 3.0, float(qmax), qmax / 1024.0, np.nextafter(np.float32(2.0), np.float32(0))):
            dl = np.array([[m, -m / 3, 0.0]])
            dq, e = knn_np.quantize_lut(dl, limbs)
            assert m * 2.0 ** e[0] <= qmax < m * 2.0 ** (e[0] + 1)
            assert abs(dq[0, 0]) <= qmax


def test_oracle_knn_tie_break_and_small_panels():
    rng = np.random.default_rng(3)
    codes = rng.integers(0, 2, (37, 70)).astype(np.uint8)
    codes[5] = codes[2]
    codes[11] = codes[2]                       # exact duplicates -> ties broken by index
    dq = rng.integers(-3, 4, (4, 70)).astype(np.int32)
    idx, d = knn_np.knn(codes, dq, 8, chunk=16)   # chunked path == single shot
    idx2, d2 = knn_np.topk_exact(knn_np.distances(codes, dq), 8)
    np.testing.assert_array_equal(idx, idx2)
    for q in range(4):
        assert list(zip(d[q], idx[q])) == sorted(zip(d[q], idx[q]))
    i3, d3 = knn_np.knn(codes[:5], dq, 8)      # N < k -> -1 padding
    assert (i3[:, 5:] == -1).all() and (i3[:, :5] >= 0).all()


def test_oracle_merge_partials():
    rng = np.random.default_rng(4)
    D = rng.integers(-50, 50, (3, 300))
    idx = np.arange(300)
    keys = knn_np.pack_key(D, np.broadcast_to(idx, D.shape))
    parts = np.stack([np.sort(keys[:, i * 100:(i + 1) * 100], 1)[:, :10] for i in range(3)])
    merged = knn_np.merge_partials(parts, 10)
    np.testing.assert_array_equal(merged, np.sort(keys, 1)[:, :10])


def test_data_contract_oracle():
    g = load_golden("data_contract")
    import json
    itos = json.loads(str(g["vocab_itos"]))
    stoi = {0: 5, 1: 6}
    assert itos[:7] == ["<pad>", "<unk>", "<sos>", "<eos>", "<mask>", "0", "1"]
    np.testing.assert_array_equal(data_np.tokenize(g["tok_seq"], g["tok_mask"], stoi), g["tok_out"])
    np.testing.assert_allclose(data_np.sequence_padding(data_np.position_normalize(g["pos_in"]), "float"),
                               g["pos_out"])
    for key in g:
        if key.startswith("mask_"):
            _, n, level, seed, w = key.split("_")
            rate = [0.30, 0.40, 0.50, 0.60, 0.70, 0.80][int(level)]
            np.testing.assert_array_equal(data_np.af_mask(g[f"af_{n}"], rate, int(seed), int(w)), g[key])


def test_infer_geometry_oracle_roundtrip():
    W, S, L, n_var = 3, 4, 1030, 2500
    win = 1020
    rng = np.random.default_rng(0)
    h = rng.random((W * S, L))
    gt = rng.random((W * S, L, 4))
    m = (rng.random((W * S, L)) < 0.5).astype(int)
    h1, h2, g2, m2 = data_np.infer_geometry(h, h, gt, m, W, n_var, win)
    assert h1.shape == (n_var, S) and g2.shape == (n_var, S, 4)
    # site j of window w for sample s sits at row w*win + j
    w, s, j = 1, 2, 17
    assert h1[w * win + j, s] == h[w * S + s, 1 + j]
