"""GPU parity of the individual HIP kernels (called through the C ABI).

Integer/index work is checked bit-exactly against the ORACLE; floating-point
kernels against a plain torch fp32 (float64 where stated) reference of the same op.
"""

import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import knn_np  # noqa: E402
from knn_helpers import decode_lut, lut_wide_flag, rand_case as _rand_case  # noqa: E402


def K():
    from src import kernels
    return kernels


def N():
    from src import native
    return native


DEV = "cuda"


def test_mfma_layout_selftest():
    assert K().selftest_mfma() == 0


# ---------------------------------------------------------------------- GEMM --
def _ref_linear(x, w, b, act, slope, r1=None, c1=None, r2=None, c2=None, resid=None):
    y = x.double() @ w.double().T
    if b is not None:
        y = y + b.double()
    if r1 is not None:
        y = y + r1.double()[:, None] * c1.double()[None]
    if r2 is not None:
        y = y + r2.double()[:, None] * c2.double()[None]
    if act == 1:
        y = torch.nn.functional.gelu(y)
    elif act == 2:
        y = torch.nn.functional.leaky_relu(y, slope)
    elif act == 3:
        y = torch.sigmoid(y)
    if resid is not None:
        y = y + resid.double()
    return y


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,Nn,Kk", [(1000, 384, 384), (257, 1152, 64), (130, 1536, 384), (64, 384, 1536), (3, 8, 8)])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_linear(dt, M, Nn, Kk, act):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + Nn + act)
    x = torch.randn(M, Kk, generator=g).to(DEV, dt)
    w = (torch.randn(Nn, Kk, generator=g) / math.sqrt(Kk)).to(DEV, dt)
    b = torch.randn(Nn, generator=g).to(DEV)
    period = max(1, M // 3)
    r1 = torch.randn(period, generator=g).to(DEV)
    c1 = torch.randn(Nn, generator=g).to(DEV)
    r2 = torch.randn(period * 2, generator=g).to(DEV)
    c2 = torch.randn(Nn, generator=g).to(DEV)
    resid = torch.randn(M, Nn, generator=g).to(DEV, dt)
    out = K().linear(x, w, b, act=act, slope=0.1, row1=(r1, 1, c1), row2=(r2, 2, c2), row_period=period,
                     resid=resid)
    rows = torch.arange(M, device=DEV) % period
    ref = _ref_linear(x.float(), w.float(), b, act, 0.1, r1[rows], c1, r2[rows * 2], c2, resid.float())
    tol = 2e-5 if dt == torch.float32 else 2e-2
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol * 4)


def test_linear_bf16_to_f32_and_plain():
    x = torch.randn(300, 256, device=DEV).to(torch.bfloat16)
    w = torch.randn(72, 256, device=DEV).to(torch.bfloat16)
    out = K().linear(x, w, out_dtype=torch.float32)
    torch.testing.assert_close(out.double(), x.double() @ w.double().T, rtol=1e-5, atol=1e-4)


# ------------------------------------------------------------------ layernorm --
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [16, 384, 1536])
def test_layernorm_with_residual_and_post(dt, n):
    M = 777
    x = torch.randn(M, n, device=DEV).to(dt)
    r = torch.randn(M, n, device=DEV).to(dt)
    gm, bt = torch.randn(n, device=DEV), torch.randn(n, device=DEV)
    ref = torch.nn.functional.layer_norm((x.float() + r.float()), (n,), gm, bt, 1e-5)
    out = K().layernorm(x, gm, bt, resid=r)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)
    # rag-fusion tail: base + scale * LN(x) * clamp(log1p(1/(maf+1e-6)), 3)
    af = torch.rand(M // 3 + 1, device=DEV)
    base = torch.randn(M, n, device=DEV).to(dt)
    out2 = K().layernorm(x, gm, bt, post_base=base, post_scale=0.37, post_af=af, af_period=af.numel(),
                         maf_weight=True, act=1)
    a = af[torch.arange(M, device=DEV) % af.numel()]
    maf = torch.minimum(a, 1 - a)
    mw = torch.log1p(1.0 / (maf + 1e-6)).clamp(max=3.0)
    y = torch.nn.functional.gelu(torch.nn.functional.layer_norm(x.float(), (n,), gm, bt, 1e-5))
    torch.testing.assert_close(out2.float(), base.float() + 0.37 * y * mw[:, None], rtol=tol, atol=tol * 2)


# ------------------------------------------------------------------ attention --
def _ref_attn(qkv, nseq, L, H, dh):
    q, k, v = qkv.double().view(nseq, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    o = torch.softmax(s, -1) @ v
    return o.permute(0, 2, 1, 3).reshape(nseq * L, H * dh)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nseq,L,H,dh", [(2, 1030, 12, 32), (3, 70, 4, 16), (1, 130, 8, 48), (2, 257, 6, 64)])
def test_attention(dt, nseq, L, H, dh):
    qkv = (torch.randn(nseq * L, 3 * H * dh, device=DEV) * 1.5).to(dt)
    out = K().attention(qkv, nseq, L, H, dh)
    ref = _ref_attn(qkv.float(), nseq, L, H, dh)
    tol = 2e-5 if dt == torch.float32 else 2e-2
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol)


# ------------------------------------------------------------------------ kNN --
@pytest.mark.parametrize("n_ref,n_sites,nq,k,limbs,tie", [
    (5000, 300, 20, 8, 2, False), (4099, 1020, 48, 32, 2, True), (3000, 512, 64, 32, 1, True),
    (777, 1028, 70, 4, 2, False), (10, 200, 5, 32, 2, False), (33, 64, 17, 1, 1, True)])
def test_knn_bit_exact_vs_oracle(n_ref, n_sites, nq, k, limbs, tie):
    from src.retrieval import PanelIndex
    W, panel, site_mask, tok = _rand_case(n_ref, n_sites, nq, n_ref + nq, tie)
    idx_t = PanelIndex.from_alleles(panel, np.zeros(1030, np.float32), DEV)
    Wt = torch.from_numpy(W).to(DEV)
    smask = torch.from_numpy(site_mask).to(DEV)
    idx, dist, keys, lut, exps = idx_t.search(torch.from_numpy(tok).to(DEV), Wt, smask, k, limbs=limbs,
                                              return_keys=True)
    # LUT == the oracle's quantisation of Delta computed in the device's f32 arithmetic
    # (oracle/lut_f32.c), bit for bit; within one quantum of the fp64 Delta's
    dq_o, e_o = knn_np.quantize_lut(knn_np.lut_delta_f32(W, tok, site_mask), limbs)
    dq_g = decode_lut(lut, nq, idx_t.n_sites_pad, limbs)
    np.testing.assert_array_equal(exps.cpu().numpy(), e_o)
    np.testing.assert_array_equal(dq_g[:, :n_sites], dq_o)
    assert np.abs(knn_np.quantize_lut(knn_np.lut_delta(W, tok, None, site_mask), limbs)[0] - dq_o).max() <= 1
    assert (dq_g[:, n_sites:] == 0).all()
    # scan + merge bit-exact against the oracle's own LUT -> top-k
    oi, od = knn_np.knn(panel, dq_o, k)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    kk = keys.cpu().numpy().view(np.uint64)
    valid = oi >= 0
    np.testing.assert_array_equal(kk[valid], knn_np.pack_key(od, oi)[valid])
    if limbs == 2:
        # binary Delta (aligned masks) reduces to the one-limb scan; either way the keys
        # equal the forced two-limb scan's
        assert lut_wide_flag(lut, nq, idx_t.n_sites_pad) == (0 if tie else 1)
        from src import kernels as K_
        with K_.option("knn_no_reduce", 1):
            keys2 = idx_t.scan_keys(lut, nq, 2, k)
        torch.testing.assert_close(keys2, keys, rtol=0, atol=0)


@pytest.mark.parametrize("tie", [False, True])
def test_knn_presample_threshold_is_exact(tie):
    """Threshold pre-pass over a panel prefix, then the full scan from that threshold:
    keys identical to the plain scan and to the oracle (also with massive distance ties)."""
    from src.retrieval import PanelIndex
    n_ref, n_sites, nq, k = 40000, 300, 40, 32
    W, panel, site_mask, tok = _rand_case(n_ref, n_sites, nq, 77, tie)
    idx_t = PanelIndex.from_alleles(panel, np.zeros(1030, np.float32), DEV)
    Wt, smask = torch.from_numpy(W).to(DEV), torch.from_numpy(site_mask).to(DEV)
    lut, _, _ = idx_t.lut(torch.from_numpy(tok).to(DEV), Wt, smask, 2)
    plain = idx_t.scan_keys(lut, nq, 2, k, presample=False)
    pre = idx_t.scan_keys(lut, nq, 2, k, presample=True)
    torch.testing.assert_close(pre, plain, rtol=0, atol=0)
    dq = decode_lut(lut, nq, idx_t.n_sites_pad, 2)[:, :n_sites]
    oi, od = knn_np.knn(panel, dq, k)
    np.testing.assert_array_equal(pre.cpu().numpy().view(np.uint64), knn_np.pack_key(od, oi))


def test_knn_shard_offsets_and_merge():
    """Panel split in 3 contiguous shards with global offsets + merge == unsplit search."""
    from src.retrieval import PanelIndex
    W, panel, site_mask, tok = _rand_case(3001, 400, 24, 5, True)
    Wt, smask, tq = torch.from_numpy(W).to(DEV), torch.from_numpy(site_mask).to(DEV), torch.from_numpy(tok).to(DEV)
    full = PanelIndex.from_alleles(panel, np.zeros(1030, np.float32), DEV)
    _, _, keys_full, lut, _ = full.search(tq, Wt, smask, 16, return_keys=True)
    bounds = [0, 1000, 2100, 3001]
    parts = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        sh = PanelIndex.from_alleles(panel[a:b], np.zeros(1030, np.float32), DEV, ref_offset=a)
        parts.append(sh.scan_keys(lut, 24, 2, 16))
    merged = K().topk_merge(torch.stack(parts), 16)
    torch.testing.assert_close(merged, keys_full, rtol=0, atol=0)


def test_panel_synth_matches_hash_restatement():
    from src.dataset.synthetic import hash_uniform
    af = torch.rand(300, device=DEV) * 0.5
    codes = K().panel_synth(257, 300, af, seed=11)
    r, c = np.meshgrid(np.arange(257), np.arange(300), indexing="ij")
    exp = (hash_uniform(11, r, c) < af.cpu().numpy().astype(np.float64)[None]).astype(np.uint8)
    np.testing.assert_array_equal(codes[:, :300].cpu().numpy(), exp)
    assert (codes[:, 300:] == 0).all()


@pytest.mark.parametrize("nq,k", [(6, 8), (37, 32)])
def test_rag_mean_vs_oracle(nq, k):
    rng = np.random.default_rng(9)
    D, L, n_sites, n_ref = 64, 1030, 500, 200
    W = rng.standard_normal((12, D)).astype(np.float32)
    pe = rng.standard_normal((L, D)).astype(np.float32)
    Ar = rng.standard_normal((L, D)).astype(np.float32)
    panel = rng.integers(0, 2, (n_ref, n_sites)).astype(np.uint8)
    idx = rng.integers(0, n_ref, (nq, k))
    idx[5, 3:] = -1                                    # missing neighbours are skipped
    idx[nq - 1, :] = -1                                # no neighbour at all: site rows are zero
    from src.retrieval import PanelIndex
    pi = PanelIndex.from_alleles(panel, np.zeros(L, np.float32), DEV)
    out = K().rag_mean(torch.from_numpy(idx).to(DEV), pi.codes, n_sites, torch.from_numpy(W).to(DEV),
                       torch.from_numpy(pe).to(DEV), torch.from_numpy(Ar).to(DEV), L, torch.float32)
    toks = np.zeros((n_ref, L), np.int64)
    toks[:, 0], toks[:, 1:1 + n_sites], toks[:, 1 + n_sites] = 2, 5 + panel, 3
    ref = np.zeros((nq, L, D), np.float32)
    for q in range(nq):
        v = idx[q][idx[q] >= 0]
        if len(v):
            ref[q] = (W[toks[v]] + pe[None] + Ar[None]).mean(0)
        else:
            ref[q] = W[toks[0]] + pe + Ar
            ref[q, 1:1 + n_sites] = pe[1:1 + n_sites] + Ar[1:1 + n_sites]
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


# ------------------------------------------------- fused row-panel GEMM epilogues --
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [384, 128, 64])
def test_linear_fused_layernorm_and_tail(dt, n):
    g = torch.Generator(device="cpu").manual_seed(n)
    M, Kk = 1000, 384
    x = torch.randn(M, Kk, generator=g).to(DEV, dt)
    w = (torch.randn(n, Kk, generator=g) / math.sqrt(Kk)).to(DEV, dt)
    b, gm, bt = (torch.randn(n, generator=g).to(DEV) for _ in range(3))
    resid = torch.randn(M, n, generator=g).to(DEV, dt)
    base = torch.randn(M, n, generator=g).to(DEV, dt)
    af = torch.rand(M // 2, generator=g).to(DEV)
    out = K().linear(x, w, b, act=2, slope=0.1, resid=resid, ln=(gm, bt), ln_act=1, post_base=base,
                     post_scale=0.3, post_af=af, post_af_period=M // 2, post_maf=True)
    v = _ref_linear(x.float(), w.float(), b, 2, 0.1, resid=resid.float())
    y = torch.nn.functional.gelu(torch.nn.functional.layer_norm(v, (n,), gm.double(), bt.double(), 1e-5))
    a = af[torch.arange(M, device=DEV) % (M // 2)].double()
    mw = torch.log1p(1.0 / (torch.minimum(a, 1 - a) + 1e-6)).clamp(max=3.0)
    ref = base.double() + 0.3 * y * mw[:, None]
    tol = 1e-4 if dt == torch.float32 else 3e-2
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_linear_stats_then_rownorm_matches_ffn(dt):
    """h = lrelu(x W1 + b1) with row stats -> out = lrelu(LN(h) W2 + b2) with the LN folded into
    the second GEMM (W2 diag(g), bias W2 b + b2, c1 = W2 g): FeedForward of feed_forward.py."""
    g = torch.Generator(device="cpu").manual_seed(1)
    M, D = 777, 384
    x = torch.randn(M, D, generator=g).to(DEV, dt)
    w1 = (torch.randn(4 * D, D, generator=g) / math.sqrt(D)).to(DEV, dt)
    w2 = (torch.randn(D, 4 * D, generator=g) / math.sqrt(4 * D)).to(DEV, dt)
    b1, b2 = torch.randn(4 * D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    gf, bf = torch.randn(4 * D, generator=g).to(DEV), torch.randn(4 * D, generator=g).to(DEV)
    parts = K().stat_tiles(4 * D)
    stats = torch.empty(parts, M, 2, device=DEV)
    h = K().linear(x, w1, b1, act=2, slope=0.1, stats_out=stats)
    hr = h.double()
    # stats are taken from the f32 accumulators, before the output is rounded to dt
    st_tol = 1e-4 if dt == torch.float32 else 2e-3
    torch.testing.assert_close(stats.sum(0)[:, 0].double(), hr.sum(1), rtol=st_tol, atol=st_tol * 100)
    w2g, b2g, c1 = K().fold_layernorm(w2.float(), b2, gf, bf, dt)
    out = K().linear(h, w2g, b2g, act=2, slope=0.1, rownorm=(stats, parts, 4 * D, c1))
    hn = torch.nn.functional.layer_norm(hr, (4 * D,), gf.double(), bf.double(), 1e-5)
    ref = torch.nn.functional.leaky_relu(hn @ w2.double().T + b2.double(), 0.1)
    tol = 1e-4 if dt == torch.float32 else 5e-2
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("D,M", [(384, 777), (384, 128 * 3), (128, 300), (256, 1), (256, 129),
                                 (384, 4 * 1030 + 5), (384, 64 * 1030)])
def test_tail32_kernel(D, M):
    """32x32-MFMA block tail (csrc/tail.hip, the engine's default bf16 path): both entry points
    (snvrag_tail_forward = W_o' + LN1 + FFN + LN2 in place; snvrag_tail_ffn_forward = FFN + LN2)
    vs float64 torch on the same bf16 operands.  Ragged M
    (row tails of 1, 1 + 128 k, 5) and 515 workgroups (every chunk rotation of the stream)."""
    g = torch.Generator(device="cpu").manual_seed(7 * D + M)
    bf, F = torch.bfloat16, torch.nn.functional
    x = torch.randn(M, D, generator=g).to(DEV, bf)
    att = (0.5 * torch.randn(M, D, generator=g)).to(DEV, bf)
    w_o = (torch.randn(D, D, generator=g) / math.sqrt(D)).to(DEV, bf)
    b_o = (0.1 * torch.randn(D, generator=g)).to(DEV)
    g1, be1 = (1 + 0.2 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    w1 = (torch.randn(4 * D, D, generator=g) / math.sqrt(D)).to(DEV, bf)
    w2 = (torch.randn(D, 4 * D, generator=g) / math.sqrt(4 * D)).to(DEV)
    b1, b2 = torch.randn(4 * D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    gf, bff = (1 + 0.2 * torch.randn(4 * D, generator=g)).to(DEV), (0.1 * torch.randn(4 * D, generator=g)).to(DEV)
    g2, be2 = (1 + 0.2 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    w2g, b2g, _ = K().fold_layernorm(w2, b2, gf, bff, bf)
    vec = K().ffn_vec(b1, b2g, w2g, g2, be2)
    ts = K().tail_pack(w_o, w1, w2g)

    def ffn_ref(x1):
        h = F.leaky_relu(x1 @ w1.double().T + b1.double(), 0.1)
        hn = F.layer_norm(h, (4 * D,), gf.double(), bff.double(), 1e-5)
        f = F.leaky_relu(hn @ w2.double().T + b2.double(), 0.1)
        return F.layer_norm(x1 + f, (D,), g2.double(), be2.double(), 1e-5)

    x1 = F.layer_norm(x.double() + att.double() @ w_o.double().T + b_o.double(), (D,), g1.double(), be1.double(), 1e-5)
    ref = ffn_ref(x1)
    # FFN-only entry on the same x (not in place)
    o2 = K().tail_ffn_forward(x, ts, vec)
    r2 = ffn_ref(x.double())
    torch.testing.assert_close(o2.double(), r2, rtol=5e-2, atol=5e-2)
    assert (o2.double() - r2).abs().mean() < 1e-2
    out = K().tail_forward(att, x, ts, b_o, g1, be1, vec)
    assert out.data_ptr() == x.data_ptr()
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.double(), ref, rtol=5e-2, atol=5e-2)
    assert (out.double() - ref).abs().mean() < 1e-2


@pytest.mark.parametrize("M", [777, 128 * 3, 1, 4 * 1030 + 5, 64 * 1030, 294 * 128 - 51])
def test_tail_wide_kernel(M):
    """Wide-row block tail (csrc/tailw.hip, option tail_wide: wave w owns features 96w..96w+95 and
    hidden chunks 4c + w, its weight fragments loaded straight into its registers; att / x1 and the
    hidden of a round are the LDS-resident operands) vs float64 torch with test_tail32_kernel's bar,
    in place; and close to tail_kernel on the same operands (the same function; the accumulation
    order of the bias and of the cross-wave row statistics differs).  Ragged M: 777, one row, a
    partial last tile, 515 and 294 tiles (the last partial round split into 32-row workgroups:
    bit-identical to the unsplit launch)."""
    D = 384
    g = torch.Generator(device="cpu").manual_seed(11 * M + 3)
    bf, F = torch.bfloat16, torch.nn.functional
    x = torch.randn(M, D, generator=g).to(DEV, bf)
    att = (0.5 * torch.randn(M, D, generator=g)).to(DEV, bf)
    w_o = (torch.randn(D, D, generator=g) / math.sqrt(D)).to(DEV, bf)
    b_o = (0.1 * torch.randn(D, generator=g)).to(DEV)
    g1, be1 = (1 + 0.2 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    w1 = (torch.randn(4 * D, D, generator=g) / math.sqrt(D)).to(DEV, bf)
    w2 = (torch.randn(D, 4 * D, generator=g) / math.sqrt(4 * D)).to(DEV)
    b1, b2 = torch.randn(4 * D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    gf, bff = (1 + 0.2 * torch.randn(4 * D, generator=g)).to(DEV), (0.1 * torch.randn(4 * D, generator=g)).to(DEV)
    g2, be2 = (1 + 0.2 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    w2g, b2g, _ = K().fold_layernorm(w2, b2, gf, bff, bf)
    vec = K().ffn_vec(b1, b2g, w2g, g2, be2)
    ts = K().tail_pack(w_o, w1, w2g)
    x1 = F.layer_norm(x.double() + att.double() @ w_o.double().T + b_o.double(), (D,), g1.double(), be1.double(), 1e-5)
    h = F.leaky_relu(x1 @ w1.double().T + b1.double(), 0.1)
    hn = F.layer_norm(h, (4 * D,), gf.double(), bff.double(), 1e-5)
    f = F.leaky_relu(hn @ w2.double().T + b2.double(), 0.1)
    ref = F.layer_norm(x1 + f, (D,), g2.double(), be2.double(), 1e-5)
    ya, yb = x.clone(), x.clone()
    with K().option("tail_wide", 1):
        out = K().tail_forward(att, ya, ts, b_o, g1, be1, vec)
    assert out.data_ptr() == ya.data_ptr()
    with K().option("tail_wide", 0):
        K().tail_forward(att, yb, ts, b_o, g1, be1, vec)
    assert torch.isfinite(ya.float()).all()
    torch.testing.assert_close(ya.double(), ref, rtol=5e-2, atol=5e-2)
    if M > 256 * 128:
        # the last partial round as 32-row workgroups (option tail_split; 64 x 1030: 12 of them,
        # 294 x 128 - 51: 151, the last ragged) computes every row exactly as a 128-row tile does
        yc = x.clone()
        with K().option("tail_wide", 1), K().option("tail_split", 0):
            K().tail_forward(att, yc, ts, b_o, g1, be1, vec)
        torch.testing.assert_close(yc, ya, rtol=0, atol=0)
    ea, eb = (ya.double() - ref).abs().mean(), (yb.double() - ref).abs().mean()
    assert ea < 1e-2 and ea < 1.25 * eb + 1e-4, (float(ea), float(eb))
    # vs tail_kernel: the hidden is rounded to bf16 in both, from differently ordered f32 sums, so
    # a hidden unit may land one bf16 step apart and move outputs by a few steps; measured at the
    # bench shape: max 0.031, mean 4e-6, 0.2 % of the outputs differ
    d = (ya.float() - yb.float()).abs()
    assert float(d.max()) <= 0.0625 and float(d.mean()) < 1e-4, (float(d.max()), float(d.mean()))
    assert int((d > 0).sum()) <= max(16, d.numel() // 50), int((d > 0).sum())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_encoder_fused_equals_unfused(dt, monkeypatch):
    """Encoder stack with LN fused into GEMM epilogues/prologues == the 8-launch unfused stack."""
    import os
    from src.model import build_model
    from src.engine import engine_for
    torch.manual_seed(0)
    m = build_model(12, 384, 2, 12).to(DEV).eval()
    eng = engine_for(m)
    eng.set_dtype(dt)
    P = eng.packed()
    x0 = torch.randn(3, 1030, 384, device=DEV).to(dt)
    ws = torch.empty(K().encoder_ws_bytes(dt, 3, 1030, 384, 12), device=DEV, dtype=torch.uint8)
    a = x0.clone()
    K().encoder_forward(a, P.layers, 12, ws)
    b = x0.clone()
    with K().option("unfused_ln", 1):
        K().encoder_forward(b, P.layers, 12, ws)
    tol = 2e-4 if dt == torch.float32 else 6e-2
    torch.testing.assert_close(a.float(), b.float(), rtol=tol, atol=tol)


def _attn_ref(qkv, nseq, L, H, dh):
    q, k, v = qkv.float().view(nseq, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    p = torch.softmax(q @ k.transpose(-1, -2) / dh ** 0.5, -1)
    return (p @ v).permute(0, 2, 1, 3).reshape(nseq * L, H * dh)


@pytest.mark.parametrize("L", [1030, 64, 77, 16, 5])
def test_attention_dh32_bf16_fixed_shift(L):
    """bf16 dh=32 kernel (fixed per-query shift + ones-MFMA row sums) vs fp32 softmax;
    L covers full tiles, a 1-key..48-key tail and L < one tile."""
    torch.manual_seed(L)
    nseq, H, dh = 3, 4, 32
    qkv = (torch.randn(nseq * L, 3 * H * dh, device=DEV) * 1.5).to(torch.bfloat16)
    K().attention_fallbacks(True)
    out = K().attention(qkv, nseq, L, H, dh)
    ref = _attn_ref(qkv, nseq, L, H, dh)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    assert K().attention_fallbacks(True) == 0


def test_attention_dh32_overflow_takes_exact_fallback():
    """Scores far above the first key tile's max overflow the fixed shift: the affected
    waves must recompute with the online-max path and still match."""
    torch.manual_seed(1)
    nseq, L, H, dh = 2, 300, 2, 32
    qkv = torch.randn(nseq * L, 3 * H * dh, device=DEV) * 0.1
    D = H * dh
    qkv[:, :D] = 4.0                       # |q| large
    qkv[200, D:2 * D] = 8.0                # one key (seq 0, position 200) with a huge score
    qkv = qkv.to(torch.bfloat16)
    K().attention_fallbacks(True)
    out = K().attention(qkv, nseq, L, H, dh)
    ref = _attn_ref(qkv, nseq, L, H, dh)
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    assert K().attention_fallbacks(True) > 0


@pytest.mark.parametrize("M,N,Kd,mode", [(1000, 1152, 384, "plain"), (517, 1536, 384, "gelu"), (77, 512, 128, "gelu"),
                                        (300, 64, 256, "plain"), (900, 1536, 384, "rank_gelu"),
                                        (1203, 384, 384, "rank_lrelu_ln"), (260, 128, 128, "rank_lrelu_ln"),
                                        (129, 256, 256, "lrelu_ln"), (4133, 1536, 384, "head2"),
                                        (1, 1024, 256, "head2"), (130, 512, 128, "head2"), (999, 1536, 768, "gelu")])
def test_stream_gemm(M, N, Kd, mode):
    """snvrag_sgemm_forward (csrc/sgemm.hip: tile-major weight stream, tile epilogues under the next
    tiles' MFMAs) vs torch fp32 on the same bf16 operands; ragged M, 1..3 pairs per slab cycle,
    the rotated pair order (blockIdx % pairs) and the three epilogues."""
    from src import native as NN
    g = torch.Generator(device="cpu").manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g) / math.sqrt(Kd)).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    ws = K().sgemm_pack(w)
    ref = x.float() @ w.float().t() + b
    rank, c = None, (None, None)
    if mode.startswith("rank"):
        period = (M + 2) // 3
        r1, r2 = torch.rand(period, generator=g).to(DEV), torch.rand(period, generator=g).to(DEV)
        c = (torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV))
        ri = torch.arange(M, device=DEV) % period
        ref = ref + r1[ri, None] * c[0][None] + r2[ri, None] * c[1][None]
        rank = (r1, r2, period)
    if mode == "head2":
        w2 = (torch.randn(2, N, generator=g) / math.sqrt(N)).to(DEV)
        b2 = torch.randn(2, generator=g).to(DEV)
        ref_l = torch.nn.functional.gelu(ref) @ w2.t() + b2
        logits, probs = K().sgemm(x, ws, N, K().sgemm_vec(b, head=(w2, b2)), epi=K().SG_HEAD2, act=NN.ACT_GELU,
                                  want_logits=True)
        torch.testing.assert_close(logits, ref_l, rtol=1e-3, atol=2e-3)
        torch.testing.assert_close(probs, torch.softmax(ref_l, -1), rtol=1e-3, atol=1e-3)
        return
    if mode.endswith("ln"):
        gm, bt = torch.rand(N, generator=g).to(DEV) + 0.5, torch.randn(N, generator=g).to(DEV)
        ref = torch.nn.functional.layer_norm(torch.nn.functional.leaky_relu(ref, 0.1) + x.float(), (N,), gm, bt, 1e-5)
        out = K().sgemm(x, ws, N, K().sgemm_vec(b, *c, ln=(gm, bt)), epi=K().SG_LN, act=NN.ACT_LRELU, slope=0.1,
                        rank=rank)
    else:
        act = NN.ACT_GELU if "gelu" in mode else NN.ACT_NONE
        if act == NN.ACT_GELU:
            ref = torch.nn.functional.gelu(ref)
        out = K().sgemm(x, ws, N, K().sgemm_vec(b, *c), act=act, rank=rank)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("M,mode", [(1000, "sigmoid"), (4133, "rank_ln"), (77, "ln"), (300, "rank_sigmoid")])
def test_fused_mlp(M, mode):
    """snvrag_mlp_forward (two projections, the 4D hidden on chip: af_adapter / af_fusion) vs torch fp32 of
    the same bf16 weights, with the hidden rounded to bf16 as the kernel's phase-2 operand is."""
    from src import native as NN  # noqa: F401
    g = torch.Generator(device="cpu").manual_seed(M)
    D, H = 384, 1536
    x = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
    w1 = (torch.randn(H, D, generator=g) / math.sqrt(D)).to(DEV, torch.bfloat16)
    w2 = (torch.randn(D, H, generator=g) / math.sqrt(H)).to(DEV, torch.bfloat16)
    b1, b2 = torch.randn(H, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    parts, rank = [b1], None
    h = x.float() @ w1.float().t() + b1
    if mode.startswith("rank"):
        period = (M + 2) // 3
        r1, r2 = torch.rand(period, generator=g).to(DEV), torch.rand(period, generator=g).to(DEV)
        c1, c2 = torch.randn(H, generator=g).to(DEV), torch.randn(H, generator=g).to(DEV)
        ri = torch.arange(M, device=DEV) % period
        h = h + r1[ri, None] * c1[None] + r2[ri, None] * c2[None]
        parts += [c1, c2]
        rank = (r1, r2, period)
    h = torch.nn.functional.gelu(h).to(torch.bfloat16).float()
    y = h @ w2.float().t() + b2
    parts.append(b2)
    if mode.endswith("ln"):
        gm, bt = torch.rand(D, generator=g).to(DEV) + 0.5, torch.randn(D, generator=g).to(DEV)
        ref = torch.nn.functional.layer_norm(y, (D,), gm, bt, 1e-5)
        parts += [gm, bt]
        epi2 = 1
    else:
        ref = torch.sigmoid(y)
        epi2 = 0
    vec = torch.cat([t.float().reshape(-1) for t in parts]).contiguous()
    out = K().mlp(x, K().mlp_pack(w1, w2), vec, epi2=epi2, rank=rank)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("M", [1030, 77, 1])
def test_mlp_afgate_vs_fp32_and_two_launch_path(M):
    """snvrag_mlp_afgate_forward (CrossAFInteraction computed in the af_adapter MLP's prologue:
    fusion.py:82-86 then :135-138 in one launch) vs torch fp32 of the same chain (the gate input
    rounded to bf16 where the two-launch path stores it) and vs snvrag_af_gate + snvrag_mlp_forward."""
    g = torch.Generator(device="cpu").manual_seed(M)
    D, H = 384, 1536
    rn = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(DEV)
    ag = [rn(32, 2, sc=0.8), rn(32, sc=0.1), rn(D, 32, sc=0.25), rn(D, sc=0.1), rn(D, 2, sc=0.7), rn(D, sc=0.1),
          1 + rn(D, sc=0.1), rn(D, sc=0.1)]
    rs = 0.37
    af, afp = torch.rand(M, generator=g).to(DEV), torch.rand(M, generator=g).to(DEV)
    af[:2], afp[:2] = torch.tensor([0.0, 1.0])[:M], torch.tensor([1e-4, 0.5])[:M]
    w1 = (torch.randn(H, D, generator=g) / math.sqrt(D)).to(DEV, torch.bfloat16)
    w2 = (torch.randn(D, H, generator=g) / math.sqrt(H)).to(DEV, torch.bfloat16)
    b1, b2 = rn(H), rn(D, sc=0.1)
    mv = torch.cat([b1, b2]).contiguous()
    ws = K().mlp_pack(w1, w2)
    # torch fp32 reference
    c = torch.stack([af, afp], -1)
    gate = torch.sigmoid(torch.nn.functional.gelu(c @ ag[0].t() + ag[1]) @ ag[2].t() + ag[3])
    enc = torch.nn.functional.gelu(torch.nn.functional.layer_norm(c @ ag[4].t() + ag[5], (D,), ag[6], ag[7], 1e-5))
    fa = (af[:, None] + rs * gate * enc).to(torch.bfloat16).float()
    h = torch.nn.functional.gelu(fa @ w1.float().t() + b1).to(torch.bfloat16).float()
    ref = torch.sigmoid(h @ w2.float().t() + b2)
    frags, vec = K().mlp_afgate_pack(ag, mv)
    out = K().mlp_afgate(af, afp, frags, rs, ws, vec)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=2e-2)
    # the fused gate input against the af_gate kernel's (both bf16): a rare one-ulp rounding flip
    from src import native as NN
    w = NN.AfGateW(*[t.contiguous().data_ptr() for t in ag], rs)
    fa2 = K().af_gate(af, afp, w, D, torch.bfloat16)
    torch.testing.assert_close(fa2.float(), fa, rtol=1e-2, atol=1e-2)
    two = K().mlp(fa2.view(M, D), ws, mv, epi2=0)
    torch.testing.assert_close(out.float(), two.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,period", [(1000, 1000), (2060, 1030), (77, 33)])
def test_stream_gemm_concatenated_input(M, period):
    """snvrag_sgemm_cat_forward (rag fusion: cat(h, aw * h_rag) -> Linear(2D, 4D) -> GELU, the cat built
    in registers) == rag_concat + the stream GEMM on the materialised cat (bit-identical: the same
    bf16 rounding of aw * h_rag, the same weight stream) and vs torch fp32."""
    from src import native as NN
    g = torch.Generator(device="cpu").manual_seed(M + period)
    D, N = 384, 1536
    q = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
    r = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
    aw = torch.rand(period, D, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, 2 * D, generator=g) / math.sqrt(2 * D)).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    ws, vec = K().sgemm_pack(w), K().sgemm_vec(b)
    out = K().sgemm_cat(q, r, aw, period, ws, N, vec)
    cat = K().rag_concat(q, r, aw, period)
    ref = K().sgemm(cat, ws, N, vec, act=NN.ACT_GELU)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    ref32 = torch.nn.functional.gelu(cat.float() @ w.float().t() + b)
    torch.testing.assert_close(out.float(), ref32, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("n,bits,k,nq", [(5008, 2040, 32, 37), (300, 33, 5, 3), (20, 1020, 32, 4)])
def test_raw_genotype_index_vs_oracle(n, bits, k, nq):
    """Raw-genotype window index (csrc/rawdb.hip + topk_merge; build_ref_db_l2.py:86-89 IndexFlatL2
    semantics): exact (D, row) top-k vs the oracle, incl. duplicated rows (ties), a panel smaller
    than k (faiss pads with -1) and a row width that is not a multiple of 32 bits."""
    from oracle import knn_np
    from src.retrieval.raw_index import RawGenotypeIndex, pack_rows
    rng = np.random.default_rng(n + bits)
    R = (rng.random((n, bits)) < 0.2).astype(np.uint8)
    if n > 40:
        R[17] = R[5]
    Q = np.concatenate([R[[5]], (rng.random((nq - 1, bits)) < 0.2).astype(np.uint8)])
    idx = RawGenotypeIndex(pack_rows(R), bits, DEV)
    D, I = idx.search(Q, k)
    oi, od = knn_np.raw_genotype_knn(R, Q, k)
    kk = min(k, n)
    np.testing.assert_array_equal(I[:, :kk], oi[:, :kk])
    np.testing.assert_array_equal(D[:, :kk], od[:, :kk].astype(np.float32))
    if n < k:
        assert (I[:, n:] == -1).all() and np.isinf(D[:, n:]).all()


@pytest.mark.parametrize("wide", [1, 0])
@pytest.mark.parametrize("D,M,NC", [(384, 777, 3), (384, 128 * 4, 3), (128, 300, 3), (256, 1, 1), (384, 64 * 1030 + 3, 3),
                                    (384, 1, 1)])
def test_proj_kernel_vs_fp64(D, M, NC, wide):
    """Projection (multi_head_attention.py:44-46) on the wide-row kernel (csrc/tailw.hip projw_kernel,
    option proj_wide = 1: the engine's QKV path at D = 384) and on the 32x32 stream kernel (csrc/tail.hip
    PROJ mode, proj_wide = 0; D 128 / 256 always): x W^T + b vs float64 torch on the same bf16 operands,
    ragged M (rows >= M are dropped by the bounds-checked stores), every chunk rotation."""
    g = torch.Generator(device="cpu").manual_seed(D + M + NC)
    x = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(NC * D, D, generator=g) / math.sqrt(D)).to(DEV, torch.bfloat16)
    b = torch.randn(NC * D, generator=g).to(DEV)
    out = torch.full((M + 1, NC * D), 7.0, device=DEV, dtype=torch.bfloat16)
    with K().option("proj_wide", wide):
        K().proj_forward(x, K().proj_pack(w), b, NC, out=out[:M])
    ref = x.double() @ w.double().T + b.double()
    torch.testing.assert_close(out[:M].double(), ref, rtol=2e-2, atol=2e-2)
    assert (out[M] == 7.0).all()                       # nothing written past the last row


@pytest.mark.parametrize("L", [1030, 520, 77])
def test_attention_dh32_variants_bit_identical(L):
    """The inference attention kernel's A/B variants (option attn_variant: 1/2 s_setprio around the
    MFMA blocks, 3 the next tile's K read ahead, 4 eight-wave workgroups sharing each K/V tile, 5 the
    V fragments read before the exps) run
    the same arithmetic in the same order: bit-identical to variant 0 (prescaled Q, the engine's
    form), and variant 0 matches the fp32 softmax."""
    import math
    torch.manual_seed(L + 5)
    nseq, H, dh = 3, 12, 32
    qkv = (torch.randn(nseq * L, 3 * H * dh, device=DEV) * 0.8)
    qkv[:, :H * dh] *= math.log2(math.e) / math.sqrt(dh)
    qkv = qkv.to(torch.bfloat16)
    scale = 1.0 / math.log2(math.e)                     # Q carries log2(e)/sqrt(dh)
    outs = {}
    for v in (0, 1, 2, 3, 4, 5):
        with K().option("attn_variant", v):
            outs[v] = K().attention(qkv, nseq, L, H, dh, scale=scale)
    q = qkv.float().clone()
    q[:, :H * dh] *= math.sqrt(dh) / math.log2(math.e)
    ref = _attn_ref(q, nseq, L, H, dh)
    torch.testing.assert_close(outs[0].float(), ref, rtol=2e-2, atol=2e-2)
    for v in (1, 2, 3, 4, 5):
        assert torch.equal(outs[v], outs[0]), v


@pytest.mark.parametrize("M", [1, 777, 128 * 256 + 5, 64 * 1030])
def test_tail_persistent_equals_tail_kernel(M):
    """The persistent block tail (tailp_kernel: one workgroup per CU over 128-row tiles, the
    activations streamed into the weight ring; option tail_persist) == tail_kernel to one bf16
    rounding step on at most 0.1 % of the outputs (the same arithmetic), in place, and the default
    tail_kernel (8 fragments read ahead) == its 4-fragment variant bit for bit, incl. a ragged last tile, a single partial tile
    and 515 tiles (two per workgroup for most CUs, every chunk rotation)."""
    D = 384
    g = torch.Generator(device="cpu").manual_seed(M)
    bf = torch.bfloat16
    x = torch.randn(M, D, generator=g).to(DEV, bf)
    att = (0.5 * torch.randn(M, D, generator=g)).to(DEV, bf)
    w_o = (torch.randn(D, D, generator=g) / math.sqrt(D)).to(DEV, bf)
    b_o = (0.1 * torch.randn(D, generator=g)).to(DEV)
    g1, be1 = (1 + 0.2 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    w1 = (torch.randn(4 * D, D, generator=g) / math.sqrt(D)).to(DEV, bf)
    w2 = (torch.randn(D, 4 * D, generator=g) / math.sqrt(4 * D)).to(DEV)
    b1, b2 = torch.randn(4 * D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    gf, bff = (1 + 0.2 * torch.randn(4 * D, generator=g)).to(DEV), (0.1 * torch.randn(4 * D, generator=g)).to(DEV)
    g2, be2 = (1 + 0.2 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    w2g, b2g, _ = K().fold_layernorm(w2, b2, gf, bff, bf)
    vec = K().ffn_vec(b1, b2g, w2g, g2, be2)
    ts = K().tail_pack(w_o, w1, w2g)
    ya, yb, yc = x.clone(), x.clone(), x.clone()
    with K().option("tail_wide", 0):                     # (the engine's default is the wide-row tail)
        with K().option("tail_persist", 1):
            K().tail_forward(att, ya, ts, b_o, g1, be1, vec)
        K().tail_forward(att, yb, ts, b_o, g1, be1, vec)
        with K().option("tail_variant", 1):              # tail_kernel with 4 fragments read ahead
            K().tail_forward(att, yc, ts, b_o, g1, be1, vec)
    assert torch.equal(yb, yc)
    assert torch.isfinite(ya.float()).all()
    # the same arithmetic; the compilers' f32 contraction choices in the LayerNorm statistics may
    # differ, which moves a handful of outputs by one bf16 rounding step (measured: one feature in
    # ~2 % of rows)
    d = (ya.float() - yb.float()).abs()
    # (one bf16 step of the value, or of a ~1e-3 value for outputs near zero)
    ulp = yb.float().abs().clamp_min(2 ** -10) * 2 ** -7
    assert bool((d <= ulp * 1.01).all()), float((d / ulp).max())
    assert int((d > 0).sum()) <= max(8, ya.numel() // 1000), int((d > 0).sum())


def _bf16_step(x: torch.Tensor) -> torch.Tensor:
    """One bf16 unit in the last place at |x| (the spacing of bf16 values around x)."""
    e = torch.floor(torch.log2(x.abs().clamp_min(1e-30)))
    return torch.exp2(e - 7)


@pytest.mark.parametrize("M,Kd,lda_pad,bias,res", [(777, 1536, 0, True, False), (49440, 1536, 0, True, False),
                                                   (256, 1152, 64, False, True), (1, 64, 0, True, True),
                                                   (255, 128, 0, False, False), (49440, 1152, 0, False, True),
                                                   (513, 1536, 8, True, True)])
def test_gemm256_vs_fp32(M, Kd, lda_pad, bias, res):
    """snvrag_gemm256_forward (csrc/gemm256.hip: 256-row workgroups, transposed 32x32x16 MFMA over
    an LDS-DMA ring) vs torch fp32 on the same bf16 operands: ragged M (the last workgroup's rows
    past M read as zeros and are not stored), strided A, bias and residual epilogues, out aliasing
    the residual.  The kernel rounds once from its f32 sum, so each output is within one bf16
    step (+ f32 summation-order noise) of the f32 reference rounded to bf16."""
    g = torch.Generator(device="cpu").manual_seed(M + Kd)
    a_full = torch.randn(M, Kd + lda_pad, generator=g).to(DEV, torch.bfloat16)
    a = a_full[:, :Kd]
    w = (torch.randn(384, Kd, generator=g) / math.sqrt(Kd)).to(DEV, torch.bfloat16)
    b = torch.randn(384, generator=g).to(DEV) if bias else None
    r = torch.randn(M, 384, generator=g).to(DEV, torch.bfloat16) if res else None
    ref = a.float() @ w.float().t()
    if b is not None:
        ref = ref + b
    if r is not None:
        ref = ref + r.float()
    wp = K().gemm256_pack(w)
    out = K().gemm256(a, wp, 384, bias=b, resid=r.clone() if r is not None else None)
    tol = _bf16_step(ref) + 1e-4 * (1 + ref.abs())
    bad = (out.float() - ref).abs() > tol
    assert int(bad.sum()) == 0, f"{int(bad.sum())} of {bad.numel()} outside one bf16 step, first at " \
                                f"{bad.nonzero()[:4].tolist()}"
    if r is not None:                                 # in place: out aliases the residual
        r2 = r.clone()
        K().gemm256(a, wp, 384, bias=b, resid=r2, out=r2)
        assert torch.equal(r2, out)


@pytest.mark.parametrize("M,base,af_period", [(777, True, 259), (1, True, 0), (70001, True, 35000),
                                              (513, False, 0)])
def test_gemm256_ln_vs_fp32(M, base, af_period):
    """snvrag_gemm256_ln_forward (gemm256 EPI 1: the rag fusion's fusion[3] -> LayerNorm -> MAF
    weighting -> residual, fusion.py:152-162) vs torch fp32 on the same bf16 operands: two-pass row
    LayerNorm across the 4 waves' feature slices, base + scale * LN * w(af[m % period]); ragged M
    (M = 70 001 takes the multi-round workgroup-height choice).  Every workgroup height gives the
    same bits (the row sums are combined in wave order whatever the height)."""
    kk = K()
    g = torch.Generator(device="cpu").manual_seed(M + 11)
    Kd = 1536
    a = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(384, Kd, generator=g) / math.sqrt(Kd)).to(DEV, torch.bfloat16)
    b = torch.randn(384, generator=g).to(DEV)
    gm, be = (1 + 0.2 * torch.randn(384, generator=g)).to(DEV), (0.1 * torch.randn(384, generator=g)).to(DEV)
    bs = torch.randn(M, 384, generator=g).to(DEV, torch.bfloat16) if base else None
    af = torch.rand(af_period if af_period else M, generator=g).to(DEV)
    af[:3] = torch.tensor([0.0, 1.0, 0.5])[:af.numel()]                     # the clamp, both MAF branches
    wp = kk.gemm256_pack(w)
    out = kk.gemm256_ln(a, wp, b, (gm, be), base=bs, post_scale=0.37, post_af=af, post_af_period=af_period)
    y = torch.nn.functional.layer_norm(a.float() @ w.float().t() + b, (384,), gm, be, 1e-5)
    ai = af[torch.arange(M, device=DEV) % af.numel()]
    mw = torch.log1p(1.0 / (torch.minimum(ai, 1 - ai) + 1e-6)).clamp(max=3.0)
    # (no base: the LayerNorm output alone, as the row-panel GEMM's post epilogue)
    ref = bs.float() + 0.37 * y * mw[:, None] if bs is not None else y
    tol = _bf16_step(ref) + 1e-3 * (1 + ref.abs())
    bad = (out.float() - ref).abs() > tol
    assert int(bad.sum()) == 0, f"{int(bad.sum())} of {bad.numel()} outside tolerance, first at " \
                                f"{bad.nonzero()[:4].tolist()}"
    try:
        for groups in (4, 8):
            kk.set_option("g2_groups", groups)
            y2 = kk.gemm256_ln(a, wp, b, (gm, be), base=bs, post_scale=0.37, post_af=af, post_af_period=af_period)
            assert torch.equal(y2, out), groups
    finally:
        kk.set_option("g2_groups", 0)


def test_gemm256_derive_pack_matches_pack():
    """snvrag_derive kind 3 from f32 masters (plain, two stacked parts, and the transposed view a
    dX GEMM packs) == snvrag_gemm256_pack of the bf16-rounded matrix, byte for byte."""
    g = torch.Generator(device="cpu").manual_seed(5)
    w = torch.randn(384, 1536, generator=g).to(DEV)
    w1, w2 = torch.randn(192, 1152, generator=g).to(DEV), torch.randn(192, 1152, generator=g).to(DEV)
    wt = torch.randn(1152, 384, generator=g).to(DEV)               # [K, N]: pack W = wt^T
    kk = K()
    outs = [torch.empty_like(kk.gemm256_pack(w.to(torch.bfloat16))),
            torch.empty_like(kk.gemm256_pack(torch.cat([w1, w2]).to(torch.bfloat16))),
            torch.empty_like(kk.gemm256_pack(wt.t().to(torch.bfloat16)))]
    jobs = [kk.derive_job(kk.DERIVE_G2PACK, [w], outs[0]), kk.derive_job(kk.DERIVE_G2PACK, [w1, w2], outs[1]),
            kk.derive_job(kk.DERIVE_G2PACK, [wt.t()], outs[2])]
    kk.derive(kk.derive_table(jobs, DEV))
    assert torch.equal(outs[0], kk.gemm256_pack(w.to(torch.bfloat16)))
    assert torch.equal(outs[1], kk.gemm256_pack(torch.cat([w1, w2]).to(torch.bfloat16)))
    assert torch.equal(outs[2], kk.gemm256_pack(wt.t().to(torch.bfloat16)))


@pytest.mark.parametrize("groups", [4, 5, 6, 7, 8])
def test_gemm256_row_groups_bit_identical(groups):
    """Every workgroup height (option g2_groups: 32 x 4 .. 8 rows; the default picks it by M) and
    the v1 kernel (g2_variant 4: W through LDS) give the same bits: the K order of each output's sum
    does not depend on the tiling."""
    kk = K()
    g = torch.Generator(device="cpu").manual_seed(groups)
    M, Kd = 2 * 32 * groups * 3 + 77, 1152
    a = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(384, Kd, generator=g) / math.sqrt(Kd)).to(DEV, torch.bfloat16)
    b = torch.randn(384, generator=g).to(DEV)
    r = torch.randn(M, 384, generator=g).to(DEV, torch.bfloat16)
    wp = kk.gemm256_pack(w)
    ref = kk.gemm256(a, wp, 384, bias=b, resid=r)
    try:
        kk.set_option("g2_groups", groups)
        y = kk.gemm256(a, wp, 384, bias=b, resid=r)
        kk.set_option("g2_groups", 0)
        kk.set_option("g2_variant", 4)
        y1 = kk.gemm256(a, wp, 384, bias=b, resid=r)
    finally:
        kk.set_option("g2_groups", 0)
        kk.set_option("g2_variant", 0)
    assert torch.equal(y, ref) and torch.equal(y1, ref)
    e = (ref.float() - (a.float() @ w.float().t() + b + r.float())).abs()
    assert e.max().item() < 0.1
