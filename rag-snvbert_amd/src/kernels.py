"""Typed torch-tensor wrappers over the C ABI (one function per ``snvrag_*`` entry).

All tensors must be contiguous device tensors; outputs are allocated here unless
passed in.  Every call runs on the current HIP stream.  No CPU fallback.
"""

from __future__ import annotations

import contextlib

import ctypes as C
from typing import Optional, Sequence, Tuple

import torch

from . import native as N
from .native import check, ptr, stream_ptr

_dt = N.dtype_code


def _c(t: torch.Tensor) -> torch.Tensor:
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t


# ------------------------------------------------------------------ linear --
def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
           act: int = N.ACT_NONE, slope: float = 0.0,
           row1: Optional[Tuple[torch.Tensor, int, torch.Tensor]] = None,
           row2: Optional[Tuple[torch.Tensor, int, torch.Tensor]] = None,
           row_period: int = 0, resid: Optional[torch.Tensor] = None,
           ln: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, ln_act: int = N.ACT_NONE, ln_eps: float = 1e-5,
           post_base: Optional[torch.Tensor] = None, post_scale: float = 1.0,
           post_af: Optional[torch.Tensor] = None, post_af_period: int = 0, post_maf: bool = False,
           stats_out: Optional[torch.Tensor] = None,
           rownorm: Optional[Tuple[torch.Tensor, int, int, torch.Tensor]] = None,
           out: Optional[torch.Tensor] = None, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """out[m, n] = act(x[m] . w[n] + bias[n] + row1[m]*col1[n] + row2[m]*col2[n]) + resid[m, n],
    optionally followed by a fused LayerNorm over the row (``ln=(g, b)``, + ``ln_act`` and the
    ``post_base + post_scale * y * maf(post_af)`` tail), or writing row statistics
    (``stats_out`` float32 [n_tiles, M, 2]); ``rownorm=(stats, n_parts, dim, c1)`` folds a
    LayerNorm of ``x`` into the epilogue (``w`` must be pre-scaled by gamma, ``c1 = w_orig @ gamma``,
    beta folded into ``bias``) — see :func:`fold_layernorm`."""
    N.require_gpu(x, w)
    K = x.shape[-1]
    M = x.numel() // K
    Nn = w.shape[0]
    assert w.shape[1] == K and w.dtype == x.dtype, (tuple(w.shape), K, w.dtype, x.dtype)
    od = out_dtype or (out.dtype if out is not None else x.dtype)
    if out is None:
        out = torch.empty(*x.shape[:-1], Nn, device=x.device, dtype=od)
    e = N.Epilogue()
    e.bias = ptr(bias)
    if row1 is not None:
        e.row1, e.row1_stride, e.col1 = ptr(row1[0]), row1[1], ptr(row1[2])
    if row2 is not None:
        e.row2, e.row2_stride, e.col2 = ptr(row2[0]), row2[1], ptr(row2[2])
    e.row_period, e.act, e.slope = row_period, act, slope
    if resid is not None:
        assert resid.dtype == od and resid.shape[-1] == Nn
        e.resid, e.ld_resid = ptr(_c(resid)), Nn
    if ln is not None:
        e.ln_g, e.ln_b, e.ln_eps, e.ln_act = ptr(ln[0]), ptr(ln[1]), ln_eps, ln_act
    if post_base is not None:
        assert post_base.dtype == od
        e.post_base, e.ld_post, e.post_scale = ptr(_c(post_base)), Nn, post_scale
    if post_af is not None:
        e.post_af, e.post_af_period, e.post_maf = ptr(_c(post_af)), post_af_period, int(post_maf)
    e.stats_out = ptr(stats_out)
    an = None
    if rownorm is not None:
        st, parts, dim, c1 = rownorm
        an = N.RowNormS(ptr(st), parts, dim, 1e-5, ptr(c1))
    check(N.lib().snvrag_linear_ex(_dt(x.dtype), _dt(od), M, Nn, K, ptr(_c(x)), K, ptr(_c(w)), K,
                                   ptr(out), Nn, C.byref(e), C.byref(an) if an is not None else None,
                                   stream_ptr()), "linear")
    return out


def fold_layernorm(w: torch.Tensor, b: torch.Tensor, g: torch.Tensor, beta: torch.Tensor, dtype: torch.dtype):
    """LN(x) W^T + b = rstd*(x (W diag g)^T) - rstd*mean*(W g) + (W beta + b): returns (W', bias', c1)."""
    w64 = w.double()
    wg = (w64 * g.double()[None, :]).to(dtype).contiguous()
    return wg, (w64 @ beta.double() + b.double()).float().contiguous(), (w64 @ g.double()).float().contiguous()


def ffn_vec(b1, b2g, w2g, ln2_g, ln2_b) -> torch.Tensor:
    """[b1 (4D) | b2' | c1 | ln2_g | ln2_b] f32; c1 = row sums of the bf16 w2g."""
    c1 = w2g.to(torch.bfloat16).double().sum(1).float()
    return torch.cat([t.detach().float().reshape(-1) for t in (b1, b2g, c1, ln2_g, ln2_b)]).contiguous()


def tail_pack(w_o: torch.Tensor, w1: torch.Tensor, w2g: torch.Tensor) -> torch.Tensor:
    """One weight stream (W_o', then per 64-unit hidden chunk W1 and W2') of the 32x32-MFMA
    block tail (csrc/tail.hip)."""
    D = w_o.shape[1]
    nbytes = int(N.lib().snvrag_tail_pack_bytes(D))
    if nbytes == 0:
        raise ValueError(f"block tail needs D in (128, 256, 384), got {D}")
    ws = [_c(t.to(torch.bfloat16).contiguous()) for t in (w_o, w1, w2g)]
    assert tuple(ws[0].shape) == (D, D) and tuple(ws[1].shape) == (4 * D, D) and tuple(ws[2].shape) == (D, 4 * D)
    out = torch.empty(nbytes, device=w_o.device, dtype=torch.uint8)
    check(N.lib().snvrag_tail_pack(D, ptr(ws[0]), ptr(ws[1]), ptr(ws[2]), ptr(out), stream_ptr()), "tail_pack")
    return out


def proj_pack(w: torch.Tensor) -> torch.Tensor:
    """Stream of W [NC*D, D] (bf16) for ``proj_forward`` (NC = W.shape[0] // D)."""
    N.require_gpu(w)
    n, D = w.shape
    NC = n // D
    nbytes = int(N.lib().snvrag_proj_pack_bytes(D, NC))
    assert nbytes > 0 and NC * D == n, "projection needs D in {128, 256, 384} and NC*D rows"
    out = torch.empty(nbytes, device=w.device, dtype=torch.uint8)
    wb = _c(w.to(torch.bfloat16))
    check(N.lib().snvrag_proj_pack(D, NC, ptr(wb), ptr(out), stream_ptr()), "proj_pack")
    return out


def proj_forward(x: torch.Tensor, wstream: torch.Tensor, bias: torch.Tensor, NC: int,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out [M, NC*D] = x W^T + bias on the 32x32-MFMA stream kernel (bf16)."""
    N.require_gpu(x)
    assert x.dtype == torch.bfloat16
    D = x.shape[-1]
    M = x.numel() // D
    if out is None:
        out = torch.empty(M, NC * D, device=x.device, dtype=torch.bfloat16)
    b = _c(bias.float())
    check(N.lib().snvrag_proj_forward(M, D, NC, ptr(_c(x)), ptr(wstream), ptr(b), ptr(out), stream_ptr()),
          "proj_forward")
    return out


def tail_forward(att: torch.Tensor, x: torch.Tensor, wstream: torch.Tensor, b_o, ln1_g, ln1_b,
                 ffn_vec: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """x <- LN2(x1 + FFN(x1)), x1 = LN1(x + att W_o^T + b_o), in place (32x32-MFMA kernel)."""
    N.require_gpu(att, x)
    assert att.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and x.is_contiguous()
    D = x.shape[-1]
    M = x.numel() // D
    f = [_c(t.float().contiguous()) for t in (b_o, ln1_g, ln1_b)]
    check(N.lib().snvrag_tail_forward(M, D, ptr(_c(att)), ptr(x), ptr(wstream), ptr(f[0]), ptr(f[1]), ptr(f[2]),
                                      ptr(_c(ffn_vec)), eps, stream_ptr()), "tail_forward")
    return x


def tail_ffn_forward(x1: torch.Tensor, wstream: torch.Tensor, ffn_vec: torch.Tensor, eps: float = 1e-5,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = LN2(x1 + FFN(x1)) (32x32-MFMA kernel, FFN part of the tail stream)."""
    N.require_gpu(x1)
    assert x1.dtype == torch.bfloat16
    D = x1.shape[-1]
    M = x1.numel() // D
    if out is None:
        out = torch.empty_like(x1)
    check(N.lib().snvrag_tail_ffn_forward(M, D, ptr(_c(x1)), ptr(out), ptr(wstream), ptr(_c(ffn_vec)), eps,
                                          stream_ptr()), "tail_ffn_forward")
    return out


def stat_tiles(n: int) -> int:
    """Column tiles of the row-panel GEMM for an N (the stats_out leading dim)."""
    for bn in (384, 256, 128, 64):
        if n % bn == 0:
            return n // bn
    raise ValueError("N must be a multiple of 64")


def layernorm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, *, resid: Optional[torch.Tensor] = None,
              eps: float = 1e-5, out: Optional[torch.Tensor] = None, out_dtype: Optional[torch.dtype] = None,
              post_base: Optional[torch.Tensor] = None, post_scale: float = 1.0,
              post_af: Optional[torch.Tensor] = None, af_period: int = 0, maf_weight: bool = False,
              act: int = N.ACT_NONE) -> torch.Tensor:
    N.require_gpu(x)
    Nn = x.shape[-1]
    M = x.numel() // Nn
    od = out_dtype or (out.dtype if out is not None else x.dtype)
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=od)
    p = None
    if post_base is not None or post_af is not None or act != N.ACT_NONE:
        p = N.LnPost()
        p.base, p.ld_base, p.scale = ptr(post_base), Nn, post_scale
        p.af, p.af_period, p.maf_weight, p.act = ptr(post_af), af_period, int(maf_weight), act
    check(N.lib().snvrag_layernorm(_dt(x.dtype), _dt(od), M, Nn, ptr(_c(x)), Nn,
                                   ptr(resid), Nn, ptr(g), ptr(b), eps, ptr(out), Nn,
                                   C.byref(p) if p is not None else None, stream_ptr()), "layernorm")
    return out


def attention(qkv: torch.Tensor, nseq: int, L: int, heads: int, dh: int,
              out: Optional[torch.Tensor] = None, scale: Optional[float] = None) -> torch.Tensor:
    """softmax(q k^T * scale) v per (sequence, head); scale defaults to 1/sqrt(dh).  scale =
    1/log2(e) declares Q pre-scaled by log2(e)/sqrt(dh) (the engine's q_scale)."""
    N.require_gpu(qkv)
    D = heads * dh
    if out is None:
        out = torch.empty(nseq * L, D, device=qkv.device, dtype=qkv.dtype)
    check(N.lib().snvrag_attention(_dt(qkv.dtype), nseq, L, heads, dh, ptr(_c(qkv)), qkv.shape[-1],
                                   ptr(out), D, 1.0 / float(dh) ** 0.5 if scale is None else float(scale),
                                   stream_ptr()), "attention")
    return out


def attention_fallbacks(reset: bool = True) -> int:
    """Waves that took the exact online-max path of the bf16 dh=32 kernel (see attention.hip)."""
    n = N.lib().snvrag_attention_fallbacks(int(reset))
    if n < 0:
        check(n, "attention_fallbacks")
    return n


# ---------------------------------------------------------------- embedding --
def af_features(af: torch.Tensor, freqs: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    N.require_gpu(af)
    nb = freqs.numel()
    out = torch.empty(*af.shape, 2 * nb, device=af.device, dtype=dtype)
    check(N.lib().snvrag_af_features(_dt(dtype), af.numel(), ptr(_c(af)), ptr(_c(freqs)), nb, ptr(out),
                                     stream_ptr()), "af_features")
    return out


def embed_tokens(tok: torch.Tensor, W: torch.Tensor, pe: torch.Tensor, afemb: Optional[torch.Tensor],
                 af_period: int, dtype: torch.dtype, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    N.require_gpu(tok)
    assert tok.dtype == torch.int64
    nseq, L = tok.shape
    D = W.shape[1]
    if out is None:
        out = torch.empty(nseq, L, D, device=tok.device, dtype=dtype)
    check(N.lib().snvrag_embed_tokens(_dt(dtype), nseq, L, D, ptr(_c(tok)), ptr(_c(W)), W.shape[0],
                                      ptr(_c(pe)), ptr(afemb), _dt(afemb.dtype) if afemb is not None else 0,
                                      af_period, ptr(out), stream_ptr()), "embed_tokens")
    return out


def posfeat(pos: torch.Tensor, w: "N.PosfeatW") -> torch.Tensor:
    N.require_gpu(pos)
    B, L = pos.shape
    out = torch.empty(B, L, device=pos.device, dtype=torch.float32)
    check(N.lib().snvrag_posfeat(B, L, ptr(_c(pos)), C.byref(w), ptr(out), stream_ptr()), "posfeat")
    return out


def af_gate(af: torch.Tensor, af_p: torch.Tensor, w: "N.AfGateW", D: int, dtype: torch.dtype) -> torch.Tensor:
    N.require_gpu(af)
    out = torch.empty(*af.shape, D, device=af.device, dtype=dtype)
    check(N.lib().snvrag_af_gate(_dt(dtype), af.numel(), D, ptr(_c(af)), ptr(_c(af_p)), C.byref(w), ptr(out),
                                 stream_ptr()), "af_gate")
    return out


def rag_concat(q: torch.Tensor, rag: torch.Tensor, wgt: torch.Tensor, period: int) -> torch.Tensor:
    D = q.shape[-1]
    M = q.numel() // D
    out = torch.empty(*q.shape[:-1], 2 * D, device=q.device, dtype=q.dtype)
    check(N.lib().snvrag_rag_weighted_concat(_dt(q.dtype), M, D, ptr(_c(q)), ptr(_c(rag)), ptr(_c(wgt)),
                                             period, ptr(out), stream_ptr()), "rag_concat")
    return out


def hap_head_out(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, want_logits: bool = True):
    K = h.shape[-1]
    M = h.numel() // K
    probs = torch.empty(*h.shape[:-1], 2, device=h.device, dtype=torch.float32)
    logits = torch.empty_like(probs) if want_logits else None
    check(N.lib().snvrag_hap_head_out(_dt(h.dtype), M, K, ptr(_c(h)), K, ptr(_c(w)), ptr(_c(b)),
                                      ptr(logits), ptr(probs), stream_ptr()), "hap_head_out")
    return logits, probs


def gt_head(p1, p2, ref, het, hom, period: int, w: "N.GtW") -> torch.Tensor:
    M = p1.numel() // 2
    out = torch.empty(*p1.shape[:-1], 4, device=p1.device, dtype=torch.float32)
    check(N.lib().snvrag_gt_head(M, ptr(_c(p1)), ptr(_c(p2)), ptr(_c(ref)), ptr(_c(het)), ptr(_c(hom)), period,
                                 C.byref(w), ptr(out), stream_ptr()), "gt_head")
    return out


# ---------------------------------------------------------------------- kNN --
def knn_lut(tok_q: torch.Tensor, W: torch.Tensor, site_mask: torch.Tensor, n_sites: int, n_sites_pad: int,
            limbs: int = 2, Aq: Optional[torch.Tensor] = None, aq_period: int = 0,
            Ar: Optional[torch.Tensor] = None, tok0: int = 5, tok1: int = 6, mask_tok: int = 4,
            Wp: Optional[torch.Tensor] = None):
    """Returns (lut bytes tensor, exps int32 [nq], consts f32 [nq]).  ``Wp``: the panel side's
    token table when it differs from the queries' (a cached panel embedding, snvrag_knn_lut_panel)."""
    N.require_gpu(tok_q)
    nq, L = tok_q.shape
    D = W.shape[1]
    nbytes = N.lib().snvrag_knn_lut_bytes(nq, n_sites_pad, limbs)
    lut = torch.empty(nbytes, device=tok_q.device, dtype=torch.int8)
    exps = torch.empty(nq, device=tok_q.device, dtype=torch.int32)
    consts = torch.empty(nq, device=tok_q.device, dtype=torch.float32)
    if Wp is not None and Wp is not W:
        assert Wp.shape == W.shape and Wp.dtype == torch.float32
        check(N.lib().snvrag_knn_lut_panel(nq, L, D, ptr(_c(tok_q)), ptr(_c(W)), ptr(_c(Wp)), ptr(Aq), aq_period,
                                           ptr(Ar), ptr(_c(site_mask)), n_sites, n_sites_pad, tok0, tok1, mask_tok,
                                           limbs, ptr(lut), ptr(exps), ptr(consts), stream_ptr()), "knn_lut_panel")
    else:
        check(N.lib().snvrag_knn_lut(nq, L, D, ptr(_c(tok_q)), ptr(_c(W)), ptr(Aq), aq_period, ptr(Ar),
                                     ptr(_c(site_mask)), n_sites, n_sites_pad, tok0, tok1, mask_tok, limbs,
                                     ptr(lut), ptr(exps), ptr(consts), stream_ptr()), "knn_lut")
    return lut, exps, consts


def knn_scan(codes: torch.Tensor, n_sites_pad: int, lut: torch.Tensor, nq: int, limbs: int, k: int,
             ref_offset: int = 0, n_parts: Optional[int] = None, th_init: Optional[torch.Tensor] = None) -> torch.Tensor:
    n_ref, ld = codes.shape
    if n_parts is None:
        n_parts = N.lib().snvrag_knn_scan_parts(n_ref, nq)
    parts = torch.empty(n_parts, nq, k, device=codes.device, dtype=torch.int64)
    if th_init is not None:
        assert th_init.dtype == torch.int32 and th_init.numel() == nq
    check(N.lib().snvrag_knn_scan(ptr(_c(codes)), n_ref, ld, n_sites_pad, ptr(lut), nq, limbs, k, ref_offset,
                                  ptr(parts), n_parts, ptr(th_init), stream_ptr()), "knn_scan")
    return parts


def knn_threshold(keys: torch.Tensor, k: int) -> torch.Tensor:
    """Per-query strict start threshold (int32 [nq]) from merged keys [nq, k]."""
    nq = keys.shape[0]
    th = torch.empty(nq, device=keys.device, dtype=torch.int32)
    check(N.lib().snvrag_knn_threshold(ptr(_c(keys)), nq, k, ptr(th), stream_ptr()), "knn_threshold")
    return th


def topk_merge(keys: torch.Tensor, k: int) -> torch.Tensor:
    """keys int64 view of uint64 [n_lists, nq, k] -> [nq, k]."""
    n_lists, nq, kk = keys.shape
    assert kk == k
    out = torch.empty(nq, k, device=keys.device, dtype=torch.int64)
    wsb = N.lib().snvrag_topk_merge_ws_bytes(n_lists, nq, k)
    ws = torch.empty(wsb, device=keys.device, dtype=torch.uint8)
    check(N.lib().snvrag_topk_merge(ptr(_c(keys)), n_lists, nq, k, ptr(out), ptr(ws), wsb, stream_ptr()),
          "topk_merge")
    return out


def knn_decode(keys: torch.Tensor, exps: Optional[torch.Tensor] = None, consts: Optional[torch.Tensor] = None):
    nq, k = keys.shape
    idx = torch.empty(nq, k, device=keys.device, dtype=torch.int64)
    dist = torch.empty(nq, k, device=keys.device, dtype=torch.float32) if exps is not None else None
    check(N.lib().snvrag_knn_decode(ptr(_c(keys)), nq, k, ptr(exps), ptr(consts), ptr(idx), ptr(dist),
                                    stream_ptr()), "knn_decode")
    return idx, dist


def knn_emb_norms(E: torch.Tensor, chunk: int = 4096) -> torch.Tensor:
    """Squared L2 norms (f32) of the bf16 rows of E [N, K] — computed once when the embedding
    index is built (the stored-norm half of IndexFlatL2's ||q||^2 + ||r||^2 - 2 q.r)."""
    out = torch.empty(E.shape[0], device=E.device, dtype=torch.float32)
    for i in range(0, E.shape[0], chunk):
        out[i:i + chunk] = E[i:i + chunk].float().pow(2).sum(1)
    return out


def knn_emb_pack(E: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The scan's index layout (csrc/knn_emb.hip header): bf16 E [N, K] row-major -> bf16
    [ceil(N / 32) * 32, K] viewed storage of 4 KiB 32-row x 64-k tiles, padding rows zero.
    ``out`` (e.g. a slice of a larger packed index starting at a row multiple of 32) is filled in
    place."""
    assert E.dtype == torch.bfloat16 and E.dim() == 2
    n, kk = E.shape
    assert kk % 64 == 0
    rows = int(N.lib().snvrag_knn_emb_packed_bytes(n, kk)) // (2 * kk)
    if out is None:
        out = torch.empty(rows, kk, device=E.device, dtype=torch.bfloat16)
    assert out.dtype == torch.bfloat16 and out.is_contiguous() and out.numel() >= rows * kk
    check(N.lib().snvrag_knn_emb_pack(ptr(_c(E)), n, kk, ptr(out), stream_ptr()), "knn_emb_pack")
    return out


def knn_emb_dist(Et: torch.Tensor, Q: torch.Tensor, rn: torch.Tensor, qn: Optional[torch.Tensor] = None,
                 splits: Optional[int] = None) -> torch.Tensor:
    """Exact squared-L2 distances [Bq, N] between bf16 query rows Q [Bq, K] and the panel's
    flattened window embeddings, packed by ``knn_emb_pack`` (Et; N = len(rn), the rows' squared
    norms) (csrc/knn_emb.hip; the reference's cdist over [N, L * D], embedding_rag_dataset.py:390-402)."""
    assert Et.dtype == torch.bfloat16 and Q.dtype == torch.bfloat16 and Et.shape[1] == Q.shape[1]
    n, kk = rn.shape[0], Et.shape[1]
    assert Et.shape[0] == (n + 31) // 32 * 32, "Et must be knn_emb_pack's output for len(rn) rows"
    bq = Q.shape[0]
    assert 0 < bq <= 128 and kk % 64 == 0
    if splits is None:
        splits = int(N.lib().snvrag_knn_emb_splits(n, kk, bq))
    if qn is None:
        qn = knn_emb_norms(Q)
    ws = torch.empty(int(N.lib().snvrag_knn_emb_ws_bytes(n, bq, splits)) // 4, device=Et.device, dtype=torch.float32)
    check(N.lib().snvrag_knn_emb_scan(ptr(_c(Et)), n, kk, ptr(_c(Q)), bq, splits, ptr(ws), stream_ptr()),
          "knn_emb_scan")
    dist = torch.empty(bq, n, device=Et.device, dtype=torch.float32)
    check(N.lib().snvrag_knn_emb_finish(ptr(ws), splits, bq, n, ptr(_c(qn.float())), ptr(_c(rn.float())), ptr(dist),
                                        stream_ptr()), "knn_emb_finish")
    return dist


def knn_emb_search(Et: torch.Tensor, Q: torch.Tensor, k: int, rn: torch.Tensor, qn: Optional[torch.Tensor] = None):
    """(dist [Bq, k], idx [Bq, k]) — the k nearest panel rows in embedding space, ascending
    (torch.topk(largest=False) of embedding_rag_dataset.py:401 over the distance row); Et packed
    by knn_emb_pack."""
    d = knn_emb_dist(Et, Q, rn, qn)
    return torch.topk(d, k, dim=1, largest=False, sorted=True)


def rag_mean(idx: torch.Tensor, codes: torch.Tensor, n_sites: int, W: torch.Tensor, pe: torch.Tensor,
             Ar: Optional[torch.Tensor], L: int, dtype: torch.dtype, tok0=5, tok1=6, sos=2, eos=3, pad=0,
             out: Optional[torch.Tensor] = None, counts: Optional[torch.Tensor] = None):
    """[nq, L, D] mean over the k neighbours of their complete-token embeddings; ``out`` (e.g. the
    rag half of the encoder's input block) is written in place.  ``counts`` (u8 [nq, ld], the
    per-site alt-allele counts over the neighbours, see ``neighbor_counts``) replaces the panel
    rows ``codes[idx]`` (sharded panels; ``codes`` is then unused)."""
    nq, k = idx.shape
    D = W.shape[1]
    if out is None:
        out = torch.empty(nq, L, D, device=idx.device, dtype=dtype)
    assert out.dtype == dtype and tuple(out.shape) == (nq, L, D) and out.is_contiguous()
    if counts is not None:
        assert counts.dtype == torch.uint8 and counts.shape[0] == nq
        check(N.lib().snvrag_rag_mean_counts(_dt(dtype), nq, L, D, k, ptr(_c(idx)), ptr(_c(counts)), counts.shape[1],
                                             n_sites, ptr(_c(W)), ptr(_c(pe)), ptr(Ar), tok0, tok1, sos, eos, pad,
                                             ptr(out), stream_ptr()), "rag_mean_counts")
        return out
    check(N.lib().snvrag_rag_mean(_dt(dtype), nq, L, D, k, ptr(_c(idx)), ptr(_c(codes)), codes.shape[1], n_sites,
                                  ptr(_c(W)), ptr(_c(pe)), ptr(Ar), tok0, tok1, sos, eos, pad, ptr(out),
                                  stream_ptr()), "rag_mean")
    return out


def neighbor_counts(idx: torch.Tensor, codes: torch.Tensor, row0: int, ld_out: Optional[int] = None,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """u8 [nq, ld_out]: per-site alt-allele counts over the neighbours ``idx`` (global, int64
    [nq, k]) that fall in this shard's rows [row0, row0 + codes.shape[0])."""
    nq, k = idx.shape
    n_rows, ld = codes.shape
    ld_out = ld_out or ld
    if out is None:
        out = torch.empty(nq, ld_out, device=idx.device, dtype=torch.uint8)
    check(N.lib().snvrag_neighbor_counts(nq, k, ptr(_c(idx)), ptr(_c(codes)), ld, row0, n_rows, ptr(out), ld_out,
                                         stream_ptr()), "neighbor_counts")
    return out


def hamming_topk(codes_wm: torch.Tensor, queries: torch.Tensor, k: int) -> torch.Tensor:
    """Exact top-k keys [nq, k] ((d + 2^30) << 32 | row, (d, row) order) of bit-packed 0/1 rows
    (word-major int32 [nw, N]) for bit-packed queries (int32 [nq, nw]); d = Hamming distance."""
    nw, n = codes_wm.shape
    nq = queries.shape[0]
    assert queries.shape[1] == nw and codes_wm.dtype == torch.int32 and queries.dtype == torch.int32
    n_lists = int(N.lib().snvrag_hamming_list_count())
    lists = torch.empty(n_lists, nq, k, device=queries.device, dtype=torch.int64)
    check(N.lib().snvrag_hamming_lists(nq, n, nw, k, ptr(_c(codes_wm)), ptr(_c(queries)), ptr(lists),
                                       stream_ptr()), "hamming_lists")
    return topk_merge(lists, k)


def panel_synth(n_ref: int, n_sites: int, af: torch.Tensor, seed: int, ld: Optional[int] = None,
                row0: int = 0) -> torch.Tensor:
    """Rows [row0, row0 + n_ref) of the hash-generated synthetic panel (u8 [n_ref, ld])."""
    N.require_gpu(af)
    ld = ld or max(256, ((n_sites + 255) // 256) * 256)
    codes = torch.empty(n_ref, ld, device=af.device, dtype=torch.uint8)
    check(N.lib().snvrag_panel_synth_rows(ptr(codes), row0, n_ref, ld, n_sites, ptr(_c(af)), seed, stream_ptr()),
          "panel_synth")
    return codes


def encoder_forward(x: torch.Tensor, layers: Sequence["N.LayerW"], heads: int, ws: torch.Tensor) -> torch.Tensor:
    nseq, L, D = x.shape
    arr = (N.LayerW * len(layers))(*layers)
    check(N.lib().snvrag_encoder_forward(_dt(x.dtype), nseq, L, D, heads, len(layers), arr, ptr(_c(x)),
                                         ptr(ws), ws.numel(), stream_ptr()), "encoder_forward")
    return x


def encoder_ws_bytes(dtype: torch.dtype, nseq: int, L: int, D: int, heads: int) -> int:
    return int(N.lib().snvrag_encoder_ws_bytes(_dt(dtype), nseq, L, D, heads))


def selftest_mfma() -> int:
    return int(N.lib().snvrag_selftest_mfma(stream_ptr()))


def set_option(name: str, value: int) -> int:
    """Set a library option (snvrag_set_option: test hooks / micro-benchmark switches, see
    include/snvrag.h); returns the previous value."""
    import ctypes
    prev = ctypes.c_int64()
    check(N.lib().snvrag_get_option(name.encode(), ctypes.byref(prev)), "get_option")
    check(N.lib().snvrag_set_option(name.encode(), int(value)), "set_option")
    return int(prev.value)


@contextlib.contextmanager
def option(name: str, value: int):
    """``with option("knn_no_reduce", 1): ...`` — the previous value restored afterwards."""
    prev = set_option(name, value)
    try:
        yield
    finally:
        set_option(name, prev)


# ---------------------------------------------------------------- training --
def attention_train_fwd(qkv: torch.Tensor, nseq: int, L: int, heads: int, dh: int, dropout_p: float = 0.0,
                        seed: int = 0):
    """bf16 attention forward that also returns lse [nseq, heads, L] (log2 domain) for the backward;
    ``dropout_p`` > 0: attention-probability dropout with the counter-based mask of ``seed``."""
    N.require_gpu(qkv)
    assert qkv.dtype == torch.bfloat16
    D = heads * dh
    out = torch.empty(nseq * L, D, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(nseq, heads, L, device=qkv.device, dtype=torch.float32)
    check(N.lib().snvrag_attention_train_fwd(nseq, L, heads, dh, ptr(_c(qkv)), qkv.shape[-1], ptr(out), D,
                                             ptr(lse), 1.0 / float(dh) ** 0.5, float(dropout_p), int(seed) & (2 ** 64 - 1),
                                             stream_ptr()), "attention_train_fwd")
    return out, lse


def attention_bwd(qkv: torch.Tensor, out: torch.Tensor, dout: torch.Tensor, lse: torch.Tensor, nseq: int, L: int,
                  heads: int, dh: int, dropout_p: float = 0.0, seed: int = 0) -> torch.Tensor:
    """d(qkv) [nseq*L, 3D] bf16 of the unmasked softmax attention (csrc/attention_train.hip)."""
    N.require_gpu(qkv, out, dout, lse)
    D = heads * dh
    dqkv = torch.empty(nseq * L, 3 * D, device=qkv.device, dtype=torch.bfloat16)
    ws = torch.empty(nseq * heads * L, device=qkv.device, dtype=torch.float32)
    check(N.lib().snvrag_attention_bwd(nseq, L, heads, dh, ptr(_c(qkv)), qkv.shape[-1], ptr(_c(out)), out.shape[-1],
                                       ptr(_c(dout)), dout.shape[-1], ptr(_c(lse)), ptr(ws), ptr(dqkv), 3 * D,
                                       1.0 / float(dh) ** 0.5, float(dropout_p), int(seed) & (2 ** 64 - 1),
                                       stream_ptr()), "attention_bwd")
    return dqkv


def focal_loss(probs: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor, gamma: float, weight: float,
               loss_acc: Optional[torch.Tensor] = None):
    """(loss_sum [1] f32 (accumulated into loss_acc when given), d(weight*loss)/dprobs)."""
    N.require_gpu(probs)
    Cc = probs.shape[-1]
    M = probs.numel() // Cc
    p = _c(probs.float().contiguous())
    lab = labels.reshape(-1).long().contiguous()
    msk = mask.reshape(-1).to(torch.uint8).contiguous()
    if loss_acc is None:
        loss_acc = torch.zeros(1, device=probs.device, dtype=torch.float32)
    grad = torch.empty_like(p)
    check(N.lib().snvrag_focal_loss(M, Cc, ptr(p), ptr(lab), ptr(msk), float(gamma), float(weight), ptr(loss_acc),
                                    ptr(grad), stream_ptr()), "focal_loss")
    return loss_acc, grad


def sqnorm(x: torch.Tensor, acc: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """sum x^2 (f32, fixed reduction order) into acc [1]; the per-block partials go to ``ws`` (a
    caller-owned f32 buffer of snvrag_sqnorm_ws_bytes(), allocated here when not given) — never
    shared between calls on different streams."""
    N.require_gpu(x)
    assert x.dtype == torch.float32
    if acc is None:
        acc = torch.empty(1, device=x.device, dtype=torch.float32)
    nb = int(N.lib().snvrag_sqnorm_ws_bytes())
    if ws is None or ws.numel() * ws.element_size() < nb:
        ws = torch.empty(nb // 4, device=x.device, dtype=torch.float32)
    check(N.lib().snvrag_sqnorm_ws(x.numel(), ptr(_c(x)), ptr(acc), ptr(ws), ws.numel() * ws.element_size(),
                                   stream_ptr()), "sqnorm")
    return acc


def adam_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, *, lr: float, betas=(0.9, 0.999),
              eps: float = 1e-8, weight_decay: float = 0.0, step: int, grad_scale: float = 1.0,
              max_norm: float = 0.0, sq: Optional[torch.Tensor] = None, p_bf16: Optional[torch.Tensor] = None):
    N.require_gpu(p, g, m, v)
    a = N.AdamS(lr, betas[0], betas[1], eps, weight_decay, grad_scale, max_norm, step)
    check(N.lib().snvrag_adam_step(p.numel(), ptr(_c(p)), ptr(_c(g)), ptr(_c(m)), ptr(_c(v)), ptr(p_bf16), ptr(sq),
                                   C.byref(a), stream_ptr()), "adam_step")


def confusion(probs: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor, counts: torch.Tensor,
              mask2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """counts int64 [3, C] (tp, fp, fn) += cal_pr over the masked rows, on the device."""
    N.require_gpu(probs)
    Cc = probs.shape[-1]
    M = probs.numel() // Cc
    p = probs.float().contiguous()
    m2 = mask2.reshape(-1).to(torch.uint8).contiguous() if mask2 is not None else None
    check(N.lib().snvrag_confusion(M, Cc, ptr(p), ptr(labels.reshape(-1).long().contiguous()),
                                   ptr(mask.reshape(-1).to(torch.uint8).contiguous()), ptr(m2), ptr(_c(counts)),
                                   stream_ptr()), "confusion")
    return counts


def infer_post(probs_h1: torch.Tensor, probs_h2: torch.Tensor):
    """(p1, p2 [...], gt [..., 4]) of infer_embedding_rag.py:145-152 (second softmax included)."""
    N.require_gpu(probs_h1, probs_h2)
    a, b = probs_h1.float().contiguous(), probs_h2.float().contiguous()
    M = a.numel() // 2
    p1 = torch.empty(a.shape[:-1], device=a.device, dtype=torch.float32)
    p2 = torch.empty_like(p1)
    gt = torch.empty(*a.shape[:-1], 4, device=a.device, dtype=torch.float32)
    check(N.lib().snvrag_infer_post(M, ptr(a), ptr(b), ptr(p1), ptr(p2), ptr(gt), stream_ptr()), "infer_post")
    return p1, p2, gt


def ln_fwd_train(x: torch.Tensor, r: Optional[torch.Tensor], g: torch.Tensor, b: torch.Tensor, eps: float,
                 p_r: float = 0.0, p_out: float = 0.0, seed: int = 0, slope_x: float = 0.0, slope_r: float = 0.0):
    """(y bf16, s bf16 = act_x(x) + drop(act_r(r)) (x itself when r is None), stats f32 [M, 2]); y
    carries the output dropout p_out (masks: counter-based hash of seed, row, column).  slope_x /
    slope_r: LeakyReLU on x (no residual; s is then the pre-activation x) / on r before its dropout."""
    N.require_gpu(x)
    Nn = x.shape[-1]
    M = x.numel() // Nn
    y = torch.empty_like(x)
    s = torch.empty_like(x) if r is not None else x
    stats = torch.empty(M, 2, device=x.device, dtype=torch.float32)
    check(N.lib().snvrag_ln_fwd_train_act(M, Nn, ptr(_c(x)), ptr(_c(r)) if r is not None else None,
                                          ptr(_c(g)), ptr(_c(b)), eps, ptr(y), ptr(s) if r is not None else None,
                                          ptr(stats), float(p_r), float(p_out), int(seed) & (2 ** 64 - 1),
                                          float(slope_x), float(slope_r), stream_ptr()), "ln_fwd_train")
    return y, s, stats


def ln_bwd(dy: torch.Tensor, s: torch.Tensor, stats: torch.Tensor, g: torch.Tensor, p_r: float = 0.0,
           p_out: float = 0.0, seed: int = 0, dg: Optional[torch.Tensor] = None,
           db: Optional[torch.Tensor] = None, slope_x: float = 0.0, slope_r: float = 0.0,
           r_pre: Optional[torch.Tensor] = None):
    """(ds bf16, dres bf16 or None, dg f32 [N], db f32 [N]) of y = drop_o(LN(s) g + b),
    s = x + drop_r(r): ds = dx, dres = dr (None when p_r == 0 and no residual activation: dr =
    ds).  dg / db given (f32, contiguous: the parameters' .grad) are accumulated into, else fresh.
    slope_x: s is the pre-activation x of y = LN(lrelu(x)); slope_r: r_pre is the pre-activation
    residual (dres through the activation)."""
    Nn = s.shape[-1]
    M = s.numel() // Nn
    ds = torch.empty_like(s)
    dres = torch.empty_like(s) if (p_r > 0 or slope_r != 0.0) else None
    assert slope_r == 0.0 or r_pre is not None
    acc = dg is not None
    if dg is None:
        dg = torch.empty(Nn, device=s.device, dtype=torch.float32)
        db = torch.empty_like(dg)
    assert db is not None and dg.is_contiguous() and db.is_contiguous() and dg.dtype == db.dtype == torch.float32
    wsb = N.lib().snvrag_ln_bwd_ws_bytes(M, Nn)
    ws = torch.empty(wsb, device=s.device, dtype=torch.uint8)
    check(N.lib().snvrag_ln_bwd_act(M, Nn, ptr(_c(dy)), ptr(_c(s)), ptr(_c(stats)), ptr(_c(g)), ptr(ds), ptr(dres),
                                    ptr(_c(r_pre)) if r_pre is not None else None, ptr(dg), ptr(db), int(acc),
                                    float(p_r), float(p_out), int(seed) & (2 ** 64 - 1), float(slope_x),
                                    float(slope_r), ptr(ws), wsb, stream_ptr()), "ln_bwd")
    return ds, dres, dg, db


def nbr_mean_drop(inv: torch.Tensor, codes: torch.Tensor, n_sites: int, W: torch.Tensor, pe: torch.Tensor,
                  Ar: torch.Tensor, p: float, seed: int, tok0: int = 5, sos: int = 2, eos: int = 3,
                  pad: int = 0) -> torch.Tensor:
    """f32 [nq, L, D]: each query's mean over its valid unique neighbours inv [nq, k] (int32, < 0:
    none) of drop(W[tok] + pe + Ar), one dropout mask per unique neighbour (csrc/train.hip)."""
    N.require_gpu(inv, codes, W)
    nq, k = inv.shape
    L, D = pe.shape
    out = torch.empty(nq, L, D, device=W.device, dtype=torch.float32)
    check(N.lib().snvrag_nbr_mean_drop_fwd(nq, k, L, D, n_sites, codes.shape[1], W.shape[0], ptr(_c(inv)),
                                           ptr(_c(codes)), ptr(_c(W)), ptr(_c(pe)), ptr(_c(Ar)), float(p),
                                           int(seed) & (2 ** 64 - 1), tok0, sos, eos, pad, ptr(out), stream_ptr()),
          "nbr_mean_drop_fwd")
    return out


def nbr_mean_drop_bwd(dout: torch.Tensor, inv: torch.Tensor, codes: torch.Tensor, n_sites: int, W: torch.Tensor,
                      pe: torch.Tensor, Ar: torch.Tensor, p: float, seed: int, dW: torch.Tensor, dAr: torch.Tensor,
                      tok0: int = 5, sos: int = 2, eos: int = 3, pad: int = 0) -> None:
    """Accumulates dW [V, D] and dAr [L, D] (f32) of :func:`nbr_mean_drop` for dout [nq, L, D] f32."""
    nq, k = inv.shape
    L, D = pe.shape
    assert dW.dtype == dAr.dtype == torch.float32 and dW.is_contiguous() and dAr.is_contiguous()
    check(N.lib().snvrag_nbr_mean_drop_bwd(nq, k, L, D, n_sites, codes.shape[1], W.shape[0], ptr(_c(inv)),
                                           ptr(_c(codes)), ptr(_c(W)), ptr(_c(pe)), ptr(_c(Ar)), float(p),
                                           int(seed) & (2 ** 64 - 1), tok0, sos, eos, pad,
                                           ptr(_c(dout.float())), ptr(dW), ptr(dAr), stream_ptr()),
          "nbr_mean_drop_bwd")


def linear_dw(dy: torch.Tensor, x: torch.Tensor, bias: bool = False, splits: int = 0,
              dw: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None):
    """dW f32 [N, K] += dy^T x and (bias) db f32 [N] += column sums of dy, for bf16 dy [M, N] and
    x [M, K] whose rows may be strided (a column slice of a fused output: dy[:, a:b]); N, K
    multiples of 128 (csrc/dw.hip).  dw / db are ACCUMULATED into when given (f32, contiguous:
    e.g. a parameter's .grad), else zero-initialised.  Returns (dw, db or None)."""
    N.require_gpu(dy, x)
    assert dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.shape[0] == x.shape[0]
    assert dy.stride(1) == 1 and x.stride(1) == 1
    M, Nn = dy.shape
    Kk = x.shape[1]
    if dw is None:
        dw = torch.zeros(Nn, Kk, device=dy.device, dtype=torch.float32)
    assert dw.dtype == torch.float32 and dw.is_contiguous() and tuple(dw.shape) == (Nn, Kk)
    if bias and db is None:
        db = torch.zeros(Nn, device=dy.device, dtype=torch.float32)
    if db is not None:
        assert db.dtype == torch.float32 and db.is_contiguous() and db.numel() == Nn
    check(N.lib().snvrag_linear_dw(M, Nn, Kk, ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(dw), ptr(db),
                                   int(splits), stream_ptr()), "linear_dw")
    return dw, db


def linear_dw_parts(dy: torch.Tensor, x: torch.Tensor, dws, dbs=None, splits: int = 0) -> None:
    """dws[i] f32 [N / n, K] += dy[:, i N/n : (i+1) N/n]^T x (and dbs[i] += its column sums) in ONE
    launch over the fused output (csrc/dw.hip, snvrag_linear_dw_parts): the q/k/v weights'
    gradient buffers of one N = 3D projection."""
    N.require_gpu(dy, x)
    assert dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.shape[0] == x.shape[0]
    assert dy.stride(1) == 1 and x.stride(1) == 1
    M, Nn = dy.shape
    Kk = x.shape[1]
    n = len(dws)
    for t in dws:
        assert t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == (Nn // n, Kk)
    if dbs is not None:
        for t in dbs:
            assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == Nn // n
    import ctypes
    wp = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dws])
    bp = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dbs]) if dbs is not None else None
    check(N.lib().snvrag_linear_dw_parts(M, Nn, Kk, ptr(dy), dy.stride(0), ptr(x), x.stride(0), n, wp, bp,
                                         int(splits), stream_ptr()), "linear_dw_parts")


def colsum(x: torch.Tensor) -> torch.Tensor:
    """f32 column sums of a bf16 matrix [..., N] (bias gradients)."""
    Nn = x.shape[-1]
    M = x.numel() // Nn
    out = torch.empty(Nn, device=x.device, dtype=torch.float32)
    wsb = N.lib().snvrag_colsum_ws_bytes(M, Nn)
    ws = torch.empty(wsb, device=x.device, dtype=torch.uint8)
    check(N.lib().snvrag_colsum_bf16(M, Nn, ptr(_c(x)), ptr(out), ptr(ws), wsb, stream_ptr()), "colsum")
    return out


SG_ACT, SG_HEAD2, SG_LN = 0, 1, 2


def sgemm_pack(w: torch.Tensor) -> torch.Tensor:
    """Tile-major fragment stream of W [N, D] for the stream GEMM (csrc/sgemm.hip)."""
    N.require_gpu(w)
    Nn, D = w.shape
    nbytes = int(N.lib().snvrag_sgemm_pack_bytes(D, Nn))
    if nbytes == 0:
        raise ValueError(f"stream GEMM needs D in (128, 256, 384) and N % 64 == 0, got {tuple(w.shape)}")
    out = torch.empty(nbytes, device=w.device, dtype=torch.uint8)
    check(N.lib().snvrag_sgemm_pack(D, Nn, ptr(_c(w.to(torch.bfloat16).contiguous())), ptr(out), stream_ptr()),
          "sgemm_pack")
    return out


def gemm256_pack(w: torch.Tensor) -> torch.Tensor:
    """Fragment stream of W [N, K] for the wide-row GEMM (csrc/gemm256.hip)."""
    N.require_gpu(w)
    Nn, Kk = w.shape
    nbytes = int(N.lib().snvrag_gemm256_pack_bytes(Nn, Kk))
    if nbytes == 0:
        raise ValueError(f"wide-row GEMM pack needs N % 128 == 0 and K % 64 == 0, got {tuple(w.shape)}")
    wb = w.to(torch.bfloat16)
    if wb.stride(1) != 1:
        wb = wb.contiguous()
    out = torch.empty(nbytes, device=w.device, dtype=torch.uint8)
    check(N.lib().snvrag_gemm256_pack(Nn, Kk, ptr(wb), wb.stride(0), ptr(out), stream_ptr()), "gemm256_pack")
    return out


def gemm256(a: torch.Tensor, wpacked: torch.Tensor, n_out: int, bias: Optional[torch.Tensor] = None,
            resid: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 [M, N] = a [M, K] W^T (+ bias f32 [N]) (+ resid bf16 [M, N]) on the wide-row GEMM
    (csrc/gemm256.hip; W packed by :func:`gemm256_pack` or derive kind DERIVE_G2PACK).  ``out`` may
    alias ``resid`` (each element is read before it is written, by the same lane)."""
    N.require_gpu(a)
    assert a.dtype == torch.bfloat16 and a.dim() == 2 and a.stride(1) == 1
    M, Kk = a.shape
    assert wpacked.numel() * wpacked.element_size() == int(N.lib().snvrag_gemm256_pack_bytes(n_out, Kk))
    if out is None:
        out = torch.empty(M, n_out, device=a.device, dtype=torch.bfloat16)
    assert out.dtype == torch.bfloat16 and out.shape == (M, n_out) and out.stride(1) == 1
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == n_out
    if resid is not None:
        assert resid.dtype == torch.bfloat16 and resid.shape == (M, n_out) and resid.stride(1) == 1
    check(N.lib().snvrag_gemm256_forward(M, n_out, Kk, ptr(a), a.stride(0), ptr(wpacked),
                                         ptr(bias) if bias is not None else None,
                                         ptr(resid) if resid is not None else None,
                                         resid.stride(0) if resid is not None else 0, ptr(out), out.stride(0),
                                         stream_ptr()), "gemm256")
    return out


def gemm256_ln(a: torch.Tensor, wpacked: torch.Tensor, bias: Optional[torch.Tensor], ln: Tuple[torch.Tensor, torch.Tensor],
               base: Optional[torch.Tensor] = None, post_scale: float = 1.0, post_af: Optional[torch.Tensor] = None,
               post_af_period: int = 0, eps: float = 1e-5, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 [M, 384] = base + post_scale * LN(a W^T + bias) * w(post_af[m % period]) on the wide-row
    GEMM (csrc/gemm256.hip EPI 1): the rag fusion's fusion[3] -> fusion[4] -> MAF -> residual
    (fusion.py:152-162), the same arithmetic as :func:`linear` with ``ln=``, ``post_base=``,
    ``post_maf=True``."""
    N.require_gpu(a)
    assert a.dtype == torch.bfloat16 and a.dim() == 2 and a.stride(1) == 1
    M, Kk = a.shape
    n_out = 384
    assert wpacked.numel() * wpacked.element_size() == int(N.lib().snvrag_gemm256_pack_bytes(n_out, Kk))
    if out is None:
        out = torch.empty(M, n_out, device=a.device, dtype=torch.bfloat16)
    assert out.dtype == torch.bfloat16 and out.shape == (M, n_out) and out.stride(1) == 1
    for t in (bias, ln[0], ln[1]) if bias is not None else ln:
        assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n_out
    if base is not None:
        assert base.dtype == torch.bfloat16 and base.shape == (M, n_out) and base.stride(1) == 1
    if post_af is not None:
        assert post_af.dtype == torch.float32 and post_af.is_contiguous()
        assert post_af.numel() >= (post_af_period if post_af_period > 0 else M)
    check(N.lib().snvrag_gemm256_ln_forward(M, n_out, Kk, ptr(a), a.stride(0), ptr(wpacked),
                                            ptr(bias) if bias is not None else None, ptr(ln[0]), ptr(ln[1]), eps,
                                            ptr(base) if base is not None else None,
                                            base.stride(0) if base is not None else 0, post_scale,
                                            ptr(post_af) if post_af is not None else None, post_af_period,
                                            ptr(out), out.stride(0), stream_ptr()), "gemm256_ln")
    return out


DERIVE_F32, DERIVE_BF16, DERIVE_SGPACK, DERIVE_G2PACK = 0, 1, 2, 3


def derive_job(kind: int, parts, dst: torch.Tensor, dst_ld: int = 0) -> "N.DeriveJob":
    """One snvrag_derive job: ``parts`` = f32 2-D (strided) views stacked along their rows (1-D
    views count as columns [n, 1]); ``dst`` receives kind DERIVE_F32 / DERIVE_BF16 (row-major with
    row stride ``dst_ld``, default the column count), DERIVE_SGPACK (the stream-GEMM pack of the
    [N, D] matrix) or DERIVE_G2PACK (the wide-row GEMM pack of the [N, K] matrix).  piece0 / pieces are filled by ``derive_table``."""
    assert 1 <= len(parts) <= 4
    views = [t.unsqueeze(1) if t.dim() == 1 else t for t in parts]
    cols = views[0].shape[1]
    assert all(v.dim() == 2 and v.shape[1] == cols and v.dtype == torch.float32 and v.is_cuda for v in views)
    j = N.DeriveJob()
    j.kind, j.nparts = kind, len(views)
    j.rows, j.cols = sum(v.shape[0] for v in views), cols
    j.dst_ld = dst_ld or cols
    for i, v in enumerate(views):
        j.part_rows[i], j.rs[i], j.cs[i], j.src[i] = v.shape[0], v.stride(0), v.stride(1), v.data_ptr()
    if kind == DERIVE_SGPACK:
        assert int(N.lib().snvrag_sgemm_pack_bytes(cols, j.rows)) == dst.numel() * dst.element_size()
        j.pieces = j.rows * cols // 8
    elif kind == DERIVE_G2PACK:
        assert int(N.lib().snvrag_gemm256_pack_bytes(j.rows, cols)) == dst.numel() * dst.element_size()
        j.pieces = j.rows * cols // 8
    else:
        assert dst.dtype == (torch.float32 if kind == DERIVE_F32 else torch.bfloat16)
        assert (j.rows - 1) * j.dst_ld + cols <= dst.numel()
        j.pieces = (j.rows * cols + 7) // 8
    j.dst = dst.data_ptr()
    return j


def derive_table(jobs, device) -> Tuple[torch.Tensor, int, int]:
    """(device job table, job count, total pieces) for :func:`derive`."""
    total = 0
    for j in jobs:
        j.piece0 = total
        total += j.pieces
    arr = (N.DeriveJob * len(jobs))(*jobs)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device), len(jobs), total


def derive(table: Tuple[torch.Tensor, int, int]) -> None:
    """Run every job of a :func:`derive_table` in one launch (csrc/sgemm.hip derive_kernel)."""
    t, n, total = table
    check(N.lib().snvrag_derive(ptr(t), n, total, stream_ptr()), "derive")


def tokgrad(tok: torch.Tensor, g: torch.Tensor, V: int, padding_idx: Optional[int] = None) -> torch.Tensor:
    """f32 [V, D] weight gradient of W[tok] for the f32 output gradient g [..., D] (csrc/train.hip)."""
    N.require_gpu(g)
    D = g.shape[-1]
    t = _c(tok.reshape(-1).long())
    g2 = _c(g.reshape(-1, D).float())
    M = t.numel()
    dw = torch.empty(V, D, device=g.device, dtype=torch.float32)
    wsb = int(N.lib().snvrag_tokgrad_ws_bytes(M, V, D))
    ws = torch.empty(wsb // 4, device=g.device, dtype=torch.float32)
    check(N.lib().snvrag_tokgrad(M, V, D, -1 if padding_idx is None else int(padding_idx), ptr(t), ptr(g2), ptr(dw),
                                 ptr(ws), wsb, stream_ptr()), "tokgrad")
    return dw


def head2_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """f32 [..., 2] = x w^T + b for bf16 x [..., K], f32 w [2, K], b [2] (csrc/train.hip head2)."""
    N.require_gpu(x)
    Kd = x.shape[-1]
    M = x.numel() // Kd
    out = torch.empty(*x.shape[:-1], 2, device=x.device, dtype=torch.float32)
    check(N.lib().snvrag_head2_fwd(M, Kd, ptr(_c(x)), ptr(_c(w.float())), ptr(_c(b.float())), ptr(out),
                                   stream_ptr()), "head2_fwd")
    return out


def head2_bwd(g: torch.Tensor, x: torch.Tensor, w: torch.Tensor, want_dx: bool = True,
              dw: Optional[torch.Tensor] = None, accumulate: bool = False):
    """(dx bf16 [..., K] or None, dw f32 [2, K]) of :func:`head2_fwd` for the f32 gradient g [..., 2];
    ``dw`` given: written or (accumulate) added in place."""
    Kd = x.shape[-1]
    M = x.numel() // Kd
    dx = torch.empty_like(x) if want_dx else None
    if dw is None:
        dw = torch.empty(2, Kd, device=x.device, dtype=torch.float32)
    wsb = int(N.lib().snvrag_head2_ws_bytes(M, Kd))
    ws = torch.empty(wsb // 4, device=x.device, dtype=torch.float32)
    check(N.lib().snvrag_head2_bwd(M, Kd, ptr(_c(g.float())), ptr(_c(x)), ptr(_c(w.float())), ptr(dx), ptr(dw),
                                   int(accumulate), ptr(ws), wsb, stream_ptr()), "head2_bwd")
    return dx, dw


def sgemm_vec(bias: torch.Tensor, c1: Optional[torch.Tensor] = None, c2: Optional[torch.Tensor] = None,
              ln: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
              head: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """f32 vector table of :func:`sgemm`: [bias | c1, c2 | ln g, b | head w_out [2, N], b_out [2]]."""
    parts = [bias]
    if c1 is not None:
        parts += [c1, c2]
    if ln is not None:
        parts += list(ln)
    if head is not None:
        parts += [head[0].reshape(-1), head[1].reshape(-1)]
    return torch.cat([t.detach().float().reshape(-1) for t in parts]).contiguous()


def sgemm(x: torch.Tensor, wstream: torch.Tensor, n_out: int, vec: torch.Tensor, *, epi: int = SG_ACT,
          act: int = N.ACT_NONE, slope: float = 0.0,
          rank: Optional[Tuple[torch.Tensor, torch.Tensor, int]] = None, eps: float = 1e-5,
          out: Optional[torch.Tensor] = None, want_logits: bool = False):
    """Stream GEMM (bf16): SG_ACT -> act(x W^T + b [+ r1 c1 + r2 c2]) [..., n_out] bf16;
    SG_LN -> LN(act(.) + x) [..., D] bf16; SG_HEAD2 -> (logits or None, probs) [..., 2] f32.
    ``rank = (r1 f32, r2 f32, period)``: row scalars indexed by row % period."""
    N.require_gpu(x)
    assert x.dtype == torch.bfloat16
    D = x.shape[-1]
    M = x.numel() // D
    probs = logits = None
    if epi == SG_HEAD2:
        probs = torch.empty(*x.shape[:-1], 2, device=x.device, dtype=torch.float32)
        logits = torch.empty_like(probs) if want_logits else None
    elif out is None:
        out = torch.empty(*x.shape[:-1], n_out, device=x.device, dtype=torch.bfloat16)
    r1 = r2 = None
    period = 0
    if rank is not None:
        r1, r2 = _c(rank[0].float()), _c(rank[1].float())
        period = int(rank[2])
        assert r1.numel() >= period and r2.numel() >= period and period > 0
    check(N.lib().snvrag_sgemm_forward(M, D, n_out, epi, act, slope, ptr(_c(x)), ptr(wstream), ptr(vec), ptr(r1),
                                       ptr(r2), period, eps, ptr(out), ptr(probs), ptr(logits), stream_ptr()),
          "sgemm")
    return (logits, probs) if epi == SG_HEAD2 else out


def mlp_pack(w1: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """Stream of the fused MLP kernel (csrc/sgemm.hip mlp_kernel): W1 [4D, D], W2 [D, 4D] (bf16)."""
    N.require_gpu(w1, w2)
    D = w1.shape[1]
    nbytes = int(N.lib().snvrag_mlp_pack_bytes(D))
    if nbytes == 0 or tuple(w1.shape) != (4 * D, D) or tuple(w2.shape) != (D, 4 * D):
        raise ValueError(f"MLP stream needs W1 [4D, D], W2 [D, 4D] with D = 384, got {tuple(w1.shape)}, {tuple(w2.shape)}")
    out = torch.empty(nbytes, device=w1.device, dtype=torch.uint8)
    check(N.lib().snvrag_mlp_pack(D, ptr(_c(w1.to(torch.bfloat16).contiguous())),
                                  ptr(_c(w2.to(torch.bfloat16).contiguous())), ptr(out), stream_ptr()), "mlp_pack")
    return out


def mlp(x: torch.Tensor, wstream: torch.Tensor, vec: torch.Tensor, *, epi2: int,
        rank: Optional[Tuple[torch.Tensor, torch.Tensor, int]] = None, eps: float = 1e-5) -> torch.Tensor:
    """EPI2(GELU(x W1^T + b1 [+ rank]) W2^T + b2) [..., D] bf16 in one launch; epi2 0 = sigmoid,
    1 = LayerNorm; vec = [b1 | c1, c2 | b2 | g, be] (f32)."""
    N.require_gpu(x)
    assert x.dtype == torch.bfloat16
    D = x.shape[-1]
    M = x.numel() // D
    out = torch.empty_like(x)
    r1 = r2 = None
    period = 0
    if rank is not None:
        r1, r2, period = _c(rank[0].float()), _c(rank[1].float()), int(rank[2])
    check(N.lib().snvrag_mlp_forward(M, D, epi2, ptr(_c(x)), ptr(wstream), ptr(vec), ptr(r1), ptr(r2), period, eps,
                                     ptr(out), stream_ptr()), "mlp")
    return out


def mlp_afgate_pack(ag_t, mlp_vec: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(gate fragments bf16, vector table f32) of :func:`mlp_afgate` from CrossAFInteraction's
    weights ``ag_t`` = [gate_net[0].weight [32, 2], .bias, gate_net[2].weight [D, 32], .bias,
    joint_encoder[0].weight [D, 2], .bias, joint_encoder[1].weight, .bias] (f32) and the af_adapter
    MLP's table ``mlp_vec`` = [b1 | b2] (include/snvrag.h snvrag_mlp_afgate_forward)."""
    g1w, g1b, g2w, g2b, jw, jb, lnw, lnb = [t.detach().float() for t in ag_t]
    D = g2w.shape[0]
    assert D == 384 and g2w.shape[1] == 32 and g1w.shape == (32, 2) and jw.shape == (D, 2)
    cols = [jw[:, 0].double(), jw[:, 1].double(), jb.double()]
    mu = [c.mean() for c in cols]
    cc = [c - m for c, m in zip(cols, mu)]
    mom = torch.stack(mu + [(cc[0] * cc[0]).mean(), (cc[1] * cc[1]).mean(), (cc[0] * cc[1]).mean(),
                            (cc[0] * cc[2]).mean(), (cc[1] * cc[2]).mean(), (cc[2] * cc[2]).mean()]).float()
    vec = torch.cat([mlp_vec.float().reshape(-1), g2b, jw[:, 0], jw[:, 1], jb, lnw, lnb, g1w.reshape(-1), g1b,
                     mom.to(g2b.device)]).contiguous()
    dev = g2w.device
    m = torch.arange(32, device=dev)
    outf = 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3)
    T = torch.arange(12, device=dev).view(12, 1, 1, 1)
    s = torch.arange(2, device=dev).view(1, 2, 1, 1)
    lane = torch.arange(64, device=dev).view(1, 1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, 8)
    rows = 32 * T + outf[lane % 32]
    cols = 16 * (lane // 32) + 8 * s + j
    w = g2w[rows.expand(12, 2, 64, 8), cols.expand(12, 2, 64, 8)]          # [T, s, lane, 8]
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    frags = torch.stack([hi, lo], 2).contiguous()                          # [T, s, part, lane, 8]
    return frags, vec


def mlp_afgate(af: torch.Tensor, af_p: torch.Tensor, frags: torch.Tensor, res_scale: float, wstream: torch.Tensor,
               vec: torch.Tensor, D: int = 384) -> torch.Tensor:
    """sigmoid(GELU(x W1^T + b1) W2^T + b2) with x = CrossAFInteraction(af, af_p) computed inside
    the launch (fusion.py:135-138); [*af.shape, D] bf16."""
    N.require_gpu(af, af_p)
    af, af_p = _c(af.float()), _c(af_p.float())
    assert af.numel() == af_p.numel()
    out = torch.empty(*af.shape, D, device=af.device, dtype=torch.bfloat16)
    check(N.lib().snvrag_mlp_afgate_forward(af.numel(), D, ptr(af), ptr(af_p), ptr(frags), res_scale, ptr(wstream),
                                            ptr(vec), ptr(out), stream_ptr()), "mlp_afgate")
    return out


def sgemm_cat(q: torch.Tensor, x2: torch.Tensor, g2: torch.Tensor, period: int, wstream: torch.Tensor, n_out: int,
              vec: torch.Tensor) -> torch.Tensor:
    """GELU([q | bf16(x2 * g2[m % period])] W^T + b) [..., n_out] (bf16; the rag fusion's
    cat(h, aw * h_rag) input of fusion.py:157 built in registers); W packed by sgemm_pack."""
    N.require_gpu(q, x2, g2)
    Dh = q.shape[-1]
    M = q.numel() // Dh
    assert q.dtype == x2.dtype == g2.dtype == torch.bfloat16 and x2.numel() == q.numel()
    assert g2.numel() >= period * Dh
    out = torch.empty(*q.shape[:-1], n_out, device=q.device, dtype=torch.bfloat16)
    check(N.lib().snvrag_sgemm_cat_forward(M, Dh, n_out, ptr(_c(q)), ptr(_c(x2)), ptr(_c(g2)), period, ptr(wstream),
                                           ptr(vec), ptr(out), stream_ptr()), "sgemm_cat")
    return out

