"""Training-mode forward of the v18 model as an autograd graph over the HIP kernels.

Semantics follow the reference in train mode (dropout active, BatchNorm batch
statistics with running-stat updates), call stack model/foundation_model.py:25-33 ->
model/bert.py:148-219:

  BERTEmbedding (embedding/bert.py:53-75)      W[tok] + pe + AFEmbedding(af) -> dropout
  neighbour K-mean (bert.py:171-183)           the rag_emb_h1/h2 [B, K, L, D] train-mode
                                               retrieval adds (autograd-connected, averaged
                                               over K here), built by neighbour_embeddings
  EmbeddingFusionModule x4 (fusion.py:336-369) one [4B, L, D] GEMM + rank-2 pos/af terms
  EnhancedRareVariantFusion x2 (fusion.py:131-162)
  12 TransformerBlocks (transformer.py:32-35) h1 and h2 batched into one 2B dimension
  EnhancedHaplotypeClassifier, GenotypeClassifier (foundation_model.py:64-80, :156-176)

Heavy nodes (every Linear with K, N multiples of 8, attention) run on libsnvrag through
``autograd_ops``; the small per-site MLPs, LayerNorm, activations and dropout are torch
elementwise kernels.  Differences from the reference, all in the stochastic parts:
  * the attention-probability dropout (attention.py:28-29) draws its keep mask from a
    counter-based hash (csrc/attn_common.h) rather than torch's generator;
  * EnhancedRareVariantFusion's AF gate (af_adapter) is computed once per sample and
    shared by the h1 and h2 calls (the reference computes it twice with independent
    dropout masks; without dropout the two are identical);
  * the neighbours' dropout masks (embedding_rag_dataset.py:412-417) come from torch's
    generator on this rank, one per unique retrieved haplotype of a window, as in the
    reference; on a sharded panel the ranks exchange those haplotypes' allele codes and the
    dropped-out query embeddings (retrieval/shards.py) so the same semantics hold.
With dropout p = 0 the graph computes the reference's train-mode function exactly
(up to bf16 rounding) — the gradient parity tests run it that way.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .autograd_ops import (GradHandoff, head2_linear, hip_add_layernorm, hip_attention, hip_linear,
                           hip_linear_rank2, nbr_mean_drop, rag_mean_train, small_linear, tiny_embedding,
                           train_dtype)


def _drop(x: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    return F.dropout(x, p, training) if (training and p > 0) else x


def af_embedding(afm, af: torch.Tensor) -> torch.Tensor:
    """AFEmbedding.forward (af_embedding.py:70-91) -> [..., D] bf16."""
    x = af.float().unsqueeze(-1) * afm.basis_freqs
    feat = torch.cat([torch.sin(2 * math.pi * x), torch.cos(2 * math.pi * x)], -1)
    pr = afm.projection
    h = hip_linear(feat, pr[0].weight, pr[0].bias)
    h = F.gelu(hip_add_layernorm(h, None, pr[1]))
    return hip_linear(h, pr[3].weight, pr[3].bias)


def _conv1d(x: torch.Tensor, conv) -> torch.Tensor:
    """nn.Conv1d (stride 1, zero padding) as one batched [Cout, Cin*k] x [Cin*k, L] product over
    the k shifted copies of x.  At these channel counts (1-4, k = 9) the library's convolution
    weight-gradient kernels take milliseconds per call; this form's backward is two small GEMMs
    and a few slices (f32 throughout, as the reference runs it with autocast off)."""
    assert conv.stride == (1,) and conv.dilation == (1,) and conv.groups == 1
    w = conv.weight
    k, p, L = w.shape[-1], conv.padding[0], x.shape[-1]
    xp = F.pad(x, (p, p))
    cols = torch.stack([xp[..., j:j + L] for j in range(k)], 2)          # [B, Cin, k, L]
    out = torch.matmul(w.reshape(w.shape[0], -1), cols.reshape(x.shape[0], -1, L))
    return out + conv.bias[:, None]


def _batchnorm(bn, x: torch.Tensor, n_updates: int = 1) -> torch.Tensor:
    """nn.BatchNorm1d over [B, C, L] in torch ops (f32).  Train mode: batch statistics (biased
    variance) for the output, and the running statistics advanced as by ``n_updates`` forward
    calls on this same batch (the reference's repeated emb_fusion calls, fusion.py:351-369).
    The library (MIOpen) batch-norm backward at these shapes (C = 4 channels over B x 1030
    positions) differs from the reference's CPU autograd by 2-24 % relative in the f32 parity
    mode; these ops' autograd matches it to ~1e-6."""
    if not (bn.training or bn.running_mean is None):
        mean, var = bn.running_mean, bn.running_var
    else:
        dims = (0, 2)
        mean = x.mean(dims)
        var = (x - mean[None, :, None]).pow(2).mean(dims)
        if bn.training and bn.track_running_stats:
            with torch.no_grad():
                n = x.numel() // x.shape[1]
                var_u = var.detach() * (n / max(n - 1, 1))
                for _ in range(n_updates):
                    bn.num_batches_tracked += 1
                    m = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
                    bn.running_mean.mul_(1 - m).add_(mean.detach(), alpha=m)
                    bn.running_var.mul_(1 - m).add_(var_u, alpha=m)
    y = (x - mean[None, :, None]) * torch.rsqrt(var[None, :, None] + bn.eps)
    if bn.affine:
        y = y * bn.weight[None, :, None] + bn.bias[None, :, None]
    return y


def pos_feat(pfm, pos: torch.Tensor, n_updates: int = 1) -> torch.Tensor:
    """PositionFeatModule.forward (fusion.py:317-332), f32, BatchNorm in the module's mode
    (train: running statistics advanced ``n_updates`` times, see _batchnorm)."""
    out = pos.float().unsqueeze(1)
    out = _batchnorm(pfm.norm1, F.leaky_relu(_conv1d(out, pfm.conv1), 0.05), n_updates)
    out = _batchnorm(pfm.norm2, F.leaky_relu(_conv1d(out, pfm.conv2), 0.05), n_updates)
    return F.leaky_relu(_conv1d(out, pfm.conv3), 0.05).squeeze(1)


def _linear_cat2(x: torch.Tensor, lin, c1: torch.Tensor, c2: torch.Tensor) -> torch.Tensor:
    """Linear(cat([x, c1, c2], -1)) with the two extra input columns as rank-1 terms: in the
    stream GEMM's epilogue (bf16 out, autograd_ops.hip_linear_rank2), or f32 in torch."""
    return hip_linear_rank2(x, lin, c1, c2)


def _ln(x: torch.Tensor, m) -> torch.Tensor:
    """LayerNorm in f32 (statistics and affine), f32 out."""
    return F.layer_norm(x.float(), (x.shape[-1],), m.weight, m.bias, m.eps)


def emb_fusion(ef, embs: torch.Tensor, pos: torch.Tensor, af: torch.Tensor, n_calls: int) -> torch.Tensor:
    """EmbeddingFusionModule.forward (fusion.py:351-369) for n_calls stacked [B, L, D] inputs.
    The reference runs pos_feat once per call: its batch-statistics output is the same each time
    and its BatchNorm running statistics advance each time, so it runs once here with n_calls
    running-statistics updates."""
    pf = pos_feat(ef.pos_feat, pos, n_calls)
    rep = lambda t: t.repeat(n_calls, 1)
    # fusion.py:360-366: LeakyReLU(0.1) of the fusion Linear runs inside the LayerNorm kernel
    y = _linear_cat2(embs, ef.fusion, rep(pf), rep(af)).to(train_dtype())
    return hip_add_layernorm(embs, y, ef.norm, act_r=0.1)


def rag_fusion(rf, orig: torch.Tensor, rag: torch.Tensor, af: torch.Tensor, af_p: torch.Tensor, p: float,
               training: bool) -> torch.Tensor:
    """EnhancedRareVariantFusion.forward (fusion.py:131-162) for h1 and h2 stacked as [2B, L, D]
    (K = 1 after the neighbour mean, so the pooling softmax weight is exactly 1)."""
    ai = rf.af_interaction
    comb = torch.stack([af, af_p], -1)
    gate = torch.sigmoid(small_linear(F.gelu(small_linear(comb, ai.gate_net[0])), ai.gate_net[2]))
    enc = F.gelu(_ln(small_linear(comb, ai.joint_encoder[0]), ai.joint_encoder[1]))
    fused_af = af.unsqueeze(-1) + ai.res_scale * (gate * enc)
    ad = rf.af_adapter
    w = _drop(F.gelu(hip_linear(fused_af, ad[0].weight, ad[0].bias)), p, training)
    w = torch.sigmoid(hip_linear(w, ad[3].weight, ad[3].bias).float())            # [B, L, D]
    w2 = w.repeat(2, 1, 1)
    pooled = (rag.float() * w2).to(train_dtype())
    fu = rf.fusion
    h = _drop(F.gelu(hip_linear(torch.cat([orig, pooled], -1), fu[0].weight, fu[0].bias)), p, training)
    h = hip_add_layernorm(hip_linear(h, fu[3].weight, fu[3].bias), None, fu[4]).float()
    af2 = af.repeat(2, 1)
    maf = torch.minimum(af2, 1 - af2).unsqueeze(-1)
    mw = torch.log1p(1.0 / (maf + 1e-6)).clamp(max=3.0)
    return (orig.float() + rf.res_scale * (h * mw)).to(train_dtype())


def transformer_block(blk, x: torch.Tensor, nseq: int, L: int, p: float, training: bool) -> torch.Tensor:
    """TransformerBlock.forward (transformer.py:32-35), eval-identical except dropout."""
    a = blk.attention
    D = x.shape[-1]
    ll = a.linear_layers
    # x feeds the q/k/v GEMM and the sublayer's add+LayerNorm: the norm's dx is handed to the GEMM's
    # dX epilogue instead of autograd adding the two gradients (autograd_ops.GradHandoff)
    h_attn, h_ffn = GradHandoff(), GradHandoff()
    qkv = hip_linear(x.reshape(-1, D), [ll[0].weight, ll[1].weight, ll[2].weight],
                     [ll[0].bias, ll[1].bias, ll[2].bias], grad_from=h_attn)
    # attention-probability dropout (attention.py:28-29), counter-based mask shared with the backward
    att = hip_attention(qkv, nseq, L, a.heads, a.dims, a.dropout.p if training else 0.0)
    o = hip_linear(att, a.output_layer.weight, a.output_layer.bias).reshape(x.shape)
    # the dropouts around the norms are fused into the LayerNorm kernels: SublayerConnection's
    # dropout(norm(x + sublayer(x))) (sublayer.py:15-16) as the output dropout, FeedForward's
    # final dropout (feed_forward.py:21) on the residual operand, and TransformerBlock's own
    # dropout (transformer.py:35) folded into the output sublayer's: two independent keep masks
    # in a row are one Bernoulli((1 - p)^2) mask scaled by 1 / (1 - p)^2
    po = p if training else 0.0
    x = hip_add_layernorm(x, o, blk.input_sublayer.norm, p_out=po, grad_to=h_attn)
    ff = blk.feed_forward
    # feed_forward.py:20-21: both LeakyReLUs run inside the LayerNorm kernels (w_1's on the FFN
    # norm's input, w_2's on the output sublayer's residual operand, before its dropout)
    h = hip_linear(x, ff.w_1.weight, ff.w_1.bias, grad_from=h_ffn)
    f = hip_linear(hip_add_layernorm(h, None, ff.norm, act_x=0.1), ff.w_2.weight, ff.w_2.bias)
    return hip_add_layernorm(x, f, blk.output_sublayer.norm, p_r=po, p_out=1.0 - (1.0 - po) ** 2, act_r=0.1,
                             grad_to=h_ffn)


@dataclass
class NeighbourGroup:
    """The neighbours of one window's queries, as train-mode retrieval hands them over.

    rows          batch rows of this window (long [nb]); the group's queries are h1 of those
                  rows then h2 (2 nb queries)
    idx_h1/idx_h2 global panel indices [nb, k] (-1: no neighbour)
    index         the window's PanelIndex (this rank's shard of it on a sharded panel)
    counts        sharded panel, no dropout: the all-reduced per-site alt-allele counts of the
                  2 nb queries' neighbours (u8 [2 nb, ld]) — the K-mean needs nothing else
    uniq/uniq_codes  sharded panel with dropout: the sorted global indices of every neighbour
                  any rank retrieved and their allele codes (u8 [U, ld], all-reduced from the
                  owning shards), so each rank can re-encode its own neighbours"""
    rows: torch.Tensor
    idx_h1: torch.Tensor
    idx_h2: torch.Tensor
    index: object
    counts: Optional[torch.Tensor] = None
    uniq: Optional[torch.Tensor] = None
    uniq_codes: Optional[torch.Tensor] = None


def neighbour_means(bert, x: Dict, B: int, L: int) -> Optional[torch.Tensor]:
    """[2B, L, D] bf16 K-means of the retrieved neighbours (bert.py:171-183): from the
    ``rag_emb_h1/h2`` the retrieval added (train or eval; [B, K, L, D] averaged over K), or —
    a batch from an older hand-off carrying only ``rag_groups`` — re-encoded here."""
    if "rag_emb_h1" in x:
        out = []
        for key in ("rag_emb_h1", "rag_emb_h2"):
            r = x[key]
            r = r.mean(1) if r.dim() == 4 else r
            out.append(r.to(train_dtype()))
        return torch.cat(out, 0)
    groups = x.get("rag_groups")
    if not groups:
        return None
    return neighbour_embeddings(bert.embedding, groups, B, L).to(train_dtype())


def neighbour_embeddings(emb, groups: List[NeighbourGroup], B: int, L: int, dense: bool = False) -> torch.Tensor:
    """Train-mode re-encode of the retrieved neighbours (embedding_rag_dataset.py:404-442): the
    complete-token sequences through ``emb`` (BERTEmbedding with its AF embedding, in its own
    train/eval mode — dropout included), autograd-connected to the token table and the AF MLP.

    Returns f32 [2B, L, D] — the mean over each query's k neighbours (bert.py:176-179), rows h1
    then h2 — or, ``dense``, the reference's [2B, k, L, D] per-neighbour embeddings.

    As in the reference, each window's UNIQUE neighbours (over h1 and h2 of its queries,
    ``cat(I1, I2).unique()``, :406) are embedded once, so every query that retrieved the same
    haplotype sees the same dropout mask; the K-mean is then one [nq, U] x [U, L*D] product.
    Without dropout the mean comes from the ``rag_mean`` kernel (or the sharded counts) and an
    analytic backward — the same function, no [U, L, D] transient."""
    D = emb.embed_size
    pe = emb.position.pe[0, :L].float().contiguous()
    p = emb.dropout.p if emb.training else 0.0
    rows_out: List[torch.Tensor] = []
    vals: List[torch.Tensor] = []
    for g in groups:
        Ar = af_embedding(emb.af_embedding, g.index.ref_af.view(1, -1))[0].float() if emb.use_af else \
            torch.zeros(L, D, device=pe.device)
        idx = torch.cat([g.idx_h1, g.idx_h2], 0)
        if g.counts is not None and (p > 0 or dense):
            raise NotImplementedError("a sharded panel hands over neighbour counts only; retrieval must "
                                      "exchange codes (uniq/uniq_codes) for dropout or dense outputs")
        if p > 0 or dense or g.uniq is not None:
            m = _unique_neighbour_embed(emb.tokenizer.weight, Ar, idx, g, pe, L, p, dense)
        else:
            m = rag_mean_train(emb.tokenizer.weight, Ar, idx, g.index.codes, g.index.n_sites, pe, L,
                               counts=g.counts).float()
        nb = g.rows.numel()
        rows_out += [g.rows, g.rows + B]
        vals += [m[:nb], m[nb:]]
    order = torch.cat(rows_out)
    stacked = torch.cat(vals, 0)
    out = stacked.new_zeros(stacked.shape)
    out = out.index_put((order,), stacked)
    return out


def _unique_padded(x: torch.Tensor):
    """(uniq, inverse) of torch.unique(x, return_inverse=True) with ``uniq`` padded to x.numel()
    by repeating its largest value — computed by sort + run starts + prefix sum, no host sync."""
    flat = x.reshape(-1)
    srt, perm = torch.sort(flat)
    start = torch.ones_like(srt, dtype=torch.bool)
    start[1:] = srt[1:] != srt[:-1]
    rank = torch.cumsum(start, 0) - 1
    inv = torch.empty_like(flat)
    inv[perm] = rank
    uniq = srt[-1:].expand(flat.numel()).clone()
    uniq[rank] = srt
    return uniq, inv.view_as(x)


def _unique_neighbour_embed(W: torch.Tensor, Ar: torch.Tensor, idx: torch.Tensor, g: NeighbourGroup,
                            pe: torch.Tensor, L: int, p: float, dense: bool, tok0: int = 5, sos: int = 2,
                            eos: int = 3, pad: int = 0) -> torch.Tensor:
    """Embed the group's unique neighbours once (dropout p, one mask per haplotype), then
    gather (dense [nq, k, L, D]) or average ([nq, L, D]) them per query; f32."""
    nq, k = idx.shape
    n_sites = g.index.n_sites
    valid = idx >= 0
    fused = not dense and train_dtype() != torch.float32 and W.shape[0] * W.shape[1] <= 16384
    if g.uniq is not None:
        uniq, rows_codes = g.uniq, g.uniq_codes
        inv = torch.searchsorted(uniq, idx.clamp(min=0))
    elif fused:
        # torch.unique's inverse without its host sync (the unique COUNT is device data): the
        # same sorted ranks, the unique list padded to nq * k with its last value (the fused
        # kernels touch only the rows ``inv`` names)
        uniq, inv = _unique_padded(idx.clamp(min=0))
        rows_codes = g.index.codes[uniq - g.index.ref_offset]
    else:
        uniq, inv = torch.unique(idx.clamp(min=0), return_inverse=True)
        rows_codes = g.index.codes[uniq - g.index.ref_offset]
    U = uniq.numel()
    if fused:
        # fused: no [U, L, D] embeddings, one dropout mask per unique neighbour (csrc/train.hip)
        inv_v = torch.where(valid, inv, torch.full_like(inv, -1))
        return nbr_mean_drop(W, Ar, inv_v, rows_codes[:, :n_sites], n_sites, pe[:L], p)
    tok = torch.full((U, L), pad, device=idx.device, dtype=torch.long)
    tok[:, 0] = sos
    if n_sites + 1 < L:
        tok[:, n_sites + 1] = eos
    tok[:, 1:1 + n_sites] = tok0 + rows_codes[:, :n_sites].long()
    e = tiny_embedding(tok, W, 0) + pe[:L] + Ar                       # [U, L, D]
    if p > 0:
        e = F.dropout(e, p, True)
    if dense:
        return e[inv] * valid[..., None, None]
    # mean over each query's valid neighbours as a [nq, U] weight matrix (repeats counted)
    nv = valid.sum(1).clamp(min=1).to(e.dtype)
    S = torch.zeros(nq, U, device=e.device, dtype=e.dtype)
    S.index_put_((torch.arange(nq, device=e.device)[:, None].expand(nq, k)[valid], inv[valid]),
                 (1.0 / nv)[:, None].expand(nq, k)[valid], accumulate=True)
    return (S @ e.reshape(U, -1)).view(nq, L, -1)


def neighbour_mean_dropout(W: torch.Tensor, Ar: torch.Tensor, idx: torch.Tensor, codes: torch.Tensor, n_sites: int,
                           pe: torch.Tensor, L: int, p: float) -> torch.Tensor:
    """[nq, L, D] bf16 train-mode neighbour mean of one window's queries with the reference's
    dropout semantics (each unique neighbour re-encoded once, embedding_rag_dataset.py:404-417,
    then bert.py:171-183's mean over k), differentiable in W and Ar."""
    from types import SimpleNamespace
    index = SimpleNamespace(codes=codes, n_sites=n_sites, ref_offset=0)
    g = NeighbourGroup(rows=idx.new_zeros(0), idx_h1=idx, idx_h2=idx[:0], index=index)
    return _unique_neighbour_embed(W, Ar, idx, g, pe, L, p, False).to(train_dtype())


def forward_train(fm, x: Dict[str, torch.Tensor]) -> List[torch.Tensor]:
    """BERTFoundationModel.forward in train mode -> the reference's 7-element output list."""
    bert = fm.bert
    training = fm.training
    p = bert.embedding.dropout.p
    h1, h2 = x["hap_1"].long(), x["hap_2"].long()
    B, L = h1.shape
    dev = h1.device
    g = lambda k: x[k].to(dev, torch.float32)
    af, pos = g("af"), g("pos")
    af_p = g("af_p") if "af_p" in x else af
    emb = bert.embedding
    D = emb.embed_size
    # 1. query embeddings (embedding/bert.py:63-75); h1 and h2 stacked
    tok = torch.cat([h1, h2], 0)
    e = tiny_embedding(tok, emb.tokenizer.weight, 0) + emb.position.pe[:, :L]
    if emb.use_af:
        e = e + af_embedding(emb.af_embedding, af).float().repeat(2, 1, 1)
    h_raw = _drop(e.to(train_dtype()), p, training)                                          # [2B, L, D]
    # (no dropout on the mean itself: the re-encoded neighbours carry their own, bert.py:171-183)
    rag = neighbour_means(bert, x, B, L)
    if rag is not None:
        fused = emb_fusion(bert.emb_fusion, torch.cat([h_raw, rag], 0), pos, af, 4)
        hx = rag_fusion(bert.rag_fusion, fused[:2 * B], fused[2 * B:], af, af_p, p, training)
    else:
        hx = emb_fusion(bert.emb_fusion, h_raw, pos, af, 2)
    # 2. encoder (bert.py:213-217), both haplotypes in one batch
    for blk in bert.transformer_blocks:
        hx = transformer_block(blk, hx, 2 * B, L, p, training)
    # 3. heads (foundation_model.py:25-33)
    hc = fm.hap_classifier
    af2, afp2 = af.repeat(2, 1), af_p.repeat(2, 1)
    hh = F.gelu(_linear_cat2(hx, hc.af_fusion[0], af2, afp2).to(train_dtype()))
    hh = hip_add_layernorm(hip_linear(hh, hc.af_fusion[2].weight, hc.af_fusion[2].bias), None, hc.af_fusion[3])
    hh = F.gelu(hip_linear(hh, hc.net[0].weight, hc.net[0].bias))
    logits = head2_linear(hh, hc.net[2])
    probs = torch.softmax(logits, -1)
    p1, p2 = probs[:B], probs[B:]
    gc = fm.gt_classifier
    gf = torch.cat([p1, p2, g("ref").unsqueeze(-1), g("het").unsqueeze(-1), g("hom").unsqueeze(-1)], -1)
    gf = _ln(F.leaky_relu(small_linear(gf, gc.gf_fusion), 0.01), gc.gf_norm)
    ff = gc.layer
    gf = F.leaky_relu(small_linear(gf, ff.w_1), 0.1)
    gf = _drop(F.leaky_relu(small_linear(_ln(gf, ff.norm), ff.w_2), 0.1), ff.dropout.p, training)
    gt = torch.softmax(small_linear(gf, gc.classifier), -1)
    return [p1, p2, gt, h_raw[:B], h_raw[B:], hx[:B], hx[B:]]
