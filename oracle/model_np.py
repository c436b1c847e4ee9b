"""ORACLE (test infrastructure): numpy fp32 restatement of the SNVBERT eval forward.

Reference (paths relative to /root/reference/src):
  BERTEmbedding.forward          model/embedding/bert.py:55-77
  AFEmbedding.forward            model/embedding/af_embedding.py:70-91
  PositionFeatModule.forward     model/fusion.py:317-332
  EmbeddingFusionModule.forward  model/fusion.py:351-369
  CrossAFInteraction.forward     model/fusion.py:82-86
  EnhancedRareVariantFusion      model/fusion.py:131-162
  BERTWithEmbeddingRAG.forward   model/bert.py:148-219
  TransformerBlock.forward       model/transformer.py:27-30 (+ sublayer.py:15-16)
  MultiHeadAttention / Attention model/attention/multi_head_attention.py:44-51, attention.py:21-31
  FeedForward                    model/utils/feed_forward.py:18-21
  EnhancedHaplotypeClassifier    model/foundation_model.py:64-80
  GenotypeClassifier             model/foundation_model.py:156-176
  BERTFoundationModel.forward    model/foundation_model.py:25-33
Eval mode only: every Dropout is the identity, BatchNorm uses running stats.
"""

from __future__ import annotations

import math
from typing import Dict

import numpy as np
from scipy.special import erf

F32 = np.float32
EPS = 1e-5


def gelu(x):
    x = x.astype(F32)
    return (0.5 * x * (1.0 + erf(x / F32(math.sqrt(2.0))))).astype(F32)


def lrelu(x, slope):
    return np.where(x >= 0, x, x * F32(slope)).astype(F32)


def sigmoid(x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(F32)


def layernorm(x, w, b):
    x = x.astype(F32)
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return ((x - mu) / np.sqrt(var + F32(EPS)) * w + b).astype(F32)


def linear(x, sd, name):
    y = x.astype(F32) @ sd[name + ".weight"].T
    if name + ".bias" in sd:
        y = y + sd[name + ".bias"]
    return y.astype(F32)


def softmax(x, axis=-1):
    m = x.max(axis, keepdims=True)
    e = np.exp((x - m).astype(F32))
    return (e / e.sum(axis, keepdims=True)).astype(F32)


# --------------------------------------------------------------------------- #
def af_embedding(af, sd, p="bert.embedding.af_embedding"):
    """af_embedding.py:79-91: [sin, cos](2*pi*af*f) -> Linear -> LN -> GELU -> Linear."""
    fr = sd[p + ".basis_freqs"]
    ex = (af[..., None].astype(F32) * fr).astype(F32)
    ang = (F32(2 * math.pi) * ex).astype(F32)
    feat = np.concatenate([np.sin(ang), np.cos(ang)], -1).astype(F32)
    h = linear(feat, sd, p + ".projection.0")
    h = layernorm(h, sd[p + ".projection.1.weight"], sd[p + ".projection.1.bias"])
    return linear(gelu(h), sd, p + ".projection.3")


def embed(tok, af, sd):
    """embedding/bert.py:66-77 (pos=True, use_af=True), eval."""
    W = sd["bert.embedding.tokenizer.weight"]
    pe = sd["bert.embedding.position.pe"][0]
    L = tok.shape[-1]
    out = (W[tok] + pe[:L]).astype(F32)
    return (out + af_embedding(af, sd)).astype(F32)


def conv1d(x, w, b, pad=4):
    """x [B, Cin, L], w [Cout, Cin, K] -> [B, Cout, L] (stride 1, zero pad)."""
    B, Cin, L = x.shape
    Cout, _, K = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad)))
    out = np.zeros((B, Cout, L), np.float32) + b[None, :, None]
    for j in range(K):
        out += np.einsum("oc,bcl->bol", w[:, :, j], xp[:, :, j:j + L]).astype(F32)
    return out.astype(F32)


def batchnorm(x, sd, p):
    rm, rv = sd[p + ".running_mean"], sd[p + ".running_var"]
    w, b = sd[p + ".weight"], sd[p + ".bias"]
    return ((x - rm[None, :, None]) / np.sqrt(rv[None, :, None] + F32(EPS)) * w[None, :, None]
            + b[None, :, None]).astype(F32)


def pos_feat(pos, sd, p="bert.emb_fusion.pos_feat"):
    """fusion.py:324-332: norm1(act1(conv1)) -> norm2(act2(conv2)) -> act3(conv3); squeeze."""
    x = pos.astype(F32)[:, None, :]
    x = batchnorm(lrelu(conv1d(x, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"]), 0.05), sd, p + ".norm1")
    x = batchnorm(lrelu(conv1d(x, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"]), 0.05), sd, p + ".norm2")
    x = lrelu(conv1d(x, sd[p + ".conv3.weight"], sd[p + ".conv3.bias"]), 0.05)
    return x[:, 0, :]


def emb_fusion(emb, pf, af, sd, p="bert.emb_fusion"):
    """fusion.py:361-369: LN(emb + lrelu0.1(Linear(cat(emb, pos_feat, af))))."""
    cat = np.concatenate([emb, pf[..., None], af[..., None]], -1).astype(F32)
    h = lrelu(linear(cat, sd, p + ".fusion"), 0.1)
    return layernorm(emb + h, sd[p + ".norm.weight"], sd[p + ".norm.bias"])


def rag_fusion(orig, rag, af, af_p, sd, p="bert.rag_fusion"):
    """fusion.py:131-162 with K=1 (bert.py:197 passes the K-mean as [B,1,L,D])."""
    c = np.stack([af, af_p], -1).astype(F32)
    q = p + ".af_interaction"
    gate = sigmoid(linear(gelu(linear(c, sd, q + ".gate_net.0")), sd, q + ".gate_net.2"))
    enc = gelu(layernorm(linear(c, sd, q + ".joint_encoder.0"),
                         sd[q + ".joint_encoder.1.weight"], sd[q + ".joint_encoder.1.bias"]))
    fused_af = (af[..., None] + sd[q + ".res_scale"] * (gate * enc)).astype(F32)
    w = sigmoid(linear(gelu(linear(fused_af, sd, p + ".af_adapter.0")), sd, p + ".af_adapter.3"))
    weighted = (rag * w).astype(F32)
    # pooling: softmax over K=1 -> weight exactly 1.0 (fusion.py:145-146)
    logit = linear(weighted, sd, p + ".pooling.0")
    pw = softmax(logit[..., None, :], axis=-2)[..., 0, :]
    pooled = (weighted * pw).astype(F32)
    h = gelu(linear(np.concatenate([orig, pooled], -1), sd, p + ".fusion.0"))
    h = layernorm(linear(h, sd, p + ".fusion.3"), sd[p + ".fusion.4.weight"], sd[p + ".fusion.4.bias"])
    maf = np.minimum(af, 1 - af)[..., None].astype(F32)
    mw = np.minimum(np.log1p(1.0 / (maf + F32(1e-6))), 3.0).astype(F32)
    return (orig + sd[p + ".res_scale"] * (h * mw)).astype(F32)


def attention(x, sd, p, heads):
    B, L, D = x.shape
    dh = D // heads
    q, k, v = [linear(x, sd, f"{p}.linear_layers.{i}").reshape(B, L, heads, dh).transpose(0, 2, 1, 3)
               for i in range(3)]
    s = (q @ k.transpose(0, 1, 3, 2)) / F32(math.sqrt(dh))
    o = (softmax(s.astype(F32)) @ v).astype(F32)
    return linear(o.transpose(0, 2, 1, 3).reshape(B, L, D), sd, p + ".output_layer")


def feed_forward(x, sd, p):
    h = lrelu(linear(x, sd, p + ".w_1"), 0.1)
    h = layernorm(h, sd[p + ".norm.weight"], sd[p + ".norm.bias"])
    return lrelu(linear(h, sd, p + ".w_2"), 0.1)


def block(x, sd, p, heads):
    x = layernorm(x + attention(x, sd, p + ".attention", heads),
                  sd[p + ".input_sublayer.norm.weight"], sd[p + ".input_sublayer.norm.bias"])
    return layernorm(x + feed_forward(x, sd, p + ".feed_forward"),
                     sd[p + ".output_sublayer.norm.weight"], sd[p + ".output_sublayer.norm.bias"])


def hap_head(x, af, af_p, sd, p="hap_classifier"):
    h = np.concatenate([x, af[..., None], af_p[..., None]], -1).astype(F32)
    h = gelu(linear(h, sd, p + ".af_fusion.0"))
    h = layernorm(linear(h, sd, p + ".af_fusion.2"), sd[p + ".af_fusion.3.weight"], sd[p + ".af_fusion.3.bias"])
    logits = linear(gelu(linear(h, sd, p + ".net.0")), sd, p + ".net.2")
    return logits, softmax(logits)


def gt_head(p1, p2, ref, het, hom, sd, p="gt_classifier"):
    h = np.concatenate([p1, p2, ref[..., None], het[..., None], hom[..., None]], -1).astype(F32)
    h = layernorm(lrelu(linear(h, sd, p + ".gf_fusion"), 0.01), sd[p + ".gf_norm.weight"], sd[p + ".gf_norm.bias"])
    h = feed_forward(h, sd, p + ".layer")
    return softmax(linear(h, sd, p + ".classifier"))


def forward(x: Dict[str, np.ndarray], sd: Dict[str, np.ndarray], layers: int, heads: int):
    """BERTFoundationModel.forward (eval).  ``x['rag_mean_h*']`` is the K-mean of the
    retrieved neighbour embeddings ([B, L, D]; absent = the no-RAG path); returns a dict."""
    af, af_p = x["af"].astype(F32), x["af_p"].astype(F32)
    e1, e2 = embed(x["hap_1"], af, sd), embed(x["hap_2"], af, sd)
    pf = pos_feat(x["pos"], sd)
    h1 = emb_fusion(e1, pf, af, sd)
    h2 = emb_fusion(e2, pf, af, sd)
    if "rag_mean_h1" in x:                  # bert.py:171-206; without neighbours :207-210
        r1 = emb_fusion(x["rag_mean_h1"].astype(F32), pf, af, sd)
        r2 = emb_fusion(x["rag_mean_h2"].astype(F32), pf, af, sd)
        h1 = rag_fusion(h1, r1, af, af_p, sd)
        h2 = rag_fusion(h2, r2, af, af_p, sd)
    for i in range(layers):
        h1 = block(h1, sd, f"bert.transformer_blocks.{i}", heads)
    for i in range(layers):
        h2 = block(h2, sd, f"bert.transformer_blocks.{i}", heads)
    l1, p1 = hap_head(h1, af, af_p, sd)
    l2, p2 = hap_head(h2, af, af_p, sd)
    gt = gt_head(p1, p2, x["ref"], x["het"], x["hom"], sd)
    return dict(logits_h1=l1, logits_h2=l2, probs_h1=p1, probs_h2=p2, gt=gt,
                h1_before=e1, h2_before=e2, h1_after=h1, h2_after=h2, posfeat=pf)


def rag_mean(ref_complete_tokens, idx, ref_af, sd):
    """K-mean of re-encoded complete neighbour tokens (embedding_rag_dataset.py:406-438,
    bert.py:176-179) for one haplotype set: idx [B, k] -> [B, L, D]."""
    toks = ref_complete_tokens[idx]                     # [B, k, L]
    B, k, L = toks.shape
    e = embed(toks.reshape(B * k, L), np.broadcast_to(ref_af, (B * k, L)), sd)
    return e.reshape(B, k, L, -1).mean(1).astype(F32)
