"""Native execution engine: packs the nn.Module parameters once (f32 master copy
and bf16 copies for the MFMA path) and runs the v18 eval forward as a sequence
of libsnvrag kernels.  Kernel graph (one batch of B samples, 2B haplotypes):

  af_features -> linear(64->D) -> LN+GELU -> linear(D->D)         AF-MLP, once per sample
  embed_tokens(h1|h2) ............................................. K1 gather (origin outputs)
  [rag means supplied by retrieval: rag_mean kernel]               K4 (neighbour histogram mean)
  posfeat ........................................................... conv chain, once per sample
  linear(D->D, rank-2 pos/af epilogue, lrelu, +resid) -> LN        emb_fusion x4 in ONE GEMM
  [af_gate ->] linear(D->4D, gelu) -> linear(4D->D, sigmoid)        rag gate, once per sample, ONE
                                                                    launch (mlp_afgate) at bf16 D=384
  rag_concat -> linear(2D->4D, gelu) -> linear(4D->D) -> LN+maf tail  rag_fusion x2 in one GEMM each
                                                                    (cat in registers; gemm256_ln)
  encoder_forward (12 blocks, h1 and h2 batched)                    K7-K10
  hap head: linear(rank-2 af/af_p, gelu) -> linear -> LN -> linear(gelu) -> hap_head_out
  gt_head

Reference call stack: model/foundation_model.py:25-33 -> model/bert.py:148-219.
"""

from __future__ import annotations

import weakref
from typing import Dict, Optional

import math
import os

import torch
import torch.nn as nn

from . import kernels as K
from . import native as N

_ENGINES: "weakref.WeakKeyDictionary[nn.Module, Engine]" = weakref.WeakKeyDictionary()


def engine_for(module: nn.Module) -> "Engine":
    eng = _ENGINES.get(module)
    if eng is None:
        eng = Engine(module)
        _ENGINES[module] = eng
    return eng


def _rag_block_current(x: Dict[str, torch.Tensor]) -> bool:
    """True when the retrieval's in-place neighbour means (``rag_block`` / ``rag_mean``) still
    back ``rag_emb_h1/h2`` (the views retrieval returned), or no rag_emb_* is given at all."""
    if "rag_emb_h1" not in x or "rag_mean" not in x:
        return True
    m, B = x["rag_mean"], x["rag_emb_h1"].shape[0]
    return (x["rag_emb_h1"].data_ptr() == m.data_ptr() and x["rag_emb_h2"].data_ptr() == m[B:].data_ptr()
            and x["rag_emb_h1"].dtype == m.dtype)


def set_compute_dtype(module: nn.Module, dtype: torch.dtype) -> None:
    """torch.float32 (exact-f32 MFMA parity path, the default) or torch.bfloat16."""
    engine_for(module).set_dtype(dtype)


class _Packed:
    pass


class Engine:
    # bf16 at D = 384: the rag fusion's fusion[3] -> LN -> MAF tail on the wide-row GEMM (gemm256
    # EPI 1) instead of the row-panel GEMM's LN epilogue (class-level A/B switch; repack on change)
    rag_tail_wide = True
    # ... and CrossAFInteraction inside the af_adapter MLP launch (mlp_afgate)
    rag_afgate_fused = True

    def __init__(self, root: nn.Module):
        self.root = root
        self.dtype = torch.float32
        self._packed: Optional[_Packed] = None
        self._key = None
        self._enc_ws: Optional[torch.Tensor] = None

    # ----------------------------------------------------------------- setup --
    def set_dtype(self, dtype: torch.dtype) -> None:
        """Compute dtype of this module and of the embedding sub-module's engine (retrieval runs
        on ``model.bert.embedding`` and writes the neighbour means in this dtype)."""
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("compute dtype must be float32 or bfloat16")
        if dtype != self.dtype:
            self.dtype, self._packed = dtype, None
        _, _, emb = self._modules()
        if emb is not None and emb is not self.root:
            engine_for(emb).set_dtype(dtype)

    def _modules(self):
        r = self.root
        from .model.foundation_model import BERTFoundationModel
        from .model.bert import BERT
        from .model.embedding.bert import BERTEmbedding
        from .model.embedding.af_embedding import AFEmbedding
        if isinstance(r, BERTFoundationModel):
            return r, r.bert, r.bert.embedding
        if isinstance(r, BERT):
            return None, r, r.embedding
        if isinstance(r, BERTEmbedding):
            return None, None, r
        if isinstance(r, AFEmbedding):
            return None, None, None
        raise TypeError(f"no native engine for {type(r).__name__}")

    def _param_key(self):
        from .autograd_ops import _EPOCH      # in-place HIP optimizer updates bump no torch version
        return (_EPOCH[0],) + tuple((p.data_ptr(), p._version) for p in self.root.parameters()) + \
            tuple((b.data_ptr(), b._version) for b in self.root.buffers())

    def packed(self, allow_train: bool = False) -> _Packed:
        """Packed weights for the eval kernels.  ``allow_train``: eval semantics are wanted even
        though the module is in train mode (retrieval search / index, which the reference also
        runs without dropout — embedding_rag_dataset.py:358-371)."""
        if self.root.training and not allow_train:
            raise NotImplementedError("the native engine runs eval semantics (dropout off); train-mode "
                                      "forwards go through src/train_forward.py (BERTFoundationModel.forward)")
        key = self._param_key()
        if self._packed is None or key != self._key:
            self._packed = self._pack()
            self._key = key
        return self._packed

    def _pack(self) -> _Packed:
        fm, bert, emb = self._modules()
        dev = next(self.root.parameters()).device
        if dev.type != "cuda":
            raise N.NativeUnavailable("model parameters must live on the HIP device (model.to('cuda'))")
        N.load()
        T = self.dtype
        P = _Packed()
        f32 = lambda t: t.detach().to(dev, torch.float32).contiguous()
        cvt = lambda t: t.detach().to(dev, T).contiguous()
        P.keep = []

        def afmlp(a):
            return dict(freqs=f32(a.basis_freqs), w0=cvt(a.projection[0].weight), b0=f32(a.projection[0].bias),
                        g=f32(a.projection[1].weight), bb=f32(a.projection[1].bias),
                        w3=cvt(a.projection[3].weight), b3=f32(a.projection[3].bias))

        if emb is None:
            P.af = afmlp(self.root)
            return P
        P.D = emb.embed_size
        P.W = f32(emb.tokenizer.weight)
        P.pe = f32(emb.position.pe[0])
        P.pe0 = torch.zeros_like(P.pe)
        P.af = afmlp(emb.af_embedding) if emb.use_af else None
        if bert is None:
            return P
        D = P.D
        P.heads, P.n_layers = bert.attn_heads, bert.n_layers
        # emb_fusion
        ef = bert.emb_fusion
        fw = f32(ef.fusion.weight)
        P.ef = dict(w=cvt(fw[:, :D]), c_pos=fw[:, D].contiguous(), c_af=fw[:, D + 1].contiguous(),
                    b=f32(ef.fusion.bias), g=f32(ef.norm.weight), bb=f32(ef.norm.bias))
        # stream GEMM (csrc/sgemm.hip, 32x32 MFMAs, tile epilogues under the next tiles' MFMAs) for
        # the K = D projections at bf16; the row-panel GEMM (gemm_rows.hip) otherwise
        sg_ok = T == torch.bfloat16 and D in (128, 256, 384)
        if sg_ok:
            P.ef["w_sg"] = K.sgemm_pack(P.ef["w"])
            P.ef["v_sg"] = K.sgemm_vec(P.ef["b"], P.ef["c_pos"], P.ef["c_af"], ln=(P.ef["g"], P.ef["bb"]))
        pf = ef.pos_feat
        P.pf_t = [f32(t) for t in (pf.conv1.weight, pf.conv1.bias, pf.conv2.weight, pf.conv2.bias,
                                   pf.conv3.weight, pf.conv3.bias, pf.norm1.weight, pf.norm1.bias,
                                   pf.norm1.running_mean, pf.norm1.running_var, pf.norm2.weight, pf.norm2.bias,
                                   pf.norm2.running_mean, pf.norm2.running_var)]
        P.pf = N.PosfeatW(*[t.data_ptr() for t in P.pf_t], pf.norm1.eps)
        # rag fusion
        rf = bert.rag_fusion
        ai = rf.af_interaction
        P.ag_t = [f32(t) for t in (ai.gate_net[0].weight, ai.gate_net[0].bias, ai.gate_net[2].weight,
                                   ai.gate_net[2].bias, ai.joint_encoder[0].weight, ai.joint_encoder[0].bias,
                                   ai.joint_encoder[1].weight, ai.joint_encoder[1].bias)]
        P.ag = N.AfGateW(*[t.data_ptr() for t in P.ag_t], float(ai.res_scale.detach().float().item()))
        P.rf = dict(a0=cvt(rf.af_adapter[0].weight), a0b=f32(rf.af_adapter[0].bias),
                    a3=cvt(rf.af_adapter[3].weight), a3b=f32(rf.af_adapter[3].bias),
                    f0=cvt(rf.fusion[0].weight), f0b=f32(rf.fusion[0].bias),
                    f3=cvt(rf.fusion[3].weight), f3b=f32(rf.fusion[3].bias),
                    g=f32(rf.fusion[4].weight), bb=f32(rf.fusion[4].bias),
                    rs=float(rf.res_scale.detach().float().item()))
        if sg_ok and D == 384 and P.rf["f0"].shape == (4 * D, 2 * D):
            P.rf["f0_sg"], P.rf["f0_v"] = K.sgemm_pack(P.rf["f0"]), K.sgemm_vec(P.rf["f0b"])
        if sg_ok and D == 384 and P.rf["f3"].shape == (D, 4 * D) and self.rag_tail_wide:
            # fusion[3] + LayerNorm + MAF weighting + residual on the wide-row GEMM (csrc/gemm256.hip EPI 1)
            P.rf["f3_g2"] = K.gemm256_pack(P.rf["f3"])
        mlp_ok = sg_ok and D == 384
        if mlp_ok and P.rf["a0"].shape == (4 * D, D) and P.rf["a3"].shape == (D, 4 * D):
            # af_adapter: Linear -> GELU -> Linear -> Sigmoid in one launch, hidden on chip
            P.rf["a_mlp"] = K.mlp_pack(P.rf["a0"], P.rf["a3"])
            P.rf["a_mlp_v"] = K.sgemm_vec(torch.cat([P.rf["a0b"], P.rf["a3b"]]))
            if self.rag_afgate_fused and P.ag_t[2].shape == (D, 32):
                # CrossAFInteraction computed in the same launch (no [B, L, D] fused_af round trip)
                P.rf["afg_frags"], P.rf["afg_v"] = K.mlp_afgate_pack(P.ag_t, P.rf["a_mlp_v"])
        elif sg_ok and P.rf["a0"].shape == (4 * D, D):
            P.rf["a0_sg"], P.rf["a0_v"] = K.sgemm_pack(P.rf["a0"]), K.sgemm_vec(P.rf["a0b"])
        # encoder
        P.layers_t, P.layers = [], []
        for blk in bert.transformer_blocks:
            a, ff = blk.attention, blk.feed_forward
            w2g, b2g, c2g = K.fold_layernorm(ff.w_2.weight.detach().to(dev), ff.w_2.bias.detach().to(dev),
                                             ff.norm.weight.detach().to(dev), ff.norm.bias.detach().to(dev), T)
            # bf16: fold log2(e)/sqrt(dh) into the q rows so attention's exp2 takes raw scores
            qs = math.log2(math.e) / math.sqrt(a.dims) if T == torch.bfloat16 else 0.0
            wq = torch.cat([l.weight for l in a.linear_layers], 0).detach().to(dev).float().clone()
            bq = torch.cat([l.bias for l in a.linear_layers], 0).detach().to(dev).float().clone()
            if qs:
                wq[:D] *= qs
                bq[:D] *= qs
            t = dict(w_qkv=cvt(wq), b_qkv=f32(bq),
                     w_o=cvt(a.output_layer.weight), b_o=f32(a.output_layer.bias),
                     ln1_g=f32(blk.input_sublayer.norm.weight), ln1_b=f32(blk.input_sublayer.norm.bias),
                     w1=cvt(ff.w_1.weight), b1=f32(ff.w_1.bias),
                     lnf_g=f32(ff.norm.weight), lnf_b=f32(ff.norm.bias),
                     w2=cvt(ff.w_2.weight), b2=f32(ff.w_2.bias),
                     ln2_g=f32(blk.output_sublayer.norm.weight), ln2_b=f32(blk.output_sublayer.norm.bias),
                     w2g=w2g, b2g=b2g, c2g=c2g)
            if T == torch.bfloat16 and D in (128, 256, 384):
                # the whole block tail (W_o' + W1 + W2') on 32x32 MFMAs (csrc/tail.hip) + its vectors
                t["ffn_v"] = K.ffn_vec(t["b1"], b2g, w2g, t["ln2_g"], t["ln2_b"])
                t["tail_w"] = K.tail_pack(t["w_o"], t["w1"], w2g)
                # QKV on the stream GEMM (csrc/sgemm.hip, 8 waves); the 32x32 projection stream
                # (csrc/tail.hip PROJ mode) for launches past the stream GEMM's 2 GiB output
                t["qkv_sg"] = K.sgemm_pack(t["w_qkv"])
                t["qkv_pw"] = K.proj_pack(t["w_qkv"])
            P.layers_t.append(t)
            P.layers.append(N.LayerW(**{k: v.data_ptr() for k, v in t.items()}, q_scale=qs))
        if fm is None:
            return P
        hc = fm.hap_classifier
        hw = f32(hc.af_fusion[0].weight)
        P.hh = dict(w0=cvt(hw[:, :D]), c_af=hw[:, D].contiguous(), c_afp=hw[:, D + 1].contiguous(),
                    b0=f32(hc.af_fusion[0].bias), w2=cvt(hc.af_fusion[2].weight), b2=f32(hc.af_fusion[2].bias),
                    g=f32(hc.af_fusion[3].weight), bb=f32(hc.af_fusion[3].bias),
                    n0=cvt(hc.net[0].weight), n0b=f32(hc.net[0].bias),
                    n2=f32(hc.net[2].weight), n2b=f32(hc.net[2].bias))
        if sg_ok and D == 384 and P.hh["w2"].shape == (D, 4 * D):
            # af_fusion: Linear over cat(x, af, af_p) -> GELU -> Linear -> LayerNorm in one launch
            P.hh["f_mlp"] = K.mlp_pack(P.hh["w0"], P.hh["w2"])
            P.hh["f_mlp_v"] = torch.cat([P.hh["b0"], P.hh["c_af"], P.hh["c_afp"], P.hh["b2"], P.hh["g"],
                                         P.hh["bb"]]).float().contiguous()
        elif sg_ok and P.hh["w0"].shape == (4 * D, D):
            P.hh["w0_sg"] = K.sgemm_pack(P.hh["w0"])
            P.hh["w0_v"] = K.sgemm_vec(P.hh["b0"], P.hh["c_af"], P.hh["c_afp"])
        if sg_ok and P.hh["n2"].shape[0] == 2 and P.hh["n0"].shape == (4 * D, D):
            # net[0] + GELU + net[2] + softmax on the stream GEMM's head epilogue
            P.hh["n0_sg"] = K.sgemm_pack(P.hh["n0"])
            P.hh["n0_v"] = K.sgemm_vec(P.hh["n0b"], head=(P.hh["n2"], P.hh["n2b"]))
        gc = fm.gt_classifier
        P.gt_t = [f32(t) for t in (gc.gf_fusion.weight, gc.gf_fusion.bias, gc.gf_norm.weight, gc.gf_norm.bias,
                                   gc.layer.w_1.weight, gc.layer.w_1.bias, gc.layer.norm.weight,
                                   gc.layer.norm.bias, gc.layer.w_2.weight, gc.layer.w_2.bias,
                                   gc.classifier.weight, gc.classifier.bias)]
        P.gt = N.GtW(*[t.data_ptr() for t in P.gt_t])
        return P

    # ---------------------------------------------------------- sub-forwards --
    def af_embedding(self, af: torch.Tensor, allow_train: bool = False) -> torch.Tensor:
        """AFEmbedding forward (af_embedding.py:79-91) -> [..., D] in compute dtype."""
        P = self.packed(allow_train)
        a = P.af
        N.require_gpu(af)
        af = af.float().contiguous()
        T = self.dtype
        feat = K.af_features(af, a["freqs"], T)
        h = K.linear(feat, a["w0"], a["b0"], ln=(a["g"], a["bb"]), ln_act=N.ACT_GELU)
        return K.linear(h, a["w3"], a["b3"])

    def embed(self, seq: torch.Tensor, af: Optional[torch.Tensor] = None, pos: bool = False,
              af_period: int = 0, afemb: Optional[torch.Tensor] = None) -> torch.Tensor:
        """BERTEmbedding forward (embedding/bert.py:66-77), eval."""
        P = self.packed()
        N.require_gpu(seq)
        seq = seq.long().contiguous()
        if afemb is None and af is not None and P.af is not None:
            afemb = self.af_embedding(af)
            af_period = af_period or afemb.shape[0]
        return K.embed_tokens(seq, P.W, P.pe if pos else P.pe0, afemb, af_period, self.dtype)

    # -------------------------------------------------------------- forward --
    def _inputs(self, x: Dict[str, torch.Tensor]):
        h1, h2 = x["hap_1"], x["hap_2"]
        N.require_gpu(h1, h2)
        g = lambda k: x[k].to(h1.device, torch.float32).contiguous()
        return (h1.long().contiguous(), h2.long().contiguous(), g("af"), g("af_p") if "af_p" in x else g("af"),
                g("pos"))

    def input_block(self, B: int, L: int, device) -> torch.Tensor:
        """A fresh [4B, L, D] encoder input block: rows [2B:] are where a caller writes the
        neighbour K-means (``K.rag_mean(..., out=block[2 * B:])``) before passing
        ``x["rag_block"] = block`` to the forward, which then embeds the queries into rows [:2B]
        without copying the 2B*L*D neighbour rows again."""
        return torch.empty(4 * B, L, self.packed(allow_train=True).D, device=device, dtype=self.dtype)

    def rag_means(self, x: Dict[str, torch.Tensor], B: int, L: int, D: int) -> Optional[torch.Tensor]:
        """[2B, L, D] K-means of retrieved neighbours in compute dtype (bert.py:171-183).
        The retrieval's ``rag_block`` / ``rag_mean`` are used only while ``rag_emb_h1`` is still
        the view of them the retrieval returned: a caller that replaced rag_emb_h1/h2 gets its
        own tensors."""
        if not _rag_block_current(x):
            x = {k: v for k, v in x.items() if k not in ("rag_block", "rag_mean")}
        if "rag_block" in x:
            return x["rag_block"][2 * B:].to(self.dtype)
        if "rag_mean" in x:
            return x["rag_mean"].to(self.dtype).contiguous()
        if "rag_emb_h1" not in x:
            return None
        out = []
        for key in ("rag_emb_h1", "rag_emb_h2"):
            r = x[key]
            r = r[:, 0] if (r.dim() == 4 and r.size(1) == 1) else (r.mean(1) if r.dim() == 4 else r)
            out.append(r.to(self.dtype))
        return torch.cat(out, 0).contiguous()

    def forward_bert(self, x: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        P = self.packed()
        T, D = self.dtype, P.D
        h1, h2, af, af_p, pos = self._inputs(x)
        B, L = h1.shape
        BL = B * L
        afemb = self.af_embedding(af)                                 # [B, L, D]
        rag = self.rag_means(x, B, L, D)
        nblk = 4 if rag is not None else 2
        # the retrieval's block: its query rows [:2B] are written in place by the embedding below
        blk = x.get("rag_block") if _rag_block_current(x) else None
        if blk is not None and (blk.dtype != T or tuple(blk.shape) != (4 * B, L, D) or not blk.is_contiguous()):
            blk = None                                # produced for another dtype: copy below
        if blk is not None:
            hm = blk                                                  # rag rows already in place
        else:
            hm = torch.empty(nblk * B, L, D, device=h1.device, dtype=T)
        K.embed_tokens(torch.cat([h1, h2], 0), P.W, P.pe, afemb, B, T, out=hm[:2 * B])
        if rag is not None and blk is None:
            hm[2 * B:].copy_(rag)
        pf = K.posfeat(pos, P.pf)                                     # [B, L]
        ef = P.ef
        if "w_sg" in ef:
            fused = K.sgemm(hm, ef["w_sg"], D, ef["v_sg"], epi=K.SG_LN, act=N.ACT_LRELU, slope=0.1,
                            rank=(pf, af, BL))
        else:
            fused = K.linear(hm, ef["w"], ef["b"], row1=(pf, 1, ef["c_pos"]), row2=(af, 1, ef["c_af"]),
                             row_period=BL, act=N.ACT_LRELU, slope=0.1, resid=hm, ln=(ef["g"], ef["bb"]))
        if rag is not None:
            rf = P.rf
            if "afg_frags" in rf:
                aw = K.mlp_afgate(af, af_p, rf["afg_frags"], P.ag.res_scale, rf["a_mlp"], rf["afg_v"], D)
            elif "a_mlp" in rf:
                fa = K.af_gate(af, af_p, P.ag, D, T)                  # [B, L, D]
                aw = K.mlp(fa, rf["a_mlp"], rf["a_mlp_v"], epi2=0)
            else:
                fa = K.af_gate(af, af_p, P.ag, D, T)
                if "a0_sg" in rf:
                    t = K.sgemm(fa, rf["a0_sg"], rf["a0"].shape[0], rf["a0_v"], act=N.ACT_GELU)
                else:
                    t = K.linear(fa, rf["a0"], rf["a0b"], act=N.ACT_GELU)
                aw = K.linear(t, rf["a3"], rf["a3b"], act=N.ACT_SIGMOID)
            if "f0_sg" in rf:
                # cat(h, aw * h_rag) built in the GEMM's registers (no [2B, L, 2D] tensor)
                h = K.sgemm_cat(fused[:2 * B], fused[2 * B:], aw, BL, rf["f0_sg"], rf["f0"].shape[0], rf["f0_v"])
            else:
                cat = K.rag_concat(fused[:2 * B], fused[2 * B:], aw, BL)   # [2B, L, 2D]
                h = K.linear(cat, rf["f0"], rf["f0b"], act=N.ACT_GELU)
            if "f3_g2" in rf:
                xx = K.gemm256_ln(h.view(-1, h.shape[-1]), rf["f3_g2"], rf["f3b"], (rf["g"], rf["bb"]),
                                  base=fused[:2 * B].view(-1, D), post_scale=rf["rs"], post_af=af.view(-1),
                                  post_af_period=BL).view(2 * B, L, D)
            else:
                xx = K.linear(h, rf["f3"], rf["f3b"], ln=(rf["g"], rf["bb"]), post_base=fused[:2 * B],
                              post_scale=rf["rs"], post_af=af, post_af_period=BL, post_maf=True)
        else:
            xx = fused[:2 * B].clone()
        ws_bytes = K.encoder_ws_bytes(T, 2 * B, L, D, P.heads)
        if self._enc_ws is None or self._enc_ws.numel() < ws_bytes or self._enc_ws.device != h1.device:
            self._enc_ws = torch.empty(ws_bytes, device=h1.device, dtype=torch.uint8)
        K.encoder_forward(xx, P.layers, P.heads, self._enc_ws)
        return dict(h1_after=xx[:B], h2_after=xx[B:], h1_before=hm[:B], h2_before=hm[B:2 * B],
                    af=af, af_p=af_p, x_all=xx, B=B, L=L)

    def forward(self, x: Dict[str, torch.Tensor], want_logits: bool = False) -> Dict[str, torch.Tensor]:
        o = self.forward_bert(x)
        P = self.packed()
        B, L = o["B"], o["L"]
        BL = B * L
        hh = P.hh
        if "f_mlp" in hh:
            h = K.mlp(o["x_all"], hh["f_mlp"], hh["f_mlp_v"], epi2=1, rank=(o["af"], o["af_p"], BL))
        else:
            if "w0_sg" in hh:
                h = K.sgemm(o["x_all"], hh["w0_sg"], hh["w0"].shape[0], hh["w0_v"], act=N.ACT_GELU,
                            rank=(o["af"], o["af_p"], BL))
            else:
                h = K.linear(o["x_all"], hh["w0"], hh["b0"], row1=(o["af"], 1, hh["c_af"]),
                             row2=(o["af_p"], 1, hh["c_afp"]), row_period=BL, act=N.ACT_GELU)
            h = K.linear(h, hh["w2"], hh["b2"], ln=(hh["g"], hh["bb"]))
        if "n0_sg" in hh:
            logits, probs = K.sgemm(h, hh["n0_sg"], hh["n0"].shape[0], hh["n0_v"], epi=K.SG_HEAD2, act=N.ACT_GELU,
                                    want_logits=want_logits)
        else:
            h = K.linear(h, hh["n0"], hh["n0b"], act=N.ACT_GELU)
            logits, probs = K.hap_head_out(h, hh["n2"], hh["n2b"], want_logits=want_logits)
        dev = probs.device
        g = lambda k: x[k].to(dev, torch.float32).contiguous()
        gt = K.gt_head(probs[:B], probs[B:], g("ref"), g("het"), g("hom"), BL, P.gt)
        o.update(probs_h1=probs[:B], probs_h2=probs[B:], gt=gt)
        if want_logits:
            o.update(logits_h1=logits[:B], logits_h2=logits[B:])
        return o
