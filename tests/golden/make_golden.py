"""Generate the committed golden fixtures by RUNNING THE REFERENCE on seeded synthetic inputs.

Run in the build container only (it reads /root/reference, which does not exist
on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

How the reference is executed (no stub modules, no copied source in the repo):

* ``src/model/*`` imports cleanly (torch only) -> the real ``BERTFoundationModel``,
  ``BERTWithEmbeddingRAG``, ``BERTEmbedding`` run the forward passes.
* ``src/dataset/*`` cannot be imported here (faiss / allel / h5py / vcfpy are not
  installed), so the handful of torch/numpy-only functions on the hot path are
  lifted out of the reference files with ``ast`` at run time and executed as-is:
  ``EmbeddingRAGDataset.process_batch_retrieval`` + ``_apply_mask_to_tokens_gpu``
  (embedding_rag_dataset.py:285-461), ``TrainDataset.generate_mask`` / ``tokenize``
  (dataset.py:377-403, :597-625), ``TorchVocab/Vocab/WordVocab`` (vocab.py),
  ``VCFProcessingModule.sequence_padding / position_normalize`` (utils.py:109-132),
  ``WindowGroupedSampler`` (sampler.py) and ``WindowMajorSampler``
  (infer_embedding_rag.py:32-51).  Their text is read from /root/reference at
  generation time; only their OUTPUTS are committed (tests/golden/*.npz).

Weights: ``src.dataset.synthetic.synth_state_dict`` (per-key seeded streams) is
loaded into the reference modules, so the GPU box rebuilds identical weights
from the same generator; ``sd_digest`` in each fixture guards drift.
"""

from __future__ import annotations

import ast
import json
import math
import pickle
import random
import sys
import textwrap
from collections import Counter, defaultdict
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

REF = Path("/root/reference")
REPO = Path(__file__).resolve().parents[2]
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(REF / "src"))
sys.path.insert(0, str(REPO / "rag-snvbert_amd"))

from model.bert import BERTWithEmbeddingRAG  # noqa: E402  (reference)
from model.foundation_model import BERTFoundationModel  # noqa: E402  (reference)
from src.dataset import synthetic  # noqa: E402  (ours: data + weight generator only)

MAX_SEQ_LEN = 1030


# --------------------------------------------------------------------------- #
# run reference functions out of their source files
# --------------------------------------------------------------------------- #
def _source(path: Path) -> tuple[str, ast.Module]:
    text = path.read_text()
    return text, ast.parse(text)


def ref_function(relpath: str, cls: str | None, name: str, glb: dict):
    text, tree = _source(REF / relpath)
    scope = tree.body
    if cls is not None:
        scope = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls).body
    node = [n for n in scope if isinstance(n, ast.FunctionDef) and n.name == name][-1]
    src = textwrap.dedent(ast.get_source_segment(text, node))
    ns = dict(glb)
    exec(compile(src, f"{relpath}:{node.lineno}", "exec"), ns)
    return ns[name]


def ref_classes(relpath: str, names: list[str], glb: dict) -> dict:
    text, tree = _source(REF / relpath)
    ns = dict(glb)
    for n in tree.body:
        if isinstance(n, ast.ClassDef) and n.name in names:
            exec(compile(ast.get_source_segment(text, n), f"{relpath}:{n.lineno}", "exec"), ns)
    return {k: ns[k] for k in names}


NP_GLB = {"np": np, "torch": torch, "defaultdict": defaultdict, "MAX_SEQ_LEN": MAX_SEQ_LEN,
          "random": random, "Counter": Counter, "pickle": pickle, "json": json,
          "timer": (lambda f: f), "Literal": __import__("typing").Literal}

vocab_mod = ref_classes("src/dataset/vocab.py", ["TorchVocab", "Vocab", "WordVocab"], NP_GLB)
WordVocabRef = vocab_mod["WordVocab"]
seq_pad = ref_function("src/dataset/utils.py", "VCFProcessingModule", "sequence_padding", NP_GLB)
pos_norm = ref_function("src/dataset/utils.py", "VCFProcessingModule", "position_normalize", NP_GLB)
generate_mask = ref_function("src/dataset/dataset.py", "TrainDataset", "generate_mask", NP_GLB)
tokenize = ref_function("src/dataset/dataset.py", "TrainDataset", "tokenize", NP_GLB)
pbr = ref_function("src/dataset/embedding_rag_dataset.py", "EmbeddingRAGDataset",
                   "process_batch_retrieval", NP_GLB)
apply_mask = ref_function("src/dataset/embedding_rag_dataset.py", "EmbeddingRAGDataset",
                          "_apply_mask_to_tokens_gpu", NP_GLB)
sampler_glb = dict(NP_GLB)
from torch.utils.data import Sampler  # noqa: E402
from typing import Iterator  # noqa: E402
sampler_glb.update(Sampler=Sampler, Iterator=Iterator)
WindowGroupedSampler = ref_classes("src/dataset/sampler.py", ["WindowGroupedSampler"],
                                   sampler_glb)["WindowGroupedSampler"]
WindowMajorSampler = ref_classes("src/infer_embedding_rag.py", ["WindowMajorSampler"],
                                 sampler_glb)["WindowMajorSampler"]

POPS = ["AFR", "AMR", "EAS", "EUR", "SAS"]
MASK_RATES = [0.30, 0.40, 0.50, 0.60, 0.70, 0.80]


def ref_vocab():
    return WordVocabRef(POPS)


def ref_mask(af_unpadded: np.ndarray, level: int, seed: int, w: int) -> np.ndarray:
    """embedding_rag_dataset.py:527-544 with the reference generate_mask."""
    probs = np.where(af_unpadded < 0.05, 0.7, MASK_RATES[level])
    old = np.random.get_state()
    np.random.seed(seed * 10000 + w)
    raw = generate_mask(SimpleNamespace(), len(af_unpadded), probs=probs)
    np.random.set_state(old)
    return raw


def build_model(d, layers, heads, vocab_size, seed):
    torch.manual_seed(0)
    model = BERTFoundationModel(BERTWithEmbeddingRAG(vocab_size, d, layers, heads))
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    sd = synthetic.synth_state_dict(shapes, seed)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    model.eval()
    return model, synthetic.state_dict_digest(sd)


def make_inputs(win: synthetic.SynthWindow, vocab, level, epoch, w):
    fake = SimpleNamespace(vocab=vocab)
    raw_mask = ref_mask(win.af, level, epoch, w)
    mask = seq_pad(raw_mask, dtype="int")
    B = win.n_samples
    h1 = tokenize(fake, win.query[:, 0].astype(np.int64), mask)
    h2 = tokenize(fake, win.query[:, 1].astype(np.int64), mask)
    ref_complete = tokenize(fake, win.panel.astype(np.int64), np.zeros_like(mask))
    f = lambda a: np.stack([seq_pad(r, dtype="float") for r in np.atleast_2d(a)]).astype(np.float32)
    af = f(np.broadcast_to(win.af, (B, win.n_sites)))
    pos = f(np.broadcast_to(pos_norm(win.pos), (B, win.n_sites)))
    lab1 = np.stack([seq_pad(q, dtype="int") for q in win.query[:, 0].astype(np.int64)])
    lab2 = np.stack([seq_pad(q, dtype="int") for q in win.query[:, 1].astype(np.int64)])
    return dict(hap_1=h1.astype(np.int64), hap_2=h2.astype(np.int64), mask=mask.astype(np.int64),
                raw_mask=raw_mask.astype(np.int64), af=af, af_p=f(win.af_p), pos=pos,
                ref=f(win.ref), het=f(win.het), hom=f(win.hom), ref_complete=ref_complete.astype(np.int64),
                ref_af=seq_pad(win.af, dtype="float").astype(np.float32),
                hap_1_label=lab1, hap_2_label=lab2,
                gt_label=(lab1 << 1) + lab2)


def canonical_knn(W: np.ndarray, q_tok: np.ndarray, r_tok_masked: np.ndarray, k: int):
    """Exact decomposed L2 (eval, aligned masks, equal AF): sum_l ||W[q_l]-W[r_l]||^2, ranked by
    (dist, idx).  Tie-exact: the distance is sum over UNORDERED token pairs {t, s} of
    count{t,s} * G[t, s] (G in fp64), so equal pair counts give bit-equal distances (a plain
    fp64 sum over positions rounds differently depending on where the mismatches sit)."""
    W64 = W.astype(np.float64)
    V = W64.shape[0]
    G = ((W64[:, None, :] - W64[None, :, :]) ** 2).sum(-1)
    G = np.minimum(G, G.T)                                             # exact symmetry
    lo = np.minimum(q_tok[:, None, :], r_tok_masked[None, :, :])
    hi = np.maximum(q_tok[:, None, :], r_tok_masked[None, :, :])
    pid = lo * V + hi                                                  # [Bq, N, L]
    counts = np.zeros(pid.shape[:2] + (V * V,), np.int64)
    for b in range(pid.shape[0]):
        for r in range(pid.shape[1]):
            counts[b, r] = np.bincount(pid[b, r], minlength=V * V)
    dist = np.zeros(pid.shape[:2], np.float64)
    Gf = G.reshape(-1)
    for c in range(V * V):                                             # fixed order
        if counts[..., c].any():
            dist = dist + counts[..., c] * Gf[c]
    idx = np.arange(dist.shape[1])
    order = np.stack([np.lexsort((idx, d)) for d in dist])[:, :k]
    return order.astype(np.int64), dist


def run_case(name, d, layers, heads, B, n_sites, n_ref, k, level=4, seed=0, epoch=2024, w=0,
             keep_intermediate=False):
    torch.set_num_threads(8)
    vocab = ref_vocab()
    model, digest = build_model(d, layers, heads, len(vocab), seed)
    win = synthetic.SynthWindow(n_sites, n_ref, B, seed=seed + 17)
    x = make_inputs(win, vocab, level, epoch, w)
    emb = model.bert.embedding
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))

    # ---- reference retrieval (process_batch_retrieval, eval / no_grad like validation) ----
    fake = SimpleNamespace(jit_cache_win_idx=-1, jit_ref_emb_search=None, jit_ref_tokens_raw=None,
                           jit_ref_af_raw=None, ref_tokens_complete=[x["ref_complete"]],
                           ref_af_windows=[x["ref_af"]], window_masks=[x["mask"]], embed_dim=d,
                           vocab=vocab)
    fake._apply_mask_to_tokens_gpu = lambda t, m: apply_mask(fake, t, m)
    batch = {key: T(x[key]) for key in ("hap_1", "hap_2", "af")}
    batch["window_idx"] = [w] * B
    with torch.no_grad():
        batch = pbr(fake, batch, emb, torch.device("cpu"), k_retrieve=k)
        # indices the reference chose (same calls as embedding_rag_dataset.py:385-402)
        L = MAX_SEQ_LEN
        e1 = emb(T(x["hap_1"]), af=T(x["af"]), pos=True).reshape(B, -1)
        e2 = emb(T(x["hap_2"]), af=T(x["af"]), pos=True).reshape(B, -1)
        ref_m = apply_mask(fake, T(x["ref_complete"]), T(x["mask"]))
        er = emb(ref_m, af=T(x["ref_af"])[None].expand(n_ref, -1), pos=True).reshape(n_ref, -1)
        dref1, Iref1 = torch.cdist(e1, er, p=2).topk(k, largest=False, dim=1)
        dref2, Iref2 = torch.cdist(e2, er, p=2).topk(k, largest=False, dim=1)

    W = model.bert.embedding.tokenizer.weight.detach().numpy()
    rm = ref_m.numpy()
    Ican1, dist1 = canonical_knn(W, x["hap_1"], rm, k)
    Ican2, dist2 = canonical_knn(W, x["hap_2"], rm, k)

    # ---- forward (reference retrieval) ----
    logits = []
    hook = model.hap_classifier.net.register_forward_hook(lambda m, i, o: logits.append(o.detach().clone()))
    fwd_keys = ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom")
    xin = {key: T(x[key]) for key in fwd_keys}
    with torch.no_grad():
        xin["rag_emb_h1"], xin["rag_emb_h2"] = batch["rag_emb_h1"], batch["rag_emb_h2"]
        out = model(xin)
        logits_ref = [l.numpy() for l in logits]
        # ---- forward with canonical neighbours ----
        logits.clear()

        def rag_from(I):
            toks = T(x["ref_complete"])[torch.from_numpy(I.reshape(-1))]
            e = emb(toks, af=T(x["ref_af"])[None].expand(toks.shape[0], -1), pos=True)
            return e.reshape(B, k, MAX_SEQ_LEN, d)
        xin2 = dict(xin)
        xin2["rag_emb_h1"], xin2["rag_emb_h2"] = rag_from(Ican1), rag_from(Ican2)
        out_can = model(xin2)
        logits_can = [l.numpy() for l in logits]
    hook.remove()

    res = dict(cfg=np.array(json.dumps(dict(d=d, layers=layers, heads=heads, vocab=len(vocab), B=B,
                                              n_sites=n_sites, n_ref=n_ref, k=k, level=level, seed=seed,
                                              epoch=epoch, w=w, sd_digest=digest))),
               panel=win.panel, query=win.query,
               Iref_h1=Iref1.numpy(), Iref_h2=Iref2.numpy(), dref_h1=dref1.numpy(), dref_h2=dref2.numpy(),
               Ican_h1=Ican1, Ican_h2=Ican2,
               dcan_h1=np.take_along_axis(dist1, Ican1, 1), dcan_h2=np.take_along_axis(dist2, Ican2, 1),
               kth_margin_h1=_kth_margin(dist1, k), kth_margin_h2=_kth_margin(dist2, k),
               probs_h1=out[0].numpy(), probs_h2=out[1].numpy(), gt=out[2].numpy(),
               logits_h1=logits_ref[0], logits_h2=logits_ref[1],
               can_probs_h1=out_can[0].numpy(), can_probs_h2=out_can[1].numpy(), can_gt=out_can[2].numpy(),
               can_logits_h1=logits_can[0], can_logits_h2=logits_can[1])
    for key in ("hap_1", "hap_2", "mask", "raw_mask", "af", "af_p", "pos", "ref", "het", "hom",
                "ref_complete", "ref_af", "hap_1_label", "hap_2_label", "gt_label"):
        res[key] = x[key]
    if keep_intermediate:
        with torch.no_grad():
            res["emb_h1"] = emb(T(x["hap_1"]), af=T(x["af"]), pos=True).numpy()
            res["af_emb"] = emb.af_embedding(T(x["af"])).numpy()
            res["posfeat"] = model.bert.emb_fusion.pos_feat(T(x["pos"])).numpy()
            res["rag_mean_h1"] = batch["rag_emb_h1"].mean(1).numpy()
            res["h1_after"] = out[5].numpy()
            res["h1_before"] = out[3].numpy()
    np.savez_compressed(OUT / f"{name}.npz", **res)
    same1 = (np.sort(Iref1.numpy(), 1) == np.sort(Ican1, 1)).all(1)
    print(f"{name}: digest={digest} ref-vs-canonical index sets equal per query: h1={same1.tolist()}")


def run_norag_case(name, d, layers, heads, B, n_sites, n_ref=8, level=4, seed=0, epoch=2024, w=0):
    """configs[0]: the same model with no retrieved embeddings in the batch (bert.py:207-210:
    emb_fusion only, no rag_fusion)."""
    torch.set_num_threads(8)
    vocab = ref_vocab()
    model, digest = build_model(d, layers, heads, len(vocab), seed)
    win = synthetic.SynthWindow(n_sites, n_ref, B, seed=seed + 17)
    x = make_inputs(win, vocab, level, epoch, w)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    logits = []
    hook = model.hap_classifier.net.register_forward_hook(lambda m, i, o: logits.append(o.detach().clone()))
    with torch.no_grad():
        out = model({key: T(x[key]) for key in ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom")})
    hook.remove()
    res = dict(cfg=np.array(json.dumps(dict(d=d, layers=layers, heads=heads, vocab=len(vocab), B=B,
                                              n_sites=n_sites, n_ref=n_ref, k=0, level=level, seed=seed,
                                              epoch=epoch, w=w, sd_digest=digest))),
               probs_h1=out[0].numpy(), probs_h2=out[1].numpy(), gt=out[2].numpy(),
               logits_h1=logits[0].numpy(), logits_h2=logits[1].numpy())
    for key in ("hap_1", "hap_2", "mask", "raw_mask", "af", "af_p", "pos", "ref", "het", "hom"):
        res[key] = x[key]
    np.savez_compressed(OUT / f"{name}.npz", **res)
    print(f"{name}: digest={digest}")


class _FlatL2:
    """Stand-in for ``faiss.IndexFlatL2`` (faiss is not installed here): the published
    semantics of that index — exact brute-force k-NN on squared L2 over the added rows —
    evaluated in float64, ties to the lower row id.  Every search is logged."""
    log: list = []

    def __init__(self, d):
        self.d, self.xb = d, np.zeros((0, d), np.float32)

    def add(self, x):
        self.xb = np.concatenate([self.xb, np.asarray(x, np.float32)])

    def search(self, q, k):
        xb = self.xb.astype(np.float64)
        dist = np.stack([((xb - r.astype(np.float64)[None]) ** 2).sum(1) for r in np.asarray(q)])
        idx = np.arange(xb.shape[0])
        I = np.stack([np.lexsort((idx, d)) for d in dist])[:, :k].astype(np.int64)
        _FlatL2.log.append((I, dist))
        return np.take_along_axis(dist, I, 1).astype(np.float32), I


def _faiss_standin():
    store = {}
    return SimpleNamespace(IndexFlatL2=_FlatL2, StandardGpuResources=lambda: None,
                           write_index=lambda index, path: store.__setitem__(path, index),
                           read_index=lambda path: store[path], index_cpu_to_gpu=lambda res, dev, index: index)


def run_infer_case(name, d, layers, heads, n_sites, n_samples, n_ref_samples, k, batch_size, seed=0,
                   ref_missing=2, compact=False, missing_rate=0.3):
    """The reference imputation path end to end on synthetic arrays: InferDataset
    (dataset.py:629-900), EmbeddingRAGInferDataset (embedding_rag_infer_dataset.py:20-324:
    510-site index windows, infer masks, panel embeddings, process_batch_retrieval) with the
    FAISS stand-in above, WindowMajorSampler + embedding_rag_collate_fn, and the inference
    loop + geometry statements of infer_embedding_rag.py:129-203 executed as written."""
    import os
    import tempfile
    import time
    from typing import Dict, List, Optional
    from torch.utils.data import DataLoader, Dataset
    torch.set_num_threads(8)
    vocab = ref_vocab()
    model, digest = build_model(d, layers, heads, len(vocab), seed)
    a = synthetic.make_infer_arrays(n_sites, n_samples, n_ref_samples, missing_rate=missing_rate,
                                    ref_missing=ref_missing, seed=seed + 5)
    vpm = SimpleNamespace(sequence_padding=seq_pad, position_normalize=pos_norm)
    glb = dict(NP_GLB, Dataset=Dataset, math=math, INFER_WINDOW_LEN=1020, REF=0, HET=1, HOM=2, AF=3, GLOBAL=5,
               VCFProcessingModule=vpm, WordVocab=WordVocabRef)
    RefInfer = ref_classes("src/dataset/dataset.py", ["InferDataset"], glb)["InferDataset"]
    glb2 = dict(NP_GLB, InferDataset=RefInfer, faiss=_faiss_standin(), os=os, time=time, tqdm=lambda it, **kw: it,
                VCFProcessingModule=vpm, INFER_WINDOW_LEN=510, Dict=Dict, List=List, Optional=Optional)
    RefRAGInfer = ref_classes("src/dataset/embedding_rag_infer_dataset.py", ["EmbeddingRAGInferDataset"],
                              glb2)["EmbeddingRAGInferDataset"]
    collate = ref_function("src/dataset/embedding_rag_dataset.py", None, "embedding_rag_collate_fn", NP_GLB)

    class _Infer(RefRAGInfer):                     # the panel arrays instead of an h5/VCF file
        def _load_ref_data(self, ref_vcf_path):
            return a["ref_gt"], a["ref_pos"]

    emb = model.bert.embedding
    panel = SimpleNamespace(pop_list=np.array(a["pops"]))
    cwd = os.getcwd()
    _FlatL2.log.clear()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)                              # the reference writes its index dir relative to the CWD
        try:
            ds = _Infer(vocab, a["vcf"], a["pos"], panel, a["freq"], {}, a["pop_to_idx"], a["pos_to_idx"],
                        ref_vcf_path="panel", embedding_layer=emb, build_ref_data=True, build_index=True)
        finally:
            os.chdir(cwd)
        n_index_searches = len(_FlatL2.log)
        items = [ds[i] for i in range(len(ds))]
        order = list(iter(WindowMajorSampler(ds)))
        batches = []
        loader = DataLoader(ds, batch_size=batch_size, sampler=WindowMajorSampler(ds), collate_fn=collate)

        class _Rec:                                # model(batch) with its outputs kept
            def __init__(self, m):
                self.m, self.bert, self.outs = m, m.bert, []

            def __call__(self, b):
                batches.append({key: (v.clone() if torch.is_tensor(v) else v) for key, v in b.items()})
                o = self.m(b)
                self.outs.append(o)
                return o
        rec = _Rec(model)
        text, tree = _source(REF / "src/infer_embedding_rag.py")
        fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "infer")
        body = [n for n in fn.body if 129 <= n.lineno <= 203]
        lines = text.splitlines()
        src = textwrap.dedent("\n".join(lines[body[0].lineno - 1:body[-1].end_lineno]))
        ns = dict(NP_GLB, infer_data_loader=loader, device=torch.device("cpu"), infer_dataset=ds,
                  embedding_layer=emb, args=SimpleNamespace(k_retrieve=k), model=rec, tqdm=lambda it, **kw: it,
                  time=time, INFER_WINDOW_LEN=1020)
        exec(compile(src, "src/infer_embedding_rag.py:129-203", "exec"), ns)
    # neighbours per query haplotype, in sampler order (process_batch_retrieval groups each batch by
    # window in first-appearance order and searches h1 then h2 per group, :256-285)
    log = _FlatL2.log[n_index_searches:]
    I1 = np.zeros((len(order), k), np.int64)
    I2 = np.zeros_like(I1)
    D1 = np.zeros((len(order), n_ref_samples * 2))
    D2 = np.zeros_like(D1)
    row = 0
    for b in batches:
        groups = defaultdict(list)
        for i, w in enumerate(b["window_idx"]):
            groups[int(w)].append(i)
        for w, rows in groups.items():
            (i1, d1), (i2, d2) = log.pop(0), log.pop(0)
            for j, r in enumerate(rows):
                I1[row + r], I2[row + r], D1[row + r], D2[row + r] = i1[j], i2[j], d1[j], d2[j]
        row += len(b["window_idx"])
    probs1 = np.concatenate([o[0].detach().numpy() for o in rec.outs])
    probs2 = np.concatenate([o[1].detach().numpy() for o in rec.outs])
    res = dict(cfg=np.array(json.dumps(dict(d=d, layers=layers, heads=heads, vocab=len(vocab), k=k, seed=seed,
                                              batch_size=batch_size, n_samples=n_samples, index_window_len=510,
                                              missing_rate=missing_rate, n_ref_samples=n_ref_samples,
                                              window_len=1020, sd_digest=digest, pops=a["pops"]))),
               ori_pos=a["ori_pos"], pos=a["pos"], vcf=a["vcf"], freq=a["freq"], ref_gt=a["ref_gt"],
               ref_pos=a["ref_pos"], order=np.array(order),
               infer_masks=np.stack(ds.infer_masks).astype(np.int8),
               ref_tokens_complete=np.stack(ds.ref_tokens_complete).astype(np.int8),
               ref_af_windows=np.stack(ds.ref_af_windows).astype(np.float32),
               I_h1=I1, I_h2=I2, kth_margin_h1=_kth_margin(D1, k), kth_margin_h2=_kth_margin(D2, k),
               batch_probs_h1=probs1, batch_probs_h2=probs2,
               hap1=ns["hap1"], hap2=ns["hap2"], gt=ns["gt"], mask=ns["mask"])
    if compact:
        # batch-size case: keep the inputs, the neighbours and the imputed haplotype
        # probabilities (float16); GP follows from them (checked on the full case)
        for key in ("batch_probs_h1", "batch_probs_h2", "gt", "ref_tokens_complete"):
            res.pop(key)
        res["hap1"], res["hap2"] = res["hap1"].astype(np.float16), res["hap2"].astype(np.float16)
        res["mask"] = res["mask"].astype(np.int8)
    else:
        for key in ("hap_1", "hap_2", "mask", "af", "af_p", "pos", "ref", "het", "hom", "window_idx", "sample_idx",
                    "start_idx", "end_idx"):
            res[f"item_{key}"] = np.stack([np.asarray(it[key]) for it in items])
    np.savez_compressed(OUT / f"{name}.npz", **res)
    print(f"{name}: digest={digest} items={len(items)} windows={ds.window_count} "
          f"min kth margin h1={res['kth_margin_h1'].min():.3g} h2={res['kth_margin_h2'].min():.3g}")


def pickled_module_case():
    """The checkpoint object the reference trainer writes (pretrain_with_val_optimized.py:531-536:
    ``torch.save(self.model.cpu(), path)``, a pickled BERTFoundationModel naming the reference's
    classes) for the fwd_tiny weights (d64 / 2 layers / 2 heads, seed 0), plus the same model's
    state_dict as arrays for the converter test (tests/test_checkpoint_cpu.py)."""
    vocab = ref_vocab()
    model, digest = build_model(64, 2, 2, len(vocab), 0)
    model.train()                                  # as saved mid-training
    torch.save(model.cpu(), OUT / "ref_module_tiny.pth")
    sd = {k: v.detach().numpy() for k, v in model.state_dict().items()}
    np.savez_compressed(OUT / "ref_module_tiny_sd.npz", keys=np.array(json.dumps(list(sd))), digest=np.array(digest),
                        **{f"t{i}": v for i, v in enumerate(sd.values())})
    print(f"ref_module_tiny: {len(sd)} tensors digest={digest}")


def _kth_margin(dist, k):
    s = np.sort(dist, 1)
    return (s[:, k] - s[:, k - 1]) if s.shape[1] > k else np.full(s.shape[0], np.inf)


def masks_fixture():
    rng = np.random.default_rng(7)
    out = {}
    for n in (5, 128, 512, 1020):
        af = rng.beta(0.3, 3.0, n).astype(np.float32)
        out[f"af_{n}"] = af
        for level in (0, 4, 5):
            for seed in (0, 1, 2024):
                for w in (0, 3):
                    out[f"mask_{n}_{level}_{seed}_{w}"] = ref_mask(af, level, seed, w)
    # tokenisation (incl. non-biallelic values -> <unk>) and padding
    vocab = ref_vocab()
    fake = SimpleNamespace(vocab=vocab)
    seq = rng.integers(-1, 3, size=(3, 40))
    m = seq_pad((rng.random(40) < 0.4).astype(int), dtype="int")
    out["tok_seq"], out["tok_mask"] = seq, m
    out["tok_out"] = tokenize(fake, seq, m)
    out["vocab_itos"] = np.array(json.dumps([str(t) for t in vocab.itos]))
    pos = np.sort(rng.choice(10 ** 6, 300, replace=False))
    out["pos_in"], out["pos_out"] = pos, seq_pad(pos_norm(pos), dtype="float")
    # samplers
    class _DS:  # minimal dataset for the samplers
        window_count = 7
        def __len__(self): return 7 * 5
    gs = WindowGroupedSampler(_DS(), shuffle=True, seed=42)
    out["grouped_sampler_ep0"] = np.array(list(iter(gs)))
    gs.set_epoch(1)
    out["grouped_sampler_ep1"] = np.array(list(iter(gs)))
    out["major_sampler"] = np.array(list(iter(WindowMajorSampler(_DS()))))
    np.savez_compressed(OUT / "data_contract.npz", **out)
    print("data_contract: ok")


if __name__ == "__main__":
    which = sys.argv[1:] or ["data", "tiny", "small", "full", "norag", "infer", "infer256", "infer384", "sweep",
                             "pickled"]
    if "data" in which:
        masks_fixture()
    if "tiny" in which:
        run_case("fwd_tiny", d=64, layers=2, heads=2, B=2, n_sites=100, n_ref=48, k=4,
                 keep_intermediate=True)
    if "small" in which:
        run_case("fwd_small", d=128, layers=2, heads=4, B=3, n_sites=300, n_ref=96, k=8, seed=1)
    if "full" in which:
        run_case("fwd_full", d=384, layers=12, heads=12, B=2, n_sites=1020, n_ref=64, k=4, seed=2)
    if "norag" in which:
        run_norag_case("fwd_norag", d=128, layers=2, heads=4, B=3, n_sites=128, seed=4)
    if "infer" in which:
        run_infer_case("infer_c5", d=64, layers=2, heads=4, n_sites=1300, n_samples=3, n_ref_samples=24, k=2,
                       batch_size=4, seed=6)
    if "infer256" in which:
        # C5 geometry: one batch of 256 sample-windows spanning both windows
        run_infer_case("infer_c5_b256", d=64, layers=2, heads=4, n_sites=1300, n_samples=128, n_ref_samples=24,
                       k=2, batch_size=256, seed=7, compact=True)
    if "infer384" in which:
        # the v18 model shape (d384 / 12 layers / 12 heads) through the whole imputation path
        run_infer_case("infer_c5_d384", d=384, layers=12, heads=12, n_sites=1300, n_samples=4, n_ref_samples=24,
                       k=2, batch_size=8, seed=8)
    if "pickled" in which:
        pickled_module_case()
    if "sweep" in which:
        # C5 mask sweep end points (10 % and 90 % of the panel sites missing from the target)
        for rate, tag in ((0.1, "m10"), (0.9, "m90")):
            run_infer_case(f"infer_c5_{tag}", d=64, layers=2, heads=4, n_sites=1300, n_samples=6, n_ref_samples=24,
                           k=2, batch_size=12, seed=9, missing_rate=rate, compact=True)
