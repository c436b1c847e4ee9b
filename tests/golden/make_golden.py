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
    which = sys.argv[1:] or ["data", "tiny", "small", "full", "norag"]
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
