"""Deterministic synthetic haplotype windows, reference panels and model weights.

There is no network on the build or GPU boxes, so no 1000-Genomes data and no
trained checkpoints.  Everything the tests, ``bench.py`` and ``smoke()`` feed
the hot path comes from here, seeded, with the distributions SURVEY.md §8(d)
fixes:

* site allele frequency  AF ~ Beta(0.3, 3.0)  (≈59 % of sites have AF < 0.05),
* reference haplotypes   Bernoulli(AF) per site,
* query haplotypes       a panel haplotype copied with a small flip rate, so
                         retrieval has a real nearest neighbour (LD-like),
* population AF          AF + N(0, 0.05) clipped, genotype freqs from HWE.

``synth_state_dict`` produces model weights keyed exactly like the
reference's ``BERTFoundationModel.state_dict()`` (keys listed by
``src/model/foundation_model.py`` + ``src/model/bert.py``), one independent
RNG stream per key, so the golden-fixture script (which loads them into the
reference's own modules) and the GPU box (which loads them into ours) see
bit-identical parameters without shipping a checkpoint.
"""

from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

MAX_SEQ_LEN = 1030  # reference: src/dataset/dataset.py:27


# --------------------------------------------------------------------------- #
# weights
# --------------------------------------------------------------------------- #
def _key_rng(key: str, seed: int) -> np.random.Generator:
    return np.random.default_rng([int(seed), zlib.crc32(key.encode()) & 0xFFFFFFFF])


def sinusoid_table(max_len: int, dims: int) -> np.ndarray:
    """Positional table with the formula of src/model/embedding/position.py:24-35,
    evaluated in float64 and rounded once to float32."""
    pe = np.zeros((max_len, dims), dtype=np.float64)
    position = np.arange(max_len, dtype=np.float64)[:, None]
    div_term = np.exp(np.arange(0, dims, 2, dtype=np.float64) * -(math.log(10000.0) / dims))
    pe[:, 0::2] = np.sin(position * div_term)
    pe[:, 1::2] = np.cos(position * div_term)
    return pe.astype(np.float32)[None]


def synth_tensor(key: str, shape: Tuple[int, ...], seed: int = 0, dtype=np.float32) -> np.ndarray:
    """One parameter/buffer, chosen by its state_dict key and shape."""
    rng = _key_rng(key, seed)
    shape = tuple(int(s) for s in shape)
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "pe":
        return sinusoid_table(shape[1], shape[2])
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "basis_freqs":
        base = np.logspace(0.0, 2.0, shape[0])
        return (base * (1.0 + 0.01 * rng.standard_normal(shape))).astype(dtype)
    if leaf == "running_mean":
        return (0.1 * rng.standard_normal(shape)).astype(dtype)
    if leaf == "running_var":
        return (0.5 + rng.random(shape)).astype(dtype)
    if leaf == "res_scale":
        return np.asarray(0.1 + 0.05 * rng.standard_normal(), dtype=dtype).reshape(shape)
    if key.endswith("tokenizer.weight"):
        w = rng.standard_normal(shape).astype(dtype)
        w[0] = 0.0  # padding_idx=0 row stays zero (nn.Embedding(padding_idx=0))
        return w
    if leaf == "bias":
        return (0.05 * rng.standard_normal(shape)).astype(dtype)
    if leaf == "weight":
        if len(shape) == 1:  # LayerNorm / BatchNorm scale
            return (1.0 + 0.1 * rng.standard_normal(shape)).astype(dtype)
        if len(shape) == 2:  # Linear [out, in]: xavier-normal scale
            std = math.sqrt(2.0 / (shape[0] + shape[1]))
            return (std * rng.standard_normal(shape)).astype(dtype)
        if len(shape) == 3:  # Conv1d [out, in, k]
            std = 1.0 / math.sqrt(shape[1] * shape[2])
            return (std * rng.standard_normal(shape)).astype(dtype)
    return (0.05 * rng.standard_normal(shape)).astype(dtype)


def synth_state_dict(shapes: Dict[str, Tuple[int, ...]] | Iterable[Tuple[str, Tuple[int, ...]]],
                     seed: int = 0) -> Dict[str, np.ndarray]:
    items = shapes.items() if isinstance(shapes, dict) else shapes
    return {k: synth_tensor(k, tuple(s), seed) for k, s in items}


def state_dict_digest(sd: Dict[str, np.ndarray]) -> str:
    """Order-independent crc of every tensor's bytes (fixture drift check)."""
    acc = 0
    for k in sorted(sd):
        v = np.ascontiguousarray(np.asarray(sd[k]))
        acc = zlib.crc32(k.encode(), acc)
        acc = zlib.crc32(v.tobytes(), acc)
    return f"{acc:08x}"


# --------------------------------------------------------------------------- #
# haplotype windows
# --------------------------------------------------------------------------- #
class SynthWindow:
    """One window of ``n_sites`` biallelic sites with a reference panel and query samples.

    Attributes (numpy):
      af        f32 [n_sites]       global AF (Freq.npy[AF][GLOBAL] restated)
      pos       i64 [n_sites]       sorted physical positions
      panel     u8  [n_ref, n_sites] reference haplotypes (alleles 0/1)
      query     u8  [n_samples, 2, n_sites] query haplotypes (hap_1, hap_2)
      af_p      f32 [n_samples, n_sites]   population AF per sample
      ref/het/hom f32 [n_samples, n_sites] HWE genotype frequencies of af_p
      source    i64 [n_samples, 2]  panel row each query haplotype was copied from
    """

    def __init__(self, n_sites: int, n_ref: int, n_samples: int, seed: int = 0,
                 flip_rate: float = 0.02, pos_span: int = 50):
        rng = np.random.default_rng([int(seed), 0x5A17])
        self.n_sites, self.n_ref, self.n_samples = n_sites, n_ref, n_samples
        self.af = rng.beta(0.3, 3.0, n_sites).astype(np.float32)
        self.pos = np.sort(rng.choice(np.arange(1, pos_span * n_sites + 2), n_sites,
                                      replace=False)).astype(np.int64)
        self.panel = (rng.random((n_ref, n_sites)) < self.af[None]).astype(np.uint8)
        src = rng.integers(0, n_ref, size=(n_samples, 2))
        flips = rng.random((n_samples, 2, n_sites)) < flip_rate
        self.query = (self.panel[src] ^ flips).astype(np.uint8)
        self.source = src.astype(np.int64)
        afp = np.clip(self.af[None] + 0.05 * rng.standard_normal((n_samples, n_sites)), 0.0, 1.0)
        self.af_p = afp.astype(np.float32)
        self.ref = ((1 - afp) ** 2).astype(np.float32)
        self.het = (2 * afp * (1 - afp)).astype(np.float32)
        self.hom = (afp ** 2).astype(np.float32)


def hash_uniform(seed: int, row: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Counter-based U[0,1) used by the on-device panel generator
    (csrc/knn.hip ``panel_synth_kernel``): splitmix64 of (seed, row, col),
    top 24 bits / 2^24.  Restated here so small panels can be checked on CPU."""
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
             + row.astype(np.uint64) * np.uint64(0xD1B54A32D192ED03)
             + col.astype(np.uint64) * np.uint64(0x8CB92BA72F3D8DD7))
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(40)).astype(np.float64) / float(1 << 24)


POPS = ["AFR", "AMR", "EAS", "EUR", "SAS"]


def make_rag_dataset(n_samples: int = 8, n_sites: int = 512, n_windows: int = 2, n_ref_samples: int = 64,
                     seed: int = 0, name: str = "val"):
    """In-memory EmbeddingRAGDataset over synthetic data with the reference's file
    contract (GT [sites, samples, 2], Freq.npy [4, n_pop+1, sites], window bounds,
    pop_to_idx / pos_to_idx).  Returns (dataset, vocab)."""
    from .embedding_rag_dataset import EmbeddingRAGDataset
    from .vocab import WordVocab
    rng = np.random.default_rng([seed, 0xDA7A])
    S = n_sites * n_windows
    af = rng.beta(0.3, 3.0, S).astype(np.float32)
    pos = np.sort(rng.choice(np.arange(1, 50 * S), S, replace=False)).astype(np.int64)
    ref = (rng.random((S, n_ref_samples, 2)) < af[:, None, None]).astype(np.int8)
    src = rng.integers(0, n_ref_samples, size=(n_samples, 2))
    vcf = np.stack([ref[:, src[:, 0], 0], ref[:, src[:, 1], 1]], -1)
    vcf = vcf ^ (rng.random(vcf.shape) < 0.02)
    pops = [POPS[i % 5] for i in range(n_samples)]
    freq = np.zeros((4, 6, S), np.float32)
    for p in range(6):
        ap = np.clip(af + (0.05 * rng.standard_normal(S) if p < 5 else 0), 0, 1)
        freq[0, p], freq[1, p], freq[2, p], freq[3, p] = (1 - ap) ** 2, 2 * ap * (1 - ap), ap ** 2, ap
    freq[3, 5] = af
    vocab = WordVocab(POPS)
    bounds = np.array([[w * n_sites, (w + 1) * n_sites] for w in range(n_windows)])
    ds = EmbeddingRAGDataset.from_arrays(vocab, vcf.astype(np.int8), pos, pops, freq, bounds,
                                         {p: i for i, p in enumerate(POPS)},
                                         {int(p): i for i, p in enumerate(pos)}, ref, pos, name=name)
    return ds, vocab


def make_infer_arrays(n_sites: int = 1300, n_samples: int = 3, n_ref_samples: int = 24, missing_rate: float = 0.3,
                      ref_missing: int = 0, seed: int = 0) -> dict:
    """In-memory imputation inputs with the reference's file contract (InferDataset.from_file,
    dataset.py:747-771; the panel of embedding_rag_infer_dataset.py:56-69):

      ori_pos / pos_to_idx  every panel site (Freq.npy columns), sorted positions;
      pos, vcf              the target VCF: the sites kept with probability 1 - missing_rate,
                            GT [n_target, n_samples, 2] copied from panel haplotypes + 2 % flips;
      ref_gt, ref_pos       the reference panel [n_ref_sites, n_ref_samples, 2]; ``ref_missing``
                            panel sites dropped from it (windows with unmatched sites);
      freq                  [4, 6, n_sites] (REF, HET, HOM, AF x 5 populations + GLOBAL)."""
    rng = np.random.default_rng([seed, 0x1F3A])
    af = rng.beta(0.3, 3.0, n_sites).astype(np.float32)
    ori_pos = np.sort(rng.choice(np.arange(1, 50 * n_sites), n_sites, replace=False)).astype(np.int64)
    panel = (rng.random((n_sites, n_ref_samples, 2)) < af[:, None, None]).astype(np.int8)
    src = rng.integers(0, n_ref_samples, size=(n_samples, 2))
    full = np.stack([panel[:, src[:, 0], 0], panel[:, src[:, 1], 1]], -1)
    full = (full ^ (rng.random(full.shape) < 0.02)).astype(np.int8)
    keep = rng.random(n_sites) >= missing_rate
    keep[0] = True                                       # a target VCF with at least one site
    freq = np.zeros((4, 6, n_sites), np.float32)
    for p in range(6):
        ap = np.clip(af + (0.05 * rng.standard_normal(n_sites) if p < 5 else 0), 0, 1)
        freq[0, p], freq[1, p], freq[2, p], freq[3, p] = (1 - ap) ** 2, 2 * ap * (1 - ap), ap ** 2, ap
    ref_rows = np.arange(n_sites)
    if ref_missing:
        drop = rng.choice(np.arange(1, n_sites), ref_missing, replace=False)
        ref_rows = np.setdiff1d(ref_rows, drop)
    return dict(ori_pos=ori_pos, pos=ori_pos[keep], vcf=full[keep], freq=freq,
                pops=[POPS[i % 5] for i in range(n_samples)], pop_to_idx={p: i for i, p in enumerate(POPS)},
                pos_to_idx={int(p): i for i, p in enumerate(ori_pos)}, ref_gt=panel[ref_rows],
                ref_pos=ori_pos[ref_rows], source=src)


def make_infer_dataset(a: dict = None, index_window_len: int = 510, **kw):
    """EmbeddingRAGInferDataset over ``make_infer_arrays`` data (or ``a``).  Returns (dataset, vocab)."""
    from .embedding_rag_infer_dataset import EmbeddingRAGInferDataset
    from .vocab import WordVocab
    a = a if a is not None else make_infer_arrays(**kw)
    vocab = WordVocab(POPS)
    ds = EmbeddingRAGInferDataset.from_arrays(vocab, a["vcf"], a["pos"], a["pops"], a["freq"], a["pop_to_idx"],
                                              a["pos_to_idx"], a["ref_gt"], a["ref_pos"],
                                              index_window_len=index_window_len)
    return ds, vocab
