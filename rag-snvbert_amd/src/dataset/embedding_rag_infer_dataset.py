"""EmbeddingRAGInferDataset — v18 imputation dataset with panel retrieval
(reference: src/dataset/embedding_rag_infer_dataset.py).

Drop-in surface (SURVEY.md §8b, row "Retrieval (infer)"):
  * ``process_batch_retrieval(batch, embedding_layer, device, k_retrieve=1) -> batch``
    with ``batch['window_idx']`` a list of 0-d tensors (:250-324); adds ``rag_emb_h1/h2``
    (the K-mean as [B, 1, L, D], see embedding_rag_dataset.py) and ``rag_idx_h1/h2``;
  * ``__getitem__`` = InferDataset's item with the window's infer mask (:226-248);
  * ``infer_masks``, ``raw_window_masks``, ``ref_tokens_complete``, ``ref_af_windows``.

Index windows.  The reference builds its per-window indexes over windows of
INFER_WINDOW_LEN = 510 panel sites (:16, :100-102) while the items it searches with are
the parent's 1020-site windows (dataset.py:26, :823): for w > 0 the index sites, the
infer mask and the query sites are different stretches of the chromosome.
``index_window_len`` selects the semantics:
  * 510 (default, ``REFERENCE_INDEX_WINDOW``): the reference's behaviour, kept so a
    drop-in run reproduces the reference's outputs;
  * ``window_len`` (1020): index windows = query windows, masks = the sites each
    query actually lacks (the aligned design).

Index.  In place of one FAISS ``IndexFlatL2(L*D)`` of fp32 embeddings per window
(:176-181, exact L2 — the same semantics as the train path's cdist + topk), the
window's panel allele codes go to HBM once (``PanelIndex``) and the exact kNN runs on
the LUT decomposition of the same L2 distance (retrieval/, csrc/knn.hip).  The index
masks the panel's tokens at the window's infer-mask sites exactly as the reference's
``ref_tokens_masked`` (:152-155); since the query AF rows (the query window's sites)
differ from the index AF rows, the search takes the exact A_q != A_r LUT form.
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch

from .dataset import INFER_WINDOW_LEN, InferDataset, PanelData
from .embedding_rag_dataset import panel_index_of, retrieve
from .utils import MAX_SEQ_LEN, sequence_padding

REFERENCE_INDEX_WINDOW = 510     # embedding_rag_infer_dataset.py:16


class EmbeddingRAGInferDataset(InferDataset):
    def __init__(self, vocab, vcf, pos, panel, freq, type_to_idx, pop_to_idx, pos_to_idx,
                 ref_vcf_path=None, embedding_layer=None, build_ref_data: bool = True, n_gpu: int = 1,
                 build_index: bool = True, name: str = "infer", ref_gt: Optional[np.ndarray] = None,
                 ref_pos: Optional[np.ndarray] = None, index_window_len: int = REFERENCE_INDEX_WINDOW,
                 window_len: int = INFER_WINDOW_LEN, index_cache_bytes: int = 64 << 30):
        super().__init__(vocab, vcf, pos, panel, freq, type_to_idx, pop_to_idx, pos_to_idx, window_len=window_len)
        self.embedding_layer = embedding_layer
        self.embed_dim = embedding_layer.embed_size if embedding_layer is not None else 384
        self.index_window_len = int(index_window_len)
        self.name = name
        self.ref_tokens_complete: List[np.ndarray] = []
        self.ref_alleles: List[np.ndarray] = []
        self.ref_af_windows: List[np.ndarray] = []
        self.infer_masks: List[np.ndarray] = []        # query masks per window (padded, :117)
        self.raw_window_masks: List[np.ndarray] = []
        self.index_masks: List[np.ndarray] = []        # panel-token masks per window (padded, :152-155)
        self.index_sites: List[np.ndarray] = []        # ori_pos rows of each index window's panel sites
        self.jit_cache_win_idx = -1
        self._index_cache: "OrderedDict[int, object]" = OrderedDict()
        self._index_cache_bytes = index_cache_bytes
        if ref_gt is None and ref_vcf_path is not None and build_ref_data and build_index:
            ref_gt, ref_pos = self._load_ref_data(ref_vcf_path)
        if build_ref_data and build_index and ref_gt is not None:
            self._build_embedding_indexes(ref_gt, ref_pos)

    # ---------------------------------------------------------------- panel --
    @staticmethod
    def _load_ref_data(ref_vcf_path: str):
        """:56-69 (h5 or VCF panel)."""
        try:
            import h5py
        except ImportError as e:
            raise RuntimeError("reading the reference panel needs h5py (not installed here); "
                               "pass ref_gt / ref_pos arrays") from e
        with h5py.File(ref_vcf_path, "r") as f:
            return f["gt"][:], f["variants/POS"][:]

    def _build_embedding_indexes(self, ref_gt: np.ndarray, ref_pos: np.ndarray) -> None:
        """:71-207 without the embedding pass: per window, the infer mask (site absent from the
        target), the panel rows of the window's sites (first occurrence of each position,
        :93-96), the global AF (:141-150) and the complete panel tokens (:157-159)."""
        ref_pos = np.asarray(ref_pos)
        first = {}
        for i, p in enumerate(ref_pos.tolist()):
            first.setdefault(p, i)
        IW = self.index_window_len
        for w in range(self.window_count):                 # the parent's window count (:100)
            start = IW * w
            end = min(start + IW, self.ori_pos.shape[0])
            mask = self.position_needed[start:end].astype(np.int64)
            n = len(mask)
            self.raw_window_masks.append(mask.copy())
            self.infer_masks.append(sequence_padding(np.pad(mask, (0, max(IW - n, 0))), "int"))
            cur = self.ori_pos[start:end]
            ref_rows = np.array([first.get(p, -1) for p in cur.tolist()], dtype=np.int64)
            keep = np.nonzero(ref_rows >= 0)[0]
            if len(keep) == 0:
                # the reference `continue`s here (:130-132), which shifts every later window's
                # index by one; refuse instead of imputing against the wrong window
                raise ValueError(f"infer window {w}: none of its sites is in the reference panel")
            mask, cur, ref_rows = mask[keep], cur[keep], ref_rows[keep]
            self.index_sites.append(start + keep)
            cols = np.array([self.pos_to_idx.get(p, -1) for p in cur.tolist()], dtype=np.int64)
            af = np.where(cols >= 0, self.freq[3][5][np.maximum(cols, 0)], 0.0).astype(np.float32)
            self.ref_af_windows.append(sequence_padding(af, "float").astype(np.float32))
            self.index_masks.append(sequence_padding(mask, "int"))
            alleles = np.asarray(ref_gt[ref_rows]).reshape(len(ref_rows), -1).T     # [n_haps, n_sites]
            self.ref_alleles.append(alleles.astype(np.int64))
            self.ref_tokens_complete.append(self.tokenize(alleles, np.zeros(MAX_SEQ_LEN, np.int64)))

    panel_shard = None

    def set_panel_shard(self, shard) -> None:
        """See EmbeddingRAGDataset.set_panel_shard (the infer masks are deterministic: no sync)."""
        self.panel_shard = shard
        self._index_cache.clear()

    def panel_index(self, w: int, device) -> "object":
        idx = self._index_cache.get(w)
        if idx is None or idx.codes.device != torch.device(device):
            idx = panel_index_of(self.ref_alleles[w], self.ref_af_windows[w], device, self.panel_shard)
            self._index_cache[w] = idx
            while sum(i.nbytes for i in self._index_cache.values()) > self._index_cache_bytes and \
                    len(self._index_cache) > 1:
                self._index_cache.popitem(last=False)
        else:
            self._index_cache.move_to_end(w)
        self.jit_cache_win_idx = w
        return idx

    load_index = panel_index                           # :209-224 (cached per window)

    # ----------------------------------------------------------------- items --
    def __getitem__(self, item: int) -> dict:
        """:226-248: the parent's item re-masked with the window's infer mask."""
        out = super().__getitem__(item)
        w = item % self.window_count
        m = self.infer_masks[w]
        out["mask"] = torch.as_tensor(m, dtype=torch.long)
        out["window_idx"] = torch.tensor(w, dtype=torch.long)
        out["hap_1"] = torch.as_tensor(self.tokenize(out["hap1_nomask"].numpy(), m), dtype=torch.long)
        out["hap_2"] = torch.as_tensor(self.tokenize(out["hap2_nomask"].numpy(), m), dtype=torch.long)
        return out

    # ------------------------------------------------------------- retrieval --
    def process_batch_retrieval(self, batch: dict, embedding_layer, device, k_retrieve: int = 1,
                                dense: bool = False, limbs: int = 2) -> dict:
        return retrieve(self, batch, embedding_layer, device, k_retrieve, self.index_masks, dense, limbs)

    @classmethod
    def from_file(cls, vocab, vcfpath, panelpath, freqpath, typepath, poppath, pospath, ref_vcf_path=None,
                  embedding_layer=None, build_ref_data=True, n_gpu=1, name="infer", **kw):
        base = InferDataset.from_file(vocab, vcfpath, panelpath, freqpath, typepath, poppath, pospath)
        return cls(vocab, base.vcf, base.pos, base.panel, base.freq, base.type_to_idx, base.pop_to_idx,
                   base.pos_to_idx, ref_vcf_path=ref_vcf_path, embedding_layer=embedding_layer,
                   build_ref_data=build_ref_data, n_gpu=n_gpu, name=name, **kw)

    @classmethod
    def from_arrays(cls, vocab, vcf, pos, pop_list, freq, pop_to_idx, pos_to_idx, ref_gt, ref_pos,
                    embedding_layer=None, name="infer", type_to_idx=None, **kw) -> "EmbeddingRAGInferDataset":
        return cls(vocab, vcf, pos, PanelData(pop_list), freq, type_to_idx or {}, pop_to_idx, pos_to_idx,
                   embedding_layer=embedding_layer, name=name, ref_gt=ref_gt, ref_pos=ref_pos, **kw)
