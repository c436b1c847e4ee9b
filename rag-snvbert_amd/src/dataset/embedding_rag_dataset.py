"""EmbeddingRAGDataset — v18 training/validation dataset with panel retrieval
(reference: src/dataset/embedding_rag_dataset.py).

Drop-in surface:
  * ``process_batch_retrieval(batch, embedding_layer, device, k_retrieve=1) -> batch``
    adds ``rag_emb_h1`` / ``rag_emb_h2`` on ``device``.  The reference fills a dense
    [B, k, L, D] tensor and the model immediately takes its mean over k
    (model/bert.py:176-179); here the K-mean is produced directly by the
    ``rag_mean`` kernel as [B, 1, L, D] — the model consumes it identically
    (bert.py:180-182) — and ``rag_idx_h1/h2`` [B, k] carry the neighbour indices.
    ``dense=True`` returns the reference's fp32 [B, k, L, D] neighbour embeddings
    (the model's mean over k then equals the K-mean path).
    Train mode (``embedding_layer.training``, :404-442): ``rag_emb_h1/h2`` are f32 and
    autograd-connected to the embedding parameters — each window's unique neighbours
    re-encoded once with the layer's dropout (``train_forward.neighbour_embeddings``) — so
    the reference trainer's hand-off of just those two keys
    (pretrain_with_val_optimized.py:192-195) trains through the retrieval; ``rag_groups``
    (the neighbour indices per window) rides along for inspection.
  * ``regenerate_masks(seed)``, ``clear_jit_cache()``, ``add_level()``,
    ``window_masks``, ``ref_tokens_complete``, ``ref_af_windows``, ``jit_cache_win_idx``.

Index: per window, the panel's allele codes are uploaded once to HBM
(``PanelIndex``); unlike the reference's fp32 embedding cache (:334-377) the
index does not depend on the mask or the weights, so a mask refresh or a weight
update never forces a rebuild.

Panel-embedding staleness (``panel_cache``).  The reference embeds a window's panel once,
in eval mode, when a batch of that window arrives and the cache holds another window
(``jit_cache_win_idx != win_idx``, :334-377; reset at every epoch start and by
``clear_jit_cache``), then keeps searching those embeddings while the weights train over the
window's following batches.  ``panel_cache="window"`` (default) reproduces that: on the same
trigger the token table W and the panel's AF embedding A_r are snapshotted (10 x D and L x D
floats instead of the reference's [n_haps, L, D] cache) and the search ranks the current
(dropped-out) query embeddings against the snapshot (``snvrag_knn_lut_panel``: panel side
W_snap, query side W).  ``panel_cache="fresh"`` searches the panel under the current weights
at every batch.  Eval mode (validation, inference) has no weight updates: both are the same.
"""

from __future__ import annotations

from collections import OrderedDict, defaultdict
from typing import Dict, List, Optional

import numpy as np
import torch

from ..train_forward import NeighbourGroup
from .dataset import PanelData, TrainDataset, Window
from .utils import mask_probs, sequence_padding
from .vocab import WordVocab

MAX_SEQ_LEN = 1030


class EmbeddingRAGDataset(TrainDataset):
    def __init__(self, vocab, vcf, pos, panel, freq, window, type_to_idx, pop_to_idx, pos_to_idx,
                 ref_gt: Optional[np.ndarray] = None, ref_pos: Optional[np.ndarray] = None,
                 embedding_layer=None, build_ref_data: bool = True, n_gpu: int = 1,
                 maf_mask_percentage: int = 10, use_dynamic_mask: bool = False, name: str = "default",
                 index_cache_bytes: int = 64 << 30, panel_cache: str = "window"):
        super().__init__(vocab, vcf, pos, panel, freq, window, type_to_idx, pop_to_idx, pos_to_idx)
        if panel_cache not in ("window", "fresh"):
            raise ValueError("panel_cache must be 'window' (the reference's per-window snapshot) or 'fresh'")
        self.panel_cache = panel_cache
        self._panel_snap = None          # (window, W snapshot, A_r snapshot, weights token) of the cached window
        self.maf_mask_percentage, self.use_dynamic_mask = maf_mask_percentage, use_dynamic_mask
        self.current_epoch, self.name = 0, name
        self.ref_tokens_complete: List[np.ndarray] = []
        self.ref_alleles: List[np.ndarray] = []
        self.raw_window_masks: List[np.ndarray] = []
        self.window_masks: List[np.ndarray] = []
        self.mask_version = 0
        self.ref_af_windows: List[np.ndarray] = []
        self.window_valid_indices: Dict[int, np.ndarray] = {}
        self.window_actual_lens: List[int] = []
        self.jit_cache_win_idx = -1
        self.embedding_layer = embedding_layer
        self.embed_dim = embedding_layer.embed_size if embedding_layer is not None else None
        self._index_cache: "OrderedDict[int, object]" = OrderedDict()
        self._index_cache_bytes = index_cache_bytes
        if build_ref_data and ref_gt is not None:
            self._load_ref_data_to_memory(ref_gt, ref_pos)

    # ---------------------------------------------------------------- panel --
    def _load_ref_data_to_memory(self, ref_gt: np.ndarray, ref_pos: np.ndarray) -> None:
        """embedding_rag_dataset.py:79-208: per-window site match, AF, AF-guided mask, complete tokens."""
        ref_pos = np.asarray(ref_pos)
        for w in range(self.window_count):
            sl = self._window_slice(w)
            train_pos = self.pos[sl]
            found = np.clip(np.searchsorted(ref_pos, train_pos), 0, len(ref_pos) - 1)
            is_match = ref_pos[found] == train_pos
            valid = np.where(is_match)[0]
            ref_idx = found[is_match]
            if len(ref_idx) < len(train_pos):
                if len(valid) == 0:
                    raise ValueError(f"window {w}: no panel sites (the reference skips it, which misaligns "
                                     "window ids; refusing)")
                train_pos = train_pos[valid]
                self.window_valid_indices[w] = valid
            n = len(train_pos)
            self.window_actual_lens.append(n)
            cols = np.array([self.pos_to_idx.get(p, -1) for p in train_pos])
            af = np.where(cols >= 0, self.freq[3][5][np.maximum(cols, 0)], 0.0).astype(np.float32)
            ref_af = sequence_padding(af, "float").astype(np.float32)
            self.ref_af_windows.append(ref_af)
            raw = self.generate_mask(n, probs=mask_probs(af, self._level))
            self.raw_window_masks.append(raw)
            self.window_masks.append(sequence_padding(raw, "int"))
            alleles = np.asarray(ref_gt[ref_idx]).reshape(len(ref_idx), -1).T   # [n_haps, n]
            self.ref_alleles.append(alleles.astype(np.int64))
            self.ref_tokens_complete.append(self.tokenize(alleles, np.zeros(MAX_SEQ_LEN, np.int64)))

    def clear_jit_cache(self) -> None:
        self.jit_cache_win_idx = -1
        self._panel_snap = None
        self._index_cache.clear()

    def regenerate_masks(self, seed: int) -> None:
        """embedding_rag_dataset.py:228-283 (np.random.seed(seed*10000 + w))."""
        self.mask_version += 1
        for w in range(self.window_count):
            n = self.window_actual_lens[w]
            probs = mask_probs(self.ref_af_windows[w][1:1 + n], self._level)
            np.random.seed(seed * 10000 + w)
            raw = self.generate_mask(n, probs=probs)
            self.raw_window_masks[w] = raw
            self.window_masks[w] = sequence_padding(raw, "int")

    def _apply_mask_to_tokens_gpu(self, tokens: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        out = tokens.clone()
        out[:, mask == 1] = self.vocab.mask_index
        return out

    # ----------------------------------------------------------------- items --
    def __getitem__(self, item: int) -> dict:
        """embedding_rag_dataset.py:486-555: seeded AF-guided mask per (epoch|2024, window).
        ``item >= len(self)``: a DistributedWindowSampler padding duplicate of item - len(self)
        — the same tokens (retrieval and forward run as usual) with an all-zero metric mask, so
        its sites enter no loss, F1 or accuracy."""
        if item >= len(self):
            out = self[item - len(self)]
            out["mask"] = torch.zeros_like(out["mask"])
            return out
        w = item % self.window_count
        # panel-filtered windows: featurise only the matched sites (the reference indexes its
        # padded arrays with the unpadded site filter here, :498-507, and raises KeyError on 'label')
        out = self.base_item(item, self.window_valid_indices.get(w))
        n = self.window_actual_lens[w]
        af = self.ref_af_windows[w][1:1 + n]
        seed = self.current_epoch if self.name == "train" else 2024
        old = np.random.get_state()
        np.random.seed(seed * 10000 + w)
        raw = self.generate_mask(n, probs=mask_probs(af, self._level))
        np.random.set_state(old)
        mask = sequence_padding(raw, "int")
        out["mask"] = mask
        out["hap_1"] = self.tokenize(out["hap1_nomask"], mask)
        out["hap_2"] = self.tokenize(out["hap2_nomask"], mask)
        return self.to_tensors(out)

    # ------------------------------------------------------------- retrieval --
    panel_shard = None

    def set_panel_shard(self, shard) -> None:
        """Hold only this rank's contiguous haplotype range of every window's panel
        (``retrieval.shards.PanelShard``; None = the whole panel).  process_batch_retrieval
        then runs the collective search — every rank must call it for every batch.

        A query's distances must not depend on which shard scores them, so every rank takes
        rank 0's window masks here (the construction-time masks come from the unseeded
        global RNG, embedding_rag_dataset.py:160-170; ``regenerate_masks(seed)`` is seeded
        and stays identical across ranks)."""
        self.panel_shard = shard
        self._index_cache.clear()
        if shard is not None:
            import torch.distributed as dist
            obj = [self.raw_window_masks if shard.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=shard.group)
            self.raw_window_masks = [np.asarray(m) for m in obj[0]]
            self.window_masks = [sequence_padding(m, "int") for m in self.raw_window_masks]
            self.mask_version += 1

    def panel_index(self, w: int, device) -> "object":
        from ..retrieval import PanelIndex
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

    def process_batch_retrieval(self, batch: dict, embedding_layer, device, k_retrieve: int = 1,
                                dense: bool = False, limbs: int = 2) -> dict:
        return retrieve(self, batch, embedding_layer, device, k_retrieve, self.window_masks, dense, limbs)

    @classmethod
    def from_arrays(cls, vocab, vcf, pos, pop_list, freq, window_bounds, pop_to_idx, pos_to_idx,
                    ref_gt, ref_pos, embedding_layer=None, name="default", type_to_idx=None) -> "EmbeddingRAGDataset":
        win = Window(np.asarray(window_bounds)[:, 0], np.asarray(window_bounds)[:, 1])
        return cls(vocab, vcf, pos, PanelData(pop_list), freq, win, type_to_idx or {}, pop_to_idx, pos_to_idx,
                   ref_gt=ref_gt, ref_pos=ref_pos, embedding_layer=embedding_layer, name=name)


def _weights_token(P) -> tuple:
    """Host-side identity of the weights the retrieval embeds with: the optimizer's update count
    (the fused Adam updates in place without bumping tensor versions) and the token table's
    storage and version (torch in-place updates, e.g. load_state_dict)."""
    from .. import autograd_ops
    base = P.W._base if P.W._base is not None else P.W
    return autograd_ops._EPOCH[0], base.data_ptr(), base._version


def h2d(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    """Host -> device copy that does not synchronise the host with the device queue: a pageable
    source is staged through the pinned caching allocator first (a pageable copy waits for the
    stream to drain — at the start of a training step that left the GPU idle while the host
    ran the retrieval's Python)."""
    if t.device == dev or dev.type != "cuda" or t.device.type != "cpu":
        return t.to(dev)
    if not t.is_pinned():
        t = t.pin_memory()
    return t.to(dev, non_blocking=True)


def panel_index_of(alleles: np.ndarray, ref_af: np.ndarray, device, shard=None):
    """PanelIndex of one window's panel, or of this rank's contiguous range of it."""
    from ..retrieval import PanelIndex
    if shard is None:
        return PanelIndex.from_alleles(alleles, ref_af, device)
    r0, r1 = shard.bounds(alleles.shape[0])
    return PanelIndex.from_alleles(alleles[r0:r1], ref_af, device, ref_offset=r0, n_total=alleles.shape[0])


def retrieve(ds, batch: dict, embedding_layer, device, k: int, masks: List[np.ndarray],
             dense: bool = False, limbs: int = 2) -> dict:
    """Shared retrieval body of the train/val and infer datasets (see module docstring).

    With ``ds.panel_shard`` set (multi-rank) each rank's index holds its own
    contiguous haplotype range and every window step runs the collective search of
    ``retrieval/shards.py`` over the union of the ranks' batch windows; the neighbour
    means then come from the all-reduced per-site alt-allele counts."""
    from ..engine import engine_for
    from .. import kernels as K
    eng = engine_for(embedding_layer)
    train = embedding_layer.training
    P = eng.packed(allow_train=True)
    dev = torch.device(device)
    h1 = h2d(batch["hap_1"], dev).long()
    h2 = h2d(batch["hap_2"], dev).long()
    af = h2d(batch["af"], dev).float()
    B, L = h1.shape
    D = P.W.shape[1]
    groups = defaultdict(list)
    for i, w in enumerate(batch["window_idx"]):
        groups[int(w)].append(i)
    shard = getattr(ds, "panel_shard", None)
    windows = list(groups)
    if shard is not None:
        from ..retrieval.shards import batch_windows
        windows = batch_windows(windows, shard.group)
    # eval: the neighbour means land directly in rows [2B:] of the encoder's input block
    block = None if train else eng.input_block(B, L, dev)
    rag_mean = None if train else block[2 * B:]
    rag_idx = torch.empty(2 * B, k, device=dev, dtype=torch.long)
    rag_groups = []
    dense_out = None
    stale = train and getattr(ds, "panel_cache", "fresh") == "window"
    for w in windows:
        rows = groups.get(w, [])
        # the reference's cache trigger (:334-336): another window cached, or reset at epoch start
        new_snap = stale and (ds.jit_cache_win_idx != w or ds._panel_snap is None or ds._panel_snap[0] != w)
        index = ds.panel_index(w, dev)
        rows_t = h2d(torch.tensor(rows, dtype=torch.long), dev)
        tok = torch.cat([h1[rows_t], h2[rows_t]], 0).contiguous()
        n = index.n_sites
        site_mask = h2d(torch.from_numpy(np.ascontiguousarray(masks[w][1:1 + n], np.uint8)), dev)
        ref_af = index.ref_af
        # A_q - A_r vanishes when the query AF rows equal the panel's window AF (always for
        # windows built from one freq table); otherwise pass both AF embeddings (exact LUT form).
        # (a device -> host answer: asked only where the search needs it — not under train-mode
        # dropout, whose exact-LUT offsets carry the AF embeddings anyway)
        afw = af[rows_t]
        same_memo = []

        def same_af() -> bool:
            if not same_memo:
                same_memo.append(bool(torch.equal(afw, ref_af.unsqueeze(0).expand_as(afw))))
            return same_memo[0]
        counts = uniq = None
        p_drop = embedding_layer.dropout.p if train else 0.0
        with torch.no_grad():
            Ar_emb = eng.af_embedding(ref_af.unsqueeze(0), True).float()[0].contiguous() \
                if P.af is not None else None
            Wp, stale_w = None, False
            if stale:
                wtok = _weights_token(P)
                if new_snap:   # eval-mode panel embedding of this window under the weights of now
                    ds._panel_snap = (w, P.W.detach().float().clone(), Ar_emb, wtok)
                _, W_s, Ar_s, wtok_s = ds._panel_snap
                # weights untouched since the snapshot (its first batch): the plain search is the
                # same.  Decided on the host from the weights' update count (optimizer steps, torch
                # in-place updates) — comparing the tensors was a device sync per training step
                stale_w = wtok != wtok_s
                if stale_w:
                    Wp, Ar_emb = W_s, Ar_s
            Aq_drop = None
            if p_drop > 0 and len(rows):
                # train mode: the reference embeds the queries WITH dropout before the distance
                # (:385-386).  u = W[tok] + Aq - Ar must equal drop(e_q) - pe - A_r, so Aq carries
                # drop(e_q) - W[tok] - pe per query row (exact-LUT form, fresh torch RNG mask)
                Afull = eng.af_embedding(torch.cat([afw, afw]), True).float() if P.af is not None else 0.0
                e_q = P.W[tok] + P.pe[:L] + Afull
                Aq_drop = (torch.nn.functional.dropout(e_q, p_drop, True) - P.W[tok] - P.pe[:L]).contiguous()
            if shard is not None:
                from ..retrieval.shards import any_rank, kernel_ops, sharded_neighbours
                drop_any = any_rank(p_drop > 0, dev, shard.group)
                # a snapshot A_r differs from the queries' current AF embedding even for equal AF
                exact = P.af is not None and not drop_any and (stale_w or any_rank(not same_af(), dev, shard.group))
                ops = kernel_ops(index, P.W, site_mask, k, limbs,
                                 aq_fn=lambda a: eng.af_embedding(a, True).float().contiguous(),
                                 Ar=Ar_emb if (exact or drop_any) else None, Wp=Wp)
                if drop_any and Aq_drop is None:
                    # a rank without queries of this window (or p = 0 while another rank drops):
                    # its rows still enter the exact-LUT launch, as undropped offsets
                    Afull = eng.af_embedding(torch.cat([afw, afw]), True).float() if P.af is not None else 0.0
                    Aq_drop = (Afull + torch.zeros(tok.shape[0], L, D, device=dev)).contiguous()
                idx, _, extra = sharded_neighbours(tok, k, ops, torch.cat([afw, afw]) if exact else None,
                                                   shard.group, aq_rows=Aq_drop if drop_any else None,
                                                   want_codes=train and (drop_any or dense))
                if train and (drop_any or dense):
                    uniq = extra
                else:
                    counts = extra
            else:
                Aq = Ar = None
                aq_period = len(rows)
                if Aq_drop is not None:
                    Aq, aq_period = Aq_drop, 2 * len(rows)
                    Ar = Ar_emb if Ar_emb is not None else torch.zeros(L, D, device=dev)
                elif P.af is not None and (stale_w or not same_af()):
                    Aq = eng.af_embedding(afw, True).float().contiguous()
                    Ar = Ar_emb
                idx, _ = index.search(tok, P.W, site_mask, k, limbs=limbs, Aq=Aq, aq_period=aq_period, Ar=Ar,
                                      Wp=Wp)
        nb = len(rows)
        if nb == 0:
            continue
        if train:
            rag_groups.append(NeighbourGroup(rows_t, idx[:nb], idx[nb:], index, counts,
                                             *(uniq if uniq is not None else (None, None))))
        else:
            if nb == B and rows == list(range(B)):      # one window, batch order: no scatter
                K.rag_mean(idx, index.codes, n, P.W, P.pe, Ar_emb, L, eng.dtype, out=rag_mean, counts=counts)
            else:
                means = K.rag_mean(idx, index.codes, n, P.W, P.pe, Ar_emb, L, eng.dtype, counts=counts)
                rag_mean[rows_t] = means[:nb]
                rag_mean[rows_t + B] = means[nb:]
        if dense and not train:
            # the reference's [B, k, L, D] fp32 neighbour embeddings (:425-442): every (query,
            # neighbour) pair as a one-neighbour "mean" in one launch
            if shard is not None:
                raise NotImplementedError("dense neighbour embeddings need the neighbours' panel rows; "
                                          "a sharded panel returns their counts only")
            if dense_out is None:
                dense_out = torch.zeros(2 * B, k, L, D, device=dev, dtype=torch.float32)
            e = K.rag_mean(idx.reshape(-1, 1), index.codes, n, P.W, P.pe, Ar_emb, L, torch.float32)
            e = e.view(2 * nb, k, L, D)
            dense_out[rows_t] = e[:nb]
            dense_out[rows_t + B] = e[nb:]
        rag_idx[rows_t] = idx[:nb]
        rag_idx[rows_t + B] = idx[nb:]
    batch["rag_idx_h1"], batch["rag_idx_h2"] = rag_idx[:B], rag_idx[B:]
    if train:
        # the reference's train-mode contract (:404-442): rag_emb_h1/h2 re-encoded WITH grad
        # (embedding dropout included) — the K-mean [B, 1, L, D] (bert.py:180-182 takes it as is)
        # or, dense, every neighbour [B, k, L, D]; f32, connected to the embedding parameters
        from ..train_forward import neighbour_embeddings
        e = neighbour_embeddings(embedding_layer, rag_groups, B, L, dense=dense)
        if dense:
            batch["rag_emb_h1"], batch["rag_emb_h2"] = e[:B], e[B:]
        else:
            batch["rag_emb_h1"], batch["rag_emb_h2"] = e[:B].unsqueeze(1), e[B:].unsqueeze(1)
        batch["rag_groups"] = rag_groups
        return batch
    if dense:
        batch["rag_emb_h1"], batch["rag_emb_h2"] = dense_out[:B], dense_out[B:]
    else:
        batch["rag_emb_h1"] = rag_mean[:B].unsqueeze(1)
        batch["rag_emb_h2"] = rag_mean[B:].unsqueeze(1)
    batch["rag_mean"] = rag_mean
    batch["rag_block"] = block
    return batch


def embedding_rag_collate_fn(batch_list, dataset=None, embedding_layer=None, k_retrieve=1):
    """CPU-only collate (embedding_rag_dataset.py:609-645)."""
    out = defaultdict(list)
    for s in batch_list:
        for key in s:
            out[key].append(s[key])
    for key in out:
        if key in ("window_idx", "hap1_nomask", "hap2_nomask"):
            continue
        try:
            out[key] = torch.stack(out[key])
        except (RuntimeError, TypeError):
            pass
    return dict(out)
