"""HBM-resident panel index of one window and its exact kNN search.

Reference behaviour replaced (src/dataset/embedding_rag_dataset.py):
  * JIT index build (:334-377): masked panel tokens -> fp32 embeddings [N, 1030, D]
    (15.8 GB at N = 10k, 1.58 TB at N = 1M).  Here: allele codes u8 [N, n_sites_pad]
    (1.03 GB at N = 1M), independent of the model weights and of the mask, so it
    never goes stale and is built once per window.
  * distance + top-k (:390-402): torch.cdist + topk(largest=False).  Here:
    LUT -> int8 MFMA scan -> exact (distance, index) top-k.
"""

from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from .. import kernels as K


def pad_sites(n_sites: int) -> int:
    """Index row length: a multiple of 256 B so the scan's 16-row LDS swizzle stays inside a row."""
    return max(256, ((n_sites + 255) // 256) * 256)


class PanelIndex:
    def __init__(self, codes: torch.Tensor, n_sites: int, ref_af: torch.Tensor, ref_offset: int = 0,
                 n_total: Optional[int] = None):
        if codes.dtype != torch.uint8 or codes.dim() != 2:
            raise ValueError("codes must be uint8 [n_ref, ld]")
        self.codes = codes
        self.n_ref, self.ld = codes.shape
        self.n_sites = int(n_sites)
        self.n_sites_pad = pad_sites(n_sites)
        if self.ld < self.n_sites_pad:
            raise ValueError("codes row shorter than padded window")
        self.ref_af = ref_af            # f32 [L] padded AF of the window (ref_af_windows[w])
        self.ref_offset = int(ref_offset)
        self.n_total = int(n_total if n_total is not None else self.n_ref + ref_offset)

    @classmethod
    def from_alleles(cls, alleles: np.ndarray, ref_af: np.ndarray, device, ref_offset: int = 0,
                     n_total: Optional[int] = None) -> "PanelIndex":
        """alleles: int [n_ref, n_sites] in {0, 1} (the panel's GT of this window)."""
        a = np.asarray(alleles)
        if a.size and (a.min() < 0 or a.max() > 1):
            raise ValueError("panel index supports biallelic 0/1 genotypes (got values outside {0,1}); "
                             "binarise multi-allelic/missing calls first")
        n_ref, n_sites = a.shape
        ld = pad_sites(n_sites)
        codes = np.zeros((n_ref, ld), np.uint8)
        codes[:, :n_sites] = a
        return cls(torch.from_numpy(codes).to(device), n_sites,
                   torch.as_tensor(np.asarray(ref_af, np.float32), device=device), ref_offset, n_total)

    @classmethod
    def synthetic(cls, n_ref: int, n_sites: int, site_af: torch.Tensor, ref_af: torch.Tensor,
                  seed: int) -> "PanelIndex":
        codes = K.panel_synth(n_ref, n_sites, site_af.float().contiguous(), seed)
        return cls(codes, n_sites, ref_af)

    @property
    def nbytes(self) -> int:
        return self.codes.numel()

    # ------------------------------------------------------------------ search --
    def lut(self, tok_q: torch.Tensor, W: torch.Tensor, site_mask: torch.Tensor, limbs: int = 2,
            Aq: Optional[torch.Tensor] = None, aq_period: int = 0, Ar: Optional[torch.Tensor] = None,
            Wp: Optional[torch.Tensor] = None):
        return K.knn_lut(tok_q.long().contiguous(), W, site_mask, self.n_sites, self.n_sites_pad, limbs,
                         Aq, aq_period, Ar, Wp=Wp)

    SAMPLE_MIN = 1 << 17       # panels at least this large get a threshold pre-pass

    def scan_keys(self, lut: torch.Tensor, nq: int, limbs: int, k: int, presample: Optional[bool] = None) -> torch.Tensor:
        """Exact local top-k keys [nq, k] (uint64 in int64 storage) with global indices.

        Large panels first scan a 1/64 prefix of the panel: its k-th best distance is an
        upper bound on the panel's, so the full scan can start from it (strictly above it
        nothing can enter the top-k) and keeps far fewer candidates; the result is the
        same exact top-k.  (1/64 measured best for the whole search on the bench panel:
        1M x 1024, 96 queries: 0.319 ms vs 0.3315 ms at 1/128 and 0.337 ms at 1/32 — the
        full scan's candidate compaction is its compute-side cost, profiles/r3_knn_probe.txt.)"""
        n_ref = self.codes.shape[0]
        if presample is None:
            presample = n_ref >= self.SAMPLE_MIN
        th = None
        if presample:
            div = int(os.environ.get("SNVRAG_SAMPLE_DIV", "64"))
            rpp = int(os.environ.get("SNVRAG_SAMPLE_RPP", "64"))
            m = max(16 * k, ((n_ref // div) + 15) // 16 * 16)
            sample = K.knn_scan(self.codes[:m], self.n_sites_pad, lut, nq, limbs, k, self.ref_offset,
                                n_parts=max(1, min(256, m // rpp)))
            th = K.knn_threshold(K.topk_merge(sample, k), k)
        parts = K.knn_scan(self.codes, self.n_sites_pad, lut, nq, limbs, k, self.ref_offset, th_init=th)
        return K.topk_merge(parts, k)

    def search(self, tok_q: torch.Tensor, W: torch.Tensor, site_mask: torch.Tensor, k: int, limbs: int = 2,
               Aq: Optional[torch.Tensor] = None, aq_period: int = 0, Ar: Optional[torch.Tensor] = None,
               return_keys: bool = False, Wp: Optional[torch.Tensor] = None):
        """idx int64 [nq, k] (-1 pads when the panel has < k haplotypes), dist f32 [nq, k] (squared L2).
        ``Wp`` / ``Ar``: the panel side's token table / AF embedding when they differ from the
        queries' (a cached, stale panel embedding: snvrag_knn_lut_panel)."""
        nq = tok_q.shape[0]
        lut, exps, consts = self.lut(tok_q, W, site_mask, limbs, Aq, aq_period, Ar, Wp=Wp)
        keys = self.scan_keys(lut, nq, limbs, k)
        idx, dist = K.knn_decode(keys, exps, consts)
        if return_keys:
            return idx, dist, keys, lut, exps
        return idx, dist
