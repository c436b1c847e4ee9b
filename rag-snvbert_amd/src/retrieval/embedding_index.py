"""Embedding-space panel index — the reference's literal retrieval, kept as a cross-check of
the token-resident index (SURVEY.md §8d "C2 embedding-space mode").

Reference behaviour restated (src/dataset/embedding_rag_dataset.py):
  * JIT index build (:334-377, mask applied by _apply_mask_to_tokens_gpu :446-461): the panel's
    masked window tokens -> BERTEmbedding in eval -> cache [N, L, D];
  * search (:390-402; FAISS IndexFlatL2 in embedding_rag_infer_dataset.py:176-177, 279-285):
    exact L2 over the flattened [L * D] rows, topk(k, largest=False).
Here the cache is bf16 [N, L * D] in HBM — stored in the scan's tiled layout (4 KiB tiles of
32 rows x 64 dims, K.knn_emb_pack: every wave load one contiguous KiB) — with its squared norms
stored at build time, and the search is the HBM-bound distance GEMM of csrc/knn_emb.hip (every
panel byte read once per query batch) followed by top-k over the distance rows.  The production path (PanelIndex)
computes the same distances from the allele codes without ever materialising E.
"""

from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .. import kernels as K
from ..dataset.vocab import EOS, MASK, PAD, SOS


def panel_tokens(codes: torch.Tensor, n_sites: int, mask: Optional[np.ndarray], L: int,
                 tok0: int = 5, tok1: int = 6) -> torch.Tensor:
    """Window tokens [N, L] of panel rows (alleles in codes[:, :n_sites]) exactly as
    WordVocab.tokenize builds a query's: <sos> alleles <eos> <pad>..., then the window mask
    (token positions, sequence_padding'd) replaced by <mask> (_apply_mask_to_tokens_gpu)."""
    n = codes.shape[0]
    tok = torch.full((n, L), PAD, dtype=torch.int64, device=codes.device)
    tok[:, 0] = SOS
    a = codes[:, :n_sites].long()
    tok[:, 1:1 + n_sites] = torch.where(a == 0, torch.full_like(a, tok0), torch.full_like(a, tok1))
    tok[:, 1 + n_sites] = EOS
    if mask is not None:
        m = torch.as_tensor(np.asarray(mask)[:L].astype(bool), device=codes.device)
        tok[:, m] = MASK
    return tok


class EmbeddingIndex:
    """bf16 [N, L * D] window embeddings of the panel (packed: ``Et``, K.knn_emb_pack's layout)
    + f32 squared norms."""

    def __init__(self, Et: torch.Tensor, norms: torch.Tensor, L: int, D: int):
        n = norms.shape[0]
        if Et.dtype != torch.bfloat16 or Et.dim() != 2 or Et.shape[1] != L * D or Et.shape[0] != (n + 31) // 32 * 32:
            raise ValueError("Et must be the packed bf16 [ceil(N / 32) * 32, L * D] index of len(norms) rows")
        self.Et, self.norms, self.L, self.D = Et, norms, L, D
        self.n = n

    @classmethod
    def from_rows(cls, E: torch.Tensor, L: int, D: int) -> "EmbeddingIndex":
        """From row-major bf16 E [N, L * D] (packed into a new buffer)."""
        if E.dtype != torch.bfloat16 or E.dim() != 2 or E.shape[1] != L * D:
            raise ValueError("E must be bf16 [N, L * D]")
        return cls(K.knn_emb_pack(E), K.knn_emb_norms(E), L, D)

    @classmethod
    def build(cls, tok: torch.Tensor, W: torch.Tensor, pe: torch.Tensor, Ar: Optional[torch.Tensor] = None,
              chunk: int = 2048) -> "EmbeddingIndex":
        """E[r] = W[tok[r]] + pe + Ar (BERTEmbedding eval; Ar = the window's AF embedding rows,
        shared by every haplotype of the window), embedded chunk by chunk (chunk a multiple of
        32) into a row-major transient and packed into the tiled index."""
        assert chunk % 32 == 0
        n, L = tok.shape
        D = W.shape[1]
        Et = torch.empty((n + 31) // 32 * 32, L * D, device=tok.device, dtype=torch.bfloat16)
        norms = torch.empty(n, device=tok.device, dtype=torch.float32)
        E = torch.empty(min(n, chunk), L * D, device=tok.device, dtype=torch.bfloat16)
        for i in range(0, n, chunk):
            j = min(n, i + chunk)
            K.embed_tokens(tok[i:j].contiguous(), W, pe, Ar, 1 if Ar is not None else 0, torch.bfloat16,
                           out=E[:j - i].view(j - i, L, D))
            norms[i:j] = K.knn_emb_norms(E[:j - i])
            K.knn_emb_pack(E[:j - i], out=Et[i:])
        return cls(Et, norms, L, D)

    def rows(self, i: int, j: int) -> torch.Tensor:
        """Row-major bf16 [j - i, L * D] copy of rows i..j-1 (i a multiple of 32)."""
        assert i % 32 == 0 and 0 <= i < j <= self.n
        t = self.Et[i:(j + 31) // 32 * 32].view(-1, self.L * self.D // 64, 4, 2, 32, 8)
        return t.permute(0, 4, 1, 2, 3, 5).reshape(-1, self.L * self.D)[:j - i]

    def embed_queries(self, tok_q: torch.Tensor, W: torch.Tensor, pe: torch.Tensor,
                      Aq: Optional[torch.Tensor] = None) -> torch.Tensor:
        nq, L = tok_q.shape
        return K.embed_tokens(tok_q.long().contiguous(), W, pe, Aq, 1 if Aq is not None else 0,
                              torch.bfloat16).view(nq, L * self.D)

    def search(self, Q: torch.Tensor, k: int):
        """(dist f32 [Bq, k] ascending, idx int64 [Bq, k]) for bf16 query rows Q [Bq, L * D];
        batches of up to 128 queries per pass over the panel."""
        ds, ix = [], []
        for i in range(0, Q.shape[0], 128):
            d, j = K.knn_emb_search(self.Et, Q[i:i + 128].contiguous(), k, self.norms)
            ds.append(d)
            ix.append(j)
        return torch.cat(ds), torch.cat(ix)
