"""BERTEmbedding — token + sinusoidal position + Fourier-AF embedding
(model/embedding/bert.py:13-77).  Same parameters; the forward is the native
``snvrag_embed_tokens`` gather fused with the AF-MLP output."""
import torch
import torch.nn as nn

from .af_embedding import AFEmbedding
from .position import PositionalEmbedding


class BERTEmbedding(nn.Module):
    def __init__(self, vocab_size: int, embed_size: int, dropout: float = 0.1, use_af: bool = True):
        super().__init__()
        self.tokenizer = nn.Embedding(vocab_size, embed_size, padding_idx=0)
        self.position = PositionalEmbedding(embed_size)
        self.use_af = use_af
        if use_af:
            self.af_embedding = AFEmbedding(embed_size=embed_size, num_basis=32)
        self.embed_size = embed_size
        self.dropout = nn.Dropout(dropout)

    def forward(self, seq, af=None, pos: bool = False):
        """[B, L] tokens (+ [B, L] AF) -> [B, L, D] on the GPU (eval semantics)."""
        from ...engine import engine_for
        return engine_for(self).embed(seq, af, pos)
