"""BERTWithEmbeddingRAG — the v18 SNVBERT encoder with retrieved-neighbour fusion
(model/bert.py:12-76, :132-219).  Parameter layout (and so state_dict keys) is
the reference's; ``forward`` runs the whole pre-encoder + 12-block stack on the
native MI355X engine and returns ``(h1, h2, h1_origin, h2_origin)`` like
bert.py:219.
"""
import torch.nn as nn

from .embedding import BERTEmbedding
from .fusion import EmbeddingFusionModule, EnhancedRareVariantFusion
from .transformer import TransformerBlock


class BERT(nn.Module):
    def __init__(self, vocab_size: int, dims: int = 512, n_layers: int = 12, attn_heads: int = 16,
                 dropout: float = 0.1):
        super().__init__()
        self.dims, self.n_layers, self.attn_heads = dims, n_layers, attn_heads
        self.feed_forward_hidden = dims * 4
        self.vocab_size = vocab_size
        self.embedding = BERTEmbedding(vocab_size=vocab_size, embed_size=dims, dropout=dropout)
        self.emb_fusion = EmbeddingFusionModule(emb_size=dims)
        self.transformer_blocks = nn.ModuleList(
            [TransformerBlock(dims, attn_heads, self.feed_forward_hidden, dropout) for _ in range(n_layers)])


class BERTWithEmbeddingRAG(BERT):
    def __init__(self, vocab_size, dims=512, n_layers=12, attn_heads=16, dropout=0.1):
        super().__init__(vocab_size, dims, n_layers, attn_heads, dropout)
        self.rag_fusion = EnhancedRareVariantFusion(dims)

    def forward(self, x: dict):
        from ..engine import engine_for
        out = engine_for(self).forward_bert(x)
        return out["h1_after"], out["h2_after"], out["h1_before"], out["h2_before"]
