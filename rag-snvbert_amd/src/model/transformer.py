"""TransformerBlock — parameters of model/transformer.py:8-30.  The block stack
runs as one native call (``snvrag_encoder_forward``) from the engine."""
import torch.nn as nn

from .attention import MultiHeadAttention
from .utils import FeedForward, SublayerConnection


class TransformerBlock(nn.Module):
    def __init__(self, dims, attn_heads, feed_forward_hidden, dropout):
        super().__init__()
        self.attention = MultiHeadAttention(heads=attn_heads, dims=dims)
        self.feed_forward = FeedForward(dims=dims, hidden_dims=feed_forward_hidden, dropout=dropout)
        self.input_sublayer = SublayerConnection(size=dims, dropout=dropout)
        self.output_sublayer = SublayerConnection(size=dims, dropout=dropout)
        self.dropout = nn.Dropout(p=dropout)
