"""MultiHeadAttention — parameters of model/attention/multi_head_attention.py:6-53
(three input projections + output projection); executed by the native encoder."""
import torch.nn as nn


class Attention(nn.Module):
    """Parameter-free scaled-dot-product attention (model/attention/attention.py)."""


class MultiHeadAttention(nn.Module):
    def __init__(self, heads: int, dims: int, dropout: float = 0.1):
        super().__init__()
        assert dims % heads == 0, "Hidden dimension must be divisible by Heads"
        self.heads, self.dims = heads, dims // heads
        self.linear_layers = nn.ModuleList([nn.Linear(dims, dims) for _ in range(3)])
        self.output_layer = nn.Linear(dims, dims)
        self.attention = Attention()
        self.dropout = nn.Dropout(p=dropout)
