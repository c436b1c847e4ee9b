"""FeedForward — parameters of model/utils/feed_forward.py:4-21:
lrelu0.1(w_2(LN_4D(lrelu0.1(w_1 x)))) -> dropout."""
import torch.nn as nn


class FeedForward(nn.Module):
    def __init__(self, dims, hidden_dims, dropout=0.1):
        super().__init__()
        self.w_1 = nn.Linear(dims, hidden_dims)
        self.w_2 = nn.Linear(hidden_dims, dims)
        self.activation1 = nn.LeakyReLU(negative_slope=0.1)
        self.activation2 = nn.LeakyReLU(negative_slope=0.1)
        self.norm = nn.LayerNorm(hidden_dims)
        self.dropout = nn.Dropout(p=dropout)
