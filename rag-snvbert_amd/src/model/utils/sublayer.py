"""SublayerConnection — post-LN residual of model/utils/sublayer.py:4-16."""
import torch.nn as nn


class SublayerConnection(nn.Module):
    def __init__(self, size, dropout):
        super().__init__()
        self.norm = nn.LayerNorm(size)
        self.dropout = nn.Dropout(p=dropout)
