"""PositionalEmbedding — parameter container of model/embedding/position.py:12-38."""
import math

import torch
import torch.nn as nn

MAX_SEQ_LEN = 1030


class PositionalEmbedding(nn.Module):
    def __init__(self, dims: int, max_len: int = MAX_SEQ_LEN):
        super().__init__()
        pe = torch.zeros([max_len, dims]).float()
        position = torch.arange(0, max_len).float().unsqueeze(1)
        div_term = (torch.arange(0, dims, 2).float() * -(math.log(10000.0) / dims)).exp()
        pe[:, 0::2] = torch.sin(position * div_term)
        pe[:, 1::2] = torch.cos(position * div_term)
        self.register_buffer("pe", pe.unsqueeze(0))

    def forward(self, x):
        return self.pe[:, :x.size(1)]
