"""AFEmbedding — parameters of model/embedding/af_embedding.py:26-70 (Fourier AF
features -> Linear -> LayerNorm -> GELU -> Linear).  Its forward runs on the
native kernels through BERTEmbedding / the engine."""
import math

import torch
import torch.nn as nn


class AFEmbedding(nn.Module):
    def __init__(self, embed_size: int = 192, num_basis: int = 32, learnable_basis: bool = True):
        super().__init__()
        self.embed_size, self.num_basis = embed_size, num_basis
        init = torch.logspace(0, math.log10(100), num_basis)
        if learnable_basis:
            self.basis_freqs = nn.Parameter(init)
        else:
            self.register_buffer("basis_freqs", 2.0 ** torch.arange(num_basis, dtype=torch.float32))
        self.projection = nn.Sequential(nn.Linear(num_basis * 2, embed_size), nn.LayerNorm(embed_size),
                                        nn.GELU(), nn.Linear(embed_size, embed_size))
        for m in self.projection:
            if isinstance(m, nn.Linear):
                nn.init.xavier_normal_(m.weight)
                nn.init.constant_(m.bias, 0.0)

    def forward(self, af: torch.Tensor) -> torch.Tensor:
        from ...engine import engine_for
        return engine_for(self).af_embedding(af)
