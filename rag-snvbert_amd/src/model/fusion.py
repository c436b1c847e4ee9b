"""Retrieved-neighbour fusion modules of the v18 model (model/fusion.py) —
parameter containers with the reference's exact structure and init:

  PositionFeatModule        fusion.py:285-332   (3x Conv1d k=9 + LeakyReLU + BatchNorm)
  EmbeddingFusionModule     fusion.py:336-369   (LN(emb + lrelu(Linear(cat(emb, pos, af)))))
  CrossAFInteraction        fusion.py:58-86
  EnhancedRareVariantFusion fusion.py:89-162

The forward math is executed by the native engine (src/engine.py), fused into
the encoder input.
"""
import torch
import torch.nn as nn


class PositionFeatModule(nn.Module):
    def __init__(self, hidden_channels: int = 4, kernel_size: int = 9, stride: int = 1, padding: int = 4):
        super().__init__()
        self.conv1 = nn.Conv1d(1, hidden_channels, kernel_size, stride, padding)
        self.act1 = nn.LeakyReLU(negative_slope=0.05)
        self.conv2 = nn.Conv1d(hidden_channels, hidden_channels, kernel_size, stride, padding)
        self.act2 = nn.LeakyReLU(negative_slope=0.05)
        self.conv3 = nn.Conv1d(hidden_channels, 1, kernel_size, stride, padding)
        self.act3 = nn.LeakyReLU(negative_slope=0.05)
        self.norm1 = nn.BatchNorm1d(num_features=hidden_channels)
        self.norm2 = nn.BatchNorm1d(num_features=hidden_channels)


class EmbeddingFusionModule(nn.Module):
    def __init__(self, emb_size):
        super().__init__()
        self.pos_feat = PositionFeatModule()
        self.fusion = nn.Linear(emb_size + 2, emb_size)
        self.act = nn.LeakyReLU(negative_slope=0.1)
        self.norm = nn.LayerNorm(emb_size)


class CrossAFInteraction(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.gate_net = nn.Sequential(nn.Linear(2, 32), nn.GELU(), nn.Linear(32, dims), nn.Sigmoid())
        self.joint_encoder = nn.Sequential(nn.Linear(2, dims), nn.LayerNorm(dims), nn.GELU())
        self.res_scale = nn.Parameter(torch.tensor(0.1))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_normal_(m.weight)
                nn.init.constant_(m.bias, 0.01)


class EnhancedRareVariantFusion(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.af_interaction = CrossAFInteraction(dims)
        self.af_adapter = nn.Sequential(nn.Linear(dims, 4 * dims), nn.GELU(), nn.Dropout(0.1),
                                        nn.Linear(4 * dims, dims), nn.Sigmoid())
        self.pooling = nn.Sequential(nn.Linear(dims, 1), nn.Softmax(dim=2))
        self.fusion = nn.Sequential(nn.Linear(2 * dims, 4 * dims), nn.GELU(), nn.Dropout(0.1),
                                    nn.Linear(4 * dims, dims), nn.LayerNorm(dims))
        self.res_scale = nn.Parameter(torch.tensor(0.1))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_normal_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0.1)
