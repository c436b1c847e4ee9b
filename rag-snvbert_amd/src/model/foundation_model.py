"""BERTFoundationModel + heads (model/foundation_model.py:13-177).

``forward(x)`` returns the reference's list
``[hap_1_probs, hap_2_probs, gt_probs, h1_before, h2_before, h1_after, h2_after]``
(foundation_model.py:25-33), computed by the native engine.  Heads return
softmax probabilities, exactly as the reference does (:79-80, :174-176).
"""
import torch.nn as nn

from .bert import BERTWithEmbeddingRAG
from .utils import FeedForward


class EnhancedHaplotypeClassifier(nn.Module):
    def __init__(self, dims, vocab_size=2):
        super().__init__()
        self.af_fusion = nn.Sequential(nn.Linear(dims + 2, 4 * dims), nn.GELU(), nn.Linear(4 * dims, dims),
                                       nn.LayerNorm(dims))
        self.net = nn.Sequential(nn.Linear(dims, 4 * dims), nn.GELU(), nn.Linear(4 * dims, vocab_size))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0.1)


class GenotypeClassifier(nn.Module):
    def __init__(self, augment_factor: int = 2, vocab_size: int = 3):
        super().__init__()
        self.hidden_dims = 4 ** augment_factor
        self.gf_fusion = nn.Linear(7, self.hidden_dims)
        self.gf_act = nn.LeakyReLU(negative_slope=0.01)
        self.gf_norm = nn.LayerNorm(self.hidden_dims)
        self.layer = FeedForward(self.hidden_dims, self.hidden_dims, dropout=0.1)
        self.classifier = nn.Linear(self.hidden_dims, vocab_size)
        self.softmax = nn.Softmax(dim=-1)


class BERTFoundationModel(nn.Module):
    def __init__(self, bert: BERTWithEmbeddingRAG):
        super().__init__()
        self.bert = bert
        self.hap_classifier = EnhancedHaplotypeClassifier(bert.dims)
        self.gt_classifier = GenotypeClassifier(2, 4)

    def forward(self, x):
        if self.training:
            # autograd graph over the HIP training kernels (src/train_forward.py)
            from ..train_forward import forward_train
            return forward_train(self, x)
        from ..engine import engine_for
        o = engine_for(self).forward(x)
        return [o["probs_h1"], o["probs_h2"], o["gt"], o["h1_before"], o["h2_before"],
                o["h1_after"], o["h2_after"]]


def build_model(vocab_size: int, dims: int = 384, n_layers: int = 12, attn_heads: int = 12,
                dropout: float = 0.1) -> BERTFoundationModel:
    return BERTFoundationModel(BERTWithEmbeddingRAG(vocab_size, dims, n_layers, attn_heads, dropout))


def model_state_shapes(vocab_size: int, dims: int, n_layers: int, attn_heads: int):
    """state_dict key -> shape of the reference model (used by the synthetic-weight generator)."""
    import torch
    with torch.device("meta"):
        m = build_model(vocab_size, dims, n_layers, attn_heads)
    return {k: tuple(v.shape) for k, v in m.state_dict().items()}
