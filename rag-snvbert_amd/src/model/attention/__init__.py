from .multi_head_attention import Attention, MultiHeadAttention
