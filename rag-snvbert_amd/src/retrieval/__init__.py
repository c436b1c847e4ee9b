"""Reference-panel retrieval on the HBM-resident token index (replaces the
reference's per-window fp32 embedding cache + cdist/topk and FAISS IndexFlatL2)."""
from .embedding_index import EmbeddingIndex, panel_tokens
from .panel_index import PanelIndex, pad_sites
from .shards import merge_keys_gathered, sharded_search
