"""SNVBERT operator surface (reference: src/model) backed by libsnvrag kernels."""
from .bert import BERT, BERTWithEmbeddingRAG
from .foundation_model import BERTFoundationModel, build_model
