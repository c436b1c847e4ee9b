from .position import PositionalEmbedding
from .af_embedding import AFEmbedding
from .bert import BERTEmbedding
