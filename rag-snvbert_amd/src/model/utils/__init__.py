from .feed_forward import FeedForward
from .sublayer import SublayerConnection
