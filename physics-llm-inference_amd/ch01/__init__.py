"""Chapter 01 attention on MI355X (the hot-path subset: attention modules)."""

from .ffn import FusedSwiGLUFFN, NaiveFFN, SwiGLUFFN
from .gqa import GroupedQueryAttention
from .attention import (
    MultiHeadAttention,
    SingleHeadAttention,
    causal_attention,
    naive_attention,
)

__all__ = ["FusedSwiGLUFFN", "NaiveFFN", "SwiGLUFFN", "GroupedQueryAttention", "MultiHeadAttention", "SingleHeadAttention", "causal_attention", "naive_attention"]
