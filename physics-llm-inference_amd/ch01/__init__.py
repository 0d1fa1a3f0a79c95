"""Chapter 01 (transformer mechanics) on MI355X: attention, GQA, FFN and the
transformer block / model on the HIP kernels."""

from .ffn import FusedSwiGLUFFN, NaiveFFN, SwiGLUFFN
from .gqa import GroupedQueryAttention
from .transformer import RMSNorm, TransformerBlock, TransformerModel
from .attention import (
    MultiHeadAttention,
    SingleHeadAttention,
    causal_attention,
    naive_attention,
)

__all__ = ["RMSNorm", "TransformerBlock", "TransformerModel", "FusedSwiGLUFFN", "NaiveFFN", "SwiGLUFFN", "GroupedQueryAttention", "MultiHeadAttention", "SingleHeadAttention", "causal_attention", "naive_attention"]
