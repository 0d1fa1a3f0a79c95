"""Chapter 02 on MI355X: KV cache, cached GQA, cached generation.

Decode attention over the cache runs on ``pli_attn_decode`` (split-K
flash-decoding).  ``naive_generate`` (``ch02/generation.py``) re-runs the
whole ``ch01.TransformerModel`` per token (every layer on the HIP kernels).
"""

from .cached_generation import (
    CachedGQA,
    CachedTransformerBlock,
    CachedTransformerModel,
    LayerKVCache,
    RMSNorm,
    SwiGLUFFN,
    cached_generate,
)
from .generation import naive_generate
from .kv_cache import GQAWithCache, KVCache, attend_cached, calculate_kv_cache_size

__all__ = [
    "KVCache",
    "GQAWithCache",
    "calculate_kv_cache_size",
    "attend_cached",
    "LayerKVCache",
    "CachedGQA",
    "CachedTransformerBlock",
    "CachedTransformerModel",
    "RMSNorm",
    "SwiGLUFFN",
    "naive_generate",
    "cached_generate",
]
