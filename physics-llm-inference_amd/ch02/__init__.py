"""Chapter 02 on MI355X: KV cache, cached GQA, cached generation.

Decode attention over the cache runs on ``pli_attn_decode`` (split-K
flash-decoding).  ``naive_generate`` (``ch02/generation.py``) re-runs the
whole ``ch01.transformer`` model per token; that model is outside the hot
path and is not mirrored.
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
    "cached_generate",
]
