"""Grouped-query attention -- mirror of ``ch01/gqa.py``.

Same constructor, parameter names and creation order as the reference
(``q_proj, k_proj, v_proj, o_proj``, ``ch01/gqa.py:9-20``), so seeded weights
and ``state_dict``s match.

On a ROCm device the reference's ``repeat_interleave`` of K and V to all
query heads (``:30-31``, G copies of K/V written and re-read through HBM) is
gone: the four projections run on ``pli_gemm`` and the flash kernel maps
query head h to kv head ``h // (H / Hkv)`` while it streams K/V, reading the
[B, S, Hkv, hd] projection outputs through strided views.  CPU tensors keep
the reference math.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

import pli_hip

from .attention import _linear


class GroupedQueryAttention(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int, num_kv_heads: int):
        super().__init__()
        assert num_heads % num_kv_heads == 0
        self.num_heads = num_heads
        self.num_kv_heads = num_kv_heads
        self.num_groups = num_heads // num_kv_heads
        self.head_dim = hidden_dim // num_heads
        self.hidden_dim = hidden_dim
        self.q_proj = nn.Linear(hidden_dim, num_heads * self.head_dim, bias=False)
        self.k_proj = nn.Linear(hidden_dim, num_kv_heads * self.head_dim, bias=False)
        self.v_proj = nn.Linear(hidden_dim, num_kv_heads * self.head_dim, bias=False)
        self.o_proj = nn.Linear(hidden_dim, hidden_dim, bias=False)

    def _forward_hip(self, x: torch.Tensor, causal: bool) -> torch.Tensor:
        B, S, _ = x.shape
        H, Hkv, hd = self.num_heads, self.num_kv_heads, self.head_dim
        q = _linear(x, self.q_proj.weight).view(B, S, H, hd).transpose(1, 2)
        k = _linear(x, self.k_proj.weight).view(B, S, Hkv, hd).transpose(1, 2)
        v = _linear(x, self.v_proj.weight).view(B, S, Hkv, hd).transpose(1, 2)
        o = torch.empty(B, S, H, hd, dtype=x.dtype, device=x.device)
        pli_hip.flash_attn_fwd(q, k, v, scale=1.0 / math.sqrt(hd), causal=causal,
                               out=o.transpose(1, 2))
        return _linear(o.view(B, S, H * hd), self.o_proj.weight)

    def forward(self, x: torch.Tensor, causal: bool = True) -> torch.Tensor:
        if x.is_cuda:
            return self._forward_hip(x, causal)
        B, S, _ = x.shape
        q = self.q_proj(x).view(B, S, self.num_heads, self.head_dim).transpose(1, 2)
        k = self.k_proj(x).view(B, S, self.num_kv_heads, self.head_dim).transpose(1, 2)
        v = self.v_proj(x).view(B, S, self.num_kv_heads, self.head_dim).transpose(1, 2)
        k = k.repeat_interleave(self.num_groups, dim=1)
        v = v.repeat_interleave(self.num_groups, dim=1)
        scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(self.head_dim)
        if causal:
            mask = torch.triu(torch.ones(S, S, device=x.device, dtype=torch.bool), diagonal=1)
            scores = scores.masked_fill(mask, float("-inf"))
        o = torch.matmul(F.softmax(scores, dim=-1), v)
        return self.o_proj(o.transpose(1, 2).contiguous().view(B, S, self.hidden_dim))

    def kv_cache_size_per_token(self, dtype: torch.dtype = torch.float16) -> int:
        """K and V bytes one token adds to the cache (``:41-43``)."""
        return 2 * self.num_kv_heads * self.head_dim * torch.tensor([], dtype=dtype).element_size()
