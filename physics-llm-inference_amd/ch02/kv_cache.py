"""KV cache and GQA-with-cache -- mirror of ``ch02/kv_cache.py``.

The cache keeps the reference's layout, [batch, max_seq_len, num_kv_heads,
head_dim] zero-initialised K and V buffers (``ch02/kv_cache.py:25-35``), and
``update`` keeps its append-and-return-the-valid-prefix contract (``:37-48``).

On a ROCm device the attention over the cache is ONE call into
``pli_attn_decode`` (split-K flash-decoding, csrc/decode_attn.hip), which
reads the cache buffer in place: no transpose, no ``repeat_interleave`` to
the query heads (``:81-86``), no [S_q, S_kv] score tensor or mask tensor
(``:88-95``).  Prompts with more query rows than the decode tile takes go to
the prefill flash kernel inside the same entry point.  Projections run on
``pli_gemm``.  CPU tensors keep the reference math.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

import pli_hip


def _proj(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    lead = x.shape[:-1]
    return pli_hip.gemm(x.reshape(-1, x.shape[-1]), w, trans_b=True).view(*lead, w.shape[0])


def attend_cached(q: torch.Tensor, k_buf: torch.Tensor, v_buf: torch.Tensor, n_kv: int
                  ) -> torch.Tensor:
    """softmax(q k^T / sqrt(hd) [+ bottom-right causal]) v over the first n_kv
    positions of [B, S, Hkv, hd] buffers; q [B, Sq, H, hd] -> [B, Sq, H, hd].
    The mask is the reference's ``triu(..., diagonal=n_kv - Sq + 1)``, applied
    only when Sq > 1 (``ch02/kv_cache.py:91-95``)."""
    sq = q.shape[1]
    if q.is_cuda:
        return pli_hip.attn_decode(q, k_buf, v_buf, n_kv, scale=1.0 / math.sqrt(q.shape[-1]),
                                   causal=sq > 1)
    groups = q.shape[2] // k_buf.shape[2]
    qt = q.transpose(1, 2)
    kt = k_buf[:, :n_kv].transpose(1, 2).repeat_interleave(groups, dim=1)
    vt = v_buf[:, :n_kv].transpose(1, 2).repeat_interleave(groups, dim=1)
    scores = torch.matmul(qt, kt.transpose(-2, -1)) / math.sqrt(q.shape[-1])
    if sq > 1:
        mask = torch.triu(torch.ones(sq, n_kv, device=q.device, dtype=torch.bool),
                          diagonal=n_kv - sq + 1)
        scores = scores.masked_fill(mask, float("-inf"))
    return torch.matmul(F.softmax(scores, dim=-1), vt).transpose(1, 2)


@dataclass
class KVCache:
    k_cache: torch.Tensor
    v_cache: torch.Tensor
    seq_len: int

    @classmethod
    def create(cls, batch_size: int, max_seq_len: int, num_kv_heads: int, head_dim: int,
               device: torch.device, dtype: torch.dtype) -> "KVCache":
        shape = (batch_size, max_seq_len, num_kv_heads, head_dim)
        return cls(k_cache=torch.zeros(shape, device=device, dtype=dtype),
                   v_cache=torch.zeros(shape, device=device, dtype=dtype), seq_len=0)

    def update(self, k: torch.Tensor, v: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Append [B, T, Hkv, hd] K/V at seq_len; return the valid prefixes."""
        start, end = self.seq_len, self.seq_len + k.shape[1]
        self.k_cache[:, start:end] = k
        self.v_cache[:, start:end] = v
        self.seq_len = end
        return self.k_cache[:, :end], self.v_cache[:, :end]

    def memory_bytes(self) -> int:
        return self.k_cache.numel() * self.k_cache.element_size() * 2


class GQAWithCache(nn.Module):
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

    def forward(self, x: torch.Tensor, kv_cache: KVCache | None = None, use_cache: bool = True
                ) -> tuple[torch.Tensor, KVCache | None]:
        B, S, _ = x.shape
        lin = _proj if x.is_cuda else (lambda t, w: F.linear(t, w))
        q = lin(x, self.q_proj.weight).view(B, S, self.num_heads, self.head_dim)
        k = lin(x, self.k_proj.weight).view(B, S, self.num_kv_heads, self.head_dim)
        v = lin(x, self.v_proj.weight).view(B, S, self.num_kv_heads, self.head_dim)
        # the reference appends only when use_cache and a cache object is given
        # (``ch02/kv_cache.py:79``); attention then spans the whole valid prefix
        if use_cache and kv_cache is not None:
            kv_cache.update(k, v)
            k_buf, v_buf, n_kv = kv_cache.k_cache, kv_cache.v_cache, kv_cache.seq_len
        else:
            k_buf, v_buf, n_kv = k, v, S
        o = attend_cached(q, k_buf, v_buf, n_kv)
        o = o.reshape(B, S, self.hidden_dim)
        return lin(o, self.o_proj.weight), kv_cache


def calculate_kv_cache_size(batch_size: int, max_seq_len: int, num_layers: int,
                            num_kv_heads: int, head_dim: int,
                            dtype: torch.dtype = torch.float16) -> dict:
    """Cache footprint (``ch02/kv_cache.py:104-122``): K and V, per token per layer."""
    elem = torch.tensor([], dtype=dtype).element_size()
    per_token_per_layer = 2 * num_kv_heads * head_dim * elem
    per_token = per_token_per_layer * num_layers
    total = per_token * max_seq_len * batch_size
    return {
        "per_token_per_layer_bytes": per_token_per_layer,
        "per_token_bytes": per_token,
        "total_bytes": total,
        "total_mb": total / 1024 / 1024,
        "total_gb": total / 1024 / 1024 / 1024,
    }
