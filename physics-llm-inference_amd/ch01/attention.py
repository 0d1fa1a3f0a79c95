"""Attention modules -- mirror of ``ch01/attention.py``.

Parameter names, shapes and creation order are the reference's
(``q_proj, k_proj, v_proj, o_proj``, bias-free ``nn.Linear``,
``ch01/attention.py:52-55``), so ``torch.manual_seed(s)`` builds bit-identical
weights and ``state_dict``s are interchangeable.

On a ROCm device ``MultiHeadAttention.forward`` runs three HIP launch kinds
and no torch math: the four projections on ``pli_gemm`` (NT, C = X W^T), the
attention core on ``pli_flash_attn_fwd`` reading Q/K/V through their
[B,H,S,hd] strided views of the projection outputs (no transpose copies) and
writing O straight into the [B,S,H*hd] layout ``o_proj`` consumes.  The causal
mask is applied inside the kernel (no ``triu`` mask tensor rebuilt per call,
``:66-67``).  CPU tensors keep the reference math in torch.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

import pli_hip


def _attn_cpu(q, k, v, causal):
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(q.size(-1))
    if causal:
        n = q.size(-2)
        mask = torch.triu(torch.ones(n, n, dtype=torch.bool, device=q.device), diagonal=1)
        scores = scores.masked_fill(mask, float("-inf"))
    return torch.matmul(F.softmax(scores, dim=-1), v)


def naive_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Single-head [B, S, d] attention, scale 1/sqrt(d) (``:8-13``)."""
    if q.is_cuda:
        return pli_hip.flash_attn_fwd(q.unsqueeze(1), k.unsqueeze(1), v.unsqueeze(1),
                                      scale=1.0 / math.sqrt(q.size(-1)), causal=False).squeeze(1)
    return _attn_cpu(q, k, v, causal=False)


def causal_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Single-head causal attention (``:16-23``)."""
    if q.is_cuda:
        return pli_hip.flash_attn_fwd(q.unsqueeze(1), k.unsqueeze(1), v.unsqueeze(1),
                                      scale=1.0 / math.sqrt(q.size(-1)), causal=True).squeeze(1)
    return _attn_cpu(q, k, v, causal=True)


def _linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x W^T on the HIP GEMM (x [..., in] -> [..., out])."""
    lead = x.shape[:-1]
    y = pli_hip.gemm(x.reshape(-1, x.shape[-1]), w, trans_b=True)
    return y.view(*lead, w.shape[0])


class SingleHeadAttention(nn.Module):
    def __init__(self, hidden_dim: int, head_dim: int):
        super().__init__()
        self.head_dim = head_dim
        self.q_proj = nn.Linear(hidden_dim, head_dim, bias=False)
        self.k_proj = nn.Linear(hidden_dim, head_dim, bias=False)
        self.v_proj = nn.Linear(hidden_dim, head_dim, bias=False)
        self.o_proj = nn.Linear(head_dim, hidden_dim, bias=False)

    def forward(self, x: torch.Tensor, causal: bool = True) -> torch.Tensor:
        if x.is_cuda:
            q, k, v = (_linear(x, p.weight) for p in (self.q_proj, self.k_proj, self.v_proj))
            o = (causal_attention if causal else naive_attention)(q, k, v)
            return _linear(o, self.o_proj.weight)
        q, k, v = self.q_proj(x), self.k_proj(x), self.v_proj(x)
        return self.o_proj(_attn_cpu(q, k, v, causal))


class MultiHeadAttention(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int):
        super().__init__()
        assert hidden_dim % num_heads == 0
        self.num_heads = num_heads
        self.head_dim = hidden_dim // num_heads
        self.hidden_dim = hidden_dim
        self.q_proj = nn.Linear(hidden_dim, hidden_dim, bias=False)
        self.k_proj = nn.Linear(hidden_dim, hidden_dim, bias=False)
        self.v_proj = nn.Linear(hidden_dim, hidden_dim, bias=False)
        self.o_proj = nn.Linear(hidden_dim, hidden_dim, bias=False)

    def _forward_hip(self, x: torch.Tensor, causal: bool) -> torch.Tensor:
        B, S, _ = x.shape
        H, hd = self.num_heads, self.head_dim

        def heads(t):  # [B,S,H*hd] -> strided [B,H,S,hd] view, no copy
            return t.view(B, S, H, hd).transpose(1, 2)

        q, k, v = (heads(_linear(x, p.weight)) for p in (self.q_proj, self.k_proj, self.v_proj))
        o = torch.empty(B, S, H, hd, dtype=x.dtype, device=x.device)
        pli_hip.flash_attn_fwd(q, k, v, scale=1.0 / math.sqrt(hd), causal=causal,
                               out=o.transpose(1, 2))
        return _linear(o.view(B, S, self.hidden_dim), self.o_proj.weight)

    def forward(self, x: torch.Tensor, causal: bool = True) -> torch.Tensor:
        if x.is_cuda:
            return self._forward_hip(x, causal)
        batch, seq_len, _ = x.shape
        q = self.q_proj(x).view(batch, seq_len, self.num_heads, self.head_dim).transpose(1, 2)
        k = self.k_proj(x).view(batch, seq_len, self.num_heads, self.head_dim).transpose(1, 2)
        v = self.v_proj(x).view(batch, seq_len, self.num_heads, self.head_dim).transpose(1, 2)
        o = _attn_cpu(q, k, v, causal)
        o = o.transpose(1, 2).contiguous().view(batch, seq_len, self.hidden_dim)
        return self.o_proj(o)
