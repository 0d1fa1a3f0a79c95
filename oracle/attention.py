"""Attention oracles (test infrastructure only -- see oracle/__init__.py).

float64 numpy restatements of the reference attention math, plus a faithful
torch restatement of the reference FlashAttention tile loop that serves as the
CPU baseline in bench.py ("kind": "port").
"""
from __future__ import annotations

import math

import numpy as np


def _softmax_lastdim(s: np.ndarray) -> np.ndarray:
    m = np.max(s, axis=-1, keepdims=True)
    m = np.where(np.isfinite(m), m, 0.0)
    e = np.exp(s - m)
    return e / np.sum(e, axis=-1, keepdims=True)


def naive_attention(q, k, v, scale: float | None = None, causal: bool = False):
    """softmax(Q K^T * scale) V in float64 over [B, H, N, D] arrays.

    Follows ``ch06/attention_memory.py:19-33`` (``scale = D ** -0.5`` default,
    materialised [B,H,N,N] scores, softmax over keys).  ``causal`` adds the
    ``torch.triu(ones, diagonal=1)`` mask of ``ch01/attention.py:66-67``,
    aligned bottom-right when Nq != Nk as in the cached prefill of
    ``ch02/cached_generation.py:85-91`` (query i sees key j iff
    j <= i + Nk - Nq).  GQA: when K/V carry fewer heads than Q, query head h
    reads KV head h // (H // Hkv) -- the grouping ``repeat_interleave`` gives in
    ``ch01/gqa.py:30-34``.
    """
    q = np.asarray(q, dtype=np.float64)
    k = np.asarray(k, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    B, H, Nq, D = q.shape
    Hkv, Nk = k.shape[1], k.shape[2]
    if scale is None:
        scale = D ** -0.5
    if Hkv != H:
        assert H % Hkv == 0
        k = np.repeat(k, H // Hkv, axis=1)
        v = np.repeat(v, H // Hkv, axis=1)
    s = np.matmul(q, np.swapaxes(k, -1, -2)) * scale
    if causal:
        i = np.arange(Nq)[:, None]
        j = np.arange(Nk)[None, :]
        s = np.where(j > i + (Nk - Nq), -np.inf, s)
    p = _softmax_lastdim(s)
    return np.matmul(p, v)


def naive_attention_3d(q, k, v, causal: bool = False):
    """Single-head [B, S, d] attention of ``ch01/attention.py:8-23`` in float64."""
    q = np.asarray(q, dtype=np.float64)[:, None]
    k = np.asarray(k, dtype=np.float64)[:, None]
    v = np.asarray(v, dtype=np.float64)[:, None]
    return naive_attention(q, k, v, scale=1.0 / math.sqrt(q.shape[-1]), causal=causal)[:, 0]


def multi_head_attention(x, wq, wk, wv, wo, num_heads: int, causal: bool = True):
    """``MultiHeadAttention.forward`` (``ch01/attention.py:57-72``) in float64.

    x [B,S,hidden]; w* are nn.Linear weights [out,in] (y = x W^T, bias-free).
    """
    x = np.asarray(x, dtype=np.float64)
    B, S, hidden = x.shape
    hd = hidden // num_heads

    def proj(w):
        return x @ np.asarray(w, dtype=np.float64).T

    def heads(t):
        return t.reshape(B, S, num_heads, hd).transpose(0, 2, 1, 3)

    q, k, v = heads(proj(wq)), heads(proj(wk)), heads(proj(wv))
    o = naive_attention(q, k, v, scale=1.0 / math.sqrt(hd), causal=causal)
    o = o.transpose(0, 2, 1, 3).reshape(B, S, hidden)
    return o @ np.asarray(wo, dtype=np.float64).T


# --- online softmax recurrences (ch06/online_softmax.py) -------------------

def standard_softmax(x):
    """``ch06/online_softmax.py:5-10`` in float64."""
    return _softmax_lastdim(np.asarray(x, dtype=np.float64))


def online_softmax(x):
    """Element-by-element (m, d) recurrence of ``ch06/online_softmax.py:13-25``."""
    x = np.asarray(x, dtype=np.float64)
    m = x[..., 0].copy()
    d = np.ones_like(m)
    for i in range(1, x.shape[-1]):
        m_new = np.maximum(m, x[..., i])
        d = d * np.exp(m - m_new) + np.exp(x[..., i] - m_new)
        m = m_new
    return np.exp(x - m[..., None]) / d[..., None]


def online_softmax_with_output(x, v):
    """(o, d) of ``ch06/online_softmax.py:28-53`` in float64.

    o is the softmax-weighted sum of v rows; d is the running denominator
    relative to the final running max.
    """
    x = np.asarray(x, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    m = x[..., 0].copy()
    d = np.ones_like(m)
    o = v[..., 0, :].copy()
    for i in range(1, x.shape[-1]):
        m_new = np.maximum(m, x[..., i])
        a = np.exp(m - m_new)
        b = np.exp(x[..., i] - m_new)
        d_new = d * a + b
        o = (o * (d * a)[..., None] + v[..., i, :] * b[..., None]) / d_new[..., None]
        m, d = m_new, d_new
    return o, d


# --- the reference tile loop, restated in torch (CPU baseline) -------------

def flash_tile_loop_torch(q, k, v, scale=None, block_q: int = 64, block_k: int = 64):
    """Restatement of ``ch06/flash_attention.py:14-74`` on torch tensors.

    Same blocking, same "normalised-O" update
    ``O = (O * l * e^{m-m'} + P V) / l'`` (``:64-65``), and the same dtype
    behaviour: every intermediate, including the running max/sum, stays in
    ``q.dtype`` (``:32-33, :44-47``).  Used (a) as the CPU-baseline workload in
    bench.py and (b) to check that the golden fixtures' reference outputs are
    reproduced bit-for-bit by a restatement.
    """
    import torch

    B, H, N, D = q.shape
    if scale is None:
        scale = D ** -0.5
    out = torch.zeros_like(q)
    for qs in range(0, N, block_q):
        qe = min(qs + block_q, N)
        qb = q[:, :, qs:qe, :]
        o = torch.zeros_like(qb)
        m = torch.full((B, H, qe - qs), float("-inf"), dtype=q.dtype, device=q.device)
        l = torch.zeros((B, H, qe - qs), dtype=q.dtype, device=q.device)
        for ks in range(0, N, block_k):
            ke = min(ks + block_k, N)
            s = torch.matmul(qb, k[:, :, ks:ke, :].transpose(-2, -1)) * scale
            m_new = torch.maximum(m, s.max(dim=-1).values)
            a = torch.exp(m - m_new)
            p = torch.exp(s - m_new.unsqueeze(-1))
            l_new = l * a + p.sum(dim=-1)
            o = (o * l.unsqueeze(-1) * a.unsqueeze(-1)
                 + torch.matmul(p, v[:, :, ks:ke, :])) / l_new.unsqueeze(-1)
            m, l = m_new, l_new
        out[:, :, qs:qe, :] = o
    return out


def attention_flops(B: int, H: int, N: int, D: int, causal: bool = False) -> int:
    """MFMA FLOPs of one forward: 4*B*H*N^2*D (QK^T and PV), halved-ish if causal.

    The reference's ``attention_flops`` (``ch06/attention_memory.py:36-49``) adds
    5*B*H*N^2 softmax FLOPs; those are VALU work and are reported separately.
    """
    if not causal:
        return 4 * B * H * N * N * D
    return 4 * B * H * D * (N * (N + 1) // 2)
