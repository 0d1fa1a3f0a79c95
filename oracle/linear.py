"""GEMV / GEMM / tensor-parallel oracles in float64 (test infrastructure only)."""
from __future__ import annotations

import numpy as np


def gemv(w, x):
    """y = W x, ``torch.mv(weight, x)`` of ``ch03/gemv_benchmark.py:34-48``."""
    return np.asarray(w, dtype=np.float64) @ np.asarray(x, dtype=np.float64)


def batched_gemv(x, w):
    """Y = X W^T, ``x @ weight.T`` of ``ch03/batching_benchmark.py:25-39``."""
    return np.asarray(x, dtype=np.float64) @ np.asarray(w, dtype=np.float64).T


def gemm(a, b):
    """C = A B (NN), ``torch.mm(a, b)`` of ``ch03/gemm_benchmark.py:35-49``."""
    return np.asarray(a, dtype=np.float64) @ np.asarray(b, dtype=np.float64)


def linear(x, w, bias=None):
    """Y = X W^T + b, ``F.linear`` as called in ``ch09/tensor_parallel.py:39,67``."""
    y = np.asarray(x, dtype=np.float64) @ np.asarray(w, dtype=np.float64).T
    if bias is not None:
        y = y + np.asarray(bias, dtype=np.float64)
    return y


def row_parallel_sum(x_full, w_full, world_size: int):
    """Sum over ranks of the row-parallel partials X[:, s_r] W[:, s_r]^T.

    ``RowParallelLinear`` (``ch09/tensor_parallel.py:43-68``) holds the column
    slice s_r of W; the all-reduce this build adds must reproduce the full
    ``F.linear(x_full, w_full)``.
    """
    x_full = np.asarray(x_full, dtype=np.float64)
    w_full = np.asarray(w_full, dtype=np.float64)
    k = x_full.shape[-1]
    assert k % world_size == 0
    part = k // world_size
    total = np.zeros(x_full.shape[:-1] + (w_full.shape[0],))
    for r in range(world_size):
        s = slice(r * part, (r + 1) * part)
        total += x_full[..., s] @ w_full[:, s].T
    return total


def silu(x):
    """x * sigmoid(x) (``F.silu``), float64."""
    x = np.asarray(x, dtype=np.float64)
    return x / (1.0 + np.exp(-x))


def swiglu(x, w_gate, w_up):
    """h = silu(x Wg^T) * (x Wu^T): the SwiGLU product of ``ch01/ffn.py:26-30``
    and ``ch09/tensor_parallel.py:95-98`` (per rank: column shards of Wg/Wu)."""
    x = np.asarray(x, dtype=np.float64)
    return silu(x @ np.asarray(w_gate, np.float64).T) * (x @ np.asarray(w_up, np.float64).T)


def swiglu_ffn(x, w_gate, w_up, w_down):
    """down(silu(gate(x)) * up(x)), ``SwiGLUFFN.forward`` (``ch01/ffn.py:26-31``)."""
    return swiglu(x, w_gate, w_up) @ np.asarray(w_down, np.float64).T


def rms_norm(x, weight, eps=1e-6, residual=None):
    """x / sqrt(mean(x^2) + eps) * weight over the last dim, float64
    (``RMSNorm.forward``, ``ch02/cached_generation.py:101-109``); with a
    residual, of h = x + residual (``CachedTransformerBlock``, ``:143-145``)."""
    h = np.asarray(x, np.float64)
    if residual is not None:
        h = h + np.asarray(residual, np.float64)
    return h / np.sqrt(np.mean(h * h, axis=-1, keepdims=True) + eps) * np.asarray(weight, np.float64)


def moe_route(logits, top_k, normalize=True):
    """Router of ``ch09/moe_layer.py:24-33`` in float64: softmax, top-k
    (descending, ties to the lower index), optional renormalisation."""
    lg = np.asarray(logits, np.float64)
    p = np.exp(lg - lg.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    idx = np.argsort(-p, axis=-1, kind="stable")[:, :top_k]
    w = np.take_along_axis(p, idx, -1)
    if normalize:
        w = w / w.sum(-1, keepdims=True)
    return w, idx


def moe_layer(x, gate_w, experts, top_k, normalize=True):
    """``MoELayer.forward`` (``ch09/moe_layer.py:58-83``) in float64:
    out[t] = sum_k w[t,k] * W2_e (silu(W1_e x) * W3_e x), e = idx[t,k];
    experts = [(w1, w2, w3), ...] as nn.Linear weights."""
    x = np.asarray(x, np.float64)
    w, idx = moe_route(x @ np.asarray(gate_w, np.float64).T, top_k, normalize)
    out = np.zeros_like(x)
    for t in range(x.shape[0]):
        for j in range(top_k):
            w1, w2, w3 = experts[idx[t, j]]
            out[t] += w[t, j] * swiglu_ffn(x[t:t + 1], w1, w3, w2)[0]
    return out
