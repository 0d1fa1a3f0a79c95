"""Feed-forward blocks -- mirror of ``ch01/ffn.py``.

Same classes, parameter names and creation order (``ch01/ffn.py:6-57``).  On a
ROCm device the SwiGLU variants run gate + up + silu·mul as ONE
``pli_gemm_swiglu`` launch (neither the gate nor the up activation is written
to HBM) followed by the down projection on ``pli_gemm``;
``FusedSwiGLUFFN``'s concatenated ``gate_up_proj`` weight is passed as its two
row halves (views, no copy).  ``NaiveFFN`` runs up/down on ``pli_gemm``.  CPU
tensors keep the reference math.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import pli_hip

from .attention import _linear


def _swiglu_down(x: torch.Tensor, w_gate: torch.Tensor, w_up: torch.Tensor,
                 w_down: torch.Tensor) -> torch.Tensor:
    lead = x.shape[:-1]
    h = pli_hip.gemm_swiglu(x.reshape(-1, x.shape[-1]), w_gate, w_up)
    return _linear(h, w_down).view(*lead, w_down.shape[0])


class NaiveFFN(nn.Module):
    def __init__(self, hidden_dim: int, intermediate_dim: int):
        super().__init__()
        self.up_proj = nn.Linear(hidden_dim, intermediate_dim, bias=False)
        self.down_proj = nn.Linear(intermediate_dim, hidden_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return _linear(F.relu(_linear(x, self.up_proj.weight)), self.down_proj.weight)
        return self.down_proj(F.relu(self.up_proj(x)))


class SwiGLUFFN(nn.Module):
    def __init__(self, hidden_dim: int, intermediate_dim: int):
        super().__init__()
        self.gate_proj = nn.Linear(hidden_dim, intermediate_dim, bias=False)
        self.up_proj = nn.Linear(hidden_dim, intermediate_dim, bias=False)
        self.down_proj = nn.Linear(intermediate_dim, hidden_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return _swiglu_down(x, self.gate_proj.weight, self.up_proj.weight,
                                self.down_proj.weight)
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


class FusedSwiGLUFFN(nn.Module):
    def __init__(self, hidden_dim: int, intermediate_dim: int):
        super().__init__()
        self.gate_up_proj = nn.Linear(hidden_dim, 2 * intermediate_dim, bias=False)
        self.down_proj = nn.Linear(intermediate_dim, hidden_dim, bias=False)
        self.intermediate_dim = intermediate_dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        i = self.intermediate_dim
        if x.is_cuda:
            w = self.gate_up_proj.weight
            return _swiglu_down(x, w[:i], w[i:], self.down_proj.weight)
        gate_up = self.gate_up_proj(x)
        return self.down_proj(F.silu(gate_up[..., :i]) * gate_up[..., i:])
