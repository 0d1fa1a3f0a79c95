"""Mixture-of-experts layer -- mirror of ``ch09/moe_layer.py``.

``MoEConfig``, ``Router``, ``ExpertLayer``, ``MoELayer`` keep the
reference's constructors, parameter names and creation order
(``ch09/moe_layer.py:8-56``), so seeded layers are interchangeable.

On a ROCm device ``MoELayer.forward`` replaces the per-expert Python loop
(``:58-83``: a boolean mask, an ``x_flat[mask]`` gather, a full expert FFN
call and masked ``+=`` per expert and per top-k slot) with five launches:

1. router logits on ``pli_gemm``;
2. ``pli_moe_route``: softmax / top-k / renormalise + expert-sorted row
   tables (offsets, row -> token gather, (token, k) -> row);
3. ``pli_gemm_grouped`` with W1/W3: every expert's silu(x W1^T) * (x W3^T)
   over its own rows, X read through the gather table (no gathered copy),
   the weights through a device table of the experts' pointers;
4. ``pli_gemm_grouped`` with W2;
5. ``pli_moe_combine``: out[t] = sum_k w[t,k] * y[row(t,k)], fixed order.

Each active expert's weights are streamed once per call, whatever its token
count (decode sizes: a weight-streaming kernel; >= 16 rows per expert: the
phased 256-row MFMA tile per (expert, slot), rows gathered by LDS-DMA).  Shapes the grouped kernel does not take (K % 128, N % 16) run every
expert densely on the HIP GEMMs and mask by the routing weights (slow, only
for toy sizes).  CPU tensors keep the reference math.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

import pli_hip


@dataclass
class MoEConfig:
    hidden_dim: int = 4096
    expert_dim: int = 14336
    num_experts: int = 8
    num_experts_per_tok: int = 2
    normalize_expert_weights: bool = True


class Router(nn.Module):
    def __init__(self, config: MoEConfig):
        super().__init__()
        self.config = config
        self.gate = nn.Linear(config.hidden_dim, config.num_experts, bias=False)

    def _logits(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and self.config.num_experts % 8 == 0:
            return pli_hip.gemm(x.reshape(-1, x.shape[-1]), self.gate.weight, trans_b=True)
        return self.gate(x).reshape(-1, self.config.num_experts)

    def forward(self, x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        c = self.config
        if x.is_cuda and c.num_experts <= 64 and c.num_experts_per_tok <= 8:
            logits = self._logits(x)
            w, idx, _, _, _ = pli_hip.moe_route(logits, c.num_experts_per_tok,
                                                c.normalize_expert_weights)
            lead = x.shape[:-1]
            return (w.to(x.dtype).view(*lead, -1), idx.long().view(*lead, -1),
                    logits.view(*lead, -1))
        logits = self.gate(x)
        weights = F.softmax(logits, dim=-1)
        top_weights, top_indices = torch.topk(weights, c.num_experts_per_tok, dim=-1)
        if c.normalize_expert_weights:
            top_weights = top_weights / top_weights.sum(dim=-1, keepdim=True)
        return top_weights, top_indices, logits


class ExpertLayer(nn.Module):
    def __init__(self, hidden_dim: int, expert_dim: int):
        super().__init__()
        self.w1 = nn.Linear(hidden_dim, expert_dim, bias=False)
        self.w2 = nn.Linear(expert_dim, hidden_dim, bias=False)
        self.w3 = nn.Linear(hidden_dim, expert_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            lead = x.shape[:-1]
            h = pli_hip.gemm_swiglu(x.reshape(-1, x.shape[-1]), self.w1.weight, self.w3.weight)
            return pli_hip.gemm(h, self.w2.weight, trans_b=True).view(*lead, -1)
        return self.w2(F.silu(self.w1(x)) * self.w3(x))


class MoELayer(nn.Module):
    def __init__(self, config: MoEConfig):
        super().__init__()
        self.config = config
        self.router = Router(config)
        self.experts = nn.ModuleList([
            ExpertLayer(config.hidden_dim, config.expert_dim) for _ in range(config.num_experts)
        ])
        self._tables = None  # (pointer key, w1 table, w3 table, w2 table)

    def _weight_tables(self):
        key = tuple((e.w1.weight.data_ptr(), e.w3.weight.data_ptr(), e.w2.weight.data_ptr())
                    for e in self.experts)
        if self._tables is None or self._tables[0] != key:
            self._tables = (key,
                            pli_hip.weight_table([e.w1.weight for e in self.experts]),
                            pli_hip.weight_table([e.w3.weight for e in self.experts]),
                            pli_hip.weight_table([e.w2.weight for e in self.experts]))
        return self._tables[1:]

    def _grouped_ok(self, x: torch.Tensor) -> bool:
        c = self.config
        return (x.dtype in (torch.bfloat16, torch.float16) and c.hidden_dim % 128 == 0
                and c.expert_dim % 128 == 0 and c.num_experts <= 64 and c.num_experts_per_tok <= 8
                and c.num_experts % 8 == 0
                and all(e.w1.weight.is_contiguous() and e.w2.weight.is_contiguous()
                        and e.w3.weight.is_contiguous() for e in self.experts))

    def _forward_hip(self, x_flat: torch.Tensor) -> torch.Tensor:
        c = self.config
        T = x_flat.shape[0]
        k = c.num_experts_per_tok
        logits = self.router._logits(x_flat)
        w, _, pos, gather, offsets = pli_hip.moe_route(logits, k, c.normalize_expert_weights)
        t1, t3, t2 = self._weight_tables()
        rows = T * k
        h = pli_hip.gemm_grouped(x_flat, gather, t1, offsets, rows, c.expert_dim, c.hidden_dim,
                                 c.hidden_dim, wu_table=t3)
        y = pli_hip.gemm_grouped(h, None, t2, offsets, rows, c.hidden_dim, c.expert_dim,
                                 c.expert_dim)
        return pli_hip.moe_combine(y, pos, w, T)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        batch_size, seq_len, hidden_dim = x.shape
        x_flat = x.reshape(-1, hidden_dim)
        if x.is_cuda and self._grouped_ok(x):
            return self._forward_hip(x_flat.contiguous()).view(batch_size, seq_len, hidden_dim)
        weights, indices, _ = self.router(x_flat)
        output = torch.zeros_like(x_flat)
        if x.is_cuda:  # dense per-expert HIP path for shapes the grouped kernel does not take
            for e, expert in enumerate(self.experts):
                we = (weights * (indices == e)).sum(dim=-1, keepdim=True).to(x.dtype)
                output += we * expert(x_flat)
            return output.view(batch_size, seq_len, hidden_dim)
        for expert_idx in range(self.config.num_experts):
            mask = (indices == expert_idx).any(dim=-1)
            if not mask.any():
                continue
            expert_output = self.experts[expert_idx](x_flat[mask])
            for kk in range(self.config.num_experts_per_tok):
                combined = mask & (indices[:, kk] == expert_idx)
                if combined.any():
                    output[combined] += (weights[combined, kk].unsqueeze(-1)
                                         * expert_output[(indices[:, kk] == expert_idx)[mask]])
        return output.view(batch_size, seq_len, hidden_dim)


def expert_load_balance_loss(router_logits: torch.Tensor, num_experts: int,
                             num_experts_per_tok: int) -> torch.Tensor:
    """Switch-style auxiliary loss (``ch09/moe_layer.py:86-97``)."""
    probs = F.softmax(router_logits, dim=-1)
    avg_probs = probs.mean(dim=0)
    top_indices = torch.topk(probs, num_experts_per_tok, dim=-1).indices
    expert_mask = torch.zeros_like(probs).scatter_(-1, top_indices, 1.0)
    return num_experts * (avg_probs * expert_mask.mean(dim=0)).sum()


def explain_moe() -> str:
    return """
Mixture of Experts on MI355X

Router: logits = x Wg^T (pli_gemm), softmax + top-k + renormalise and the
expert-sorted row tables in one routing launch (pli_moe_route).
Experts: two grouped launches over all experts (pli_gemm_grouped): fused
SwiGLU (W1, W3) then W2, each expert's weights streamed once; tokens are
read through the gather table.  Combine: one deterministic weighted sum.
"""


if __name__ == "__main__":
    # the chapter's demo (ch09/moe_layer.py)
    print(explain_moe())
    print("\n" + "=" * 60 + "\nMoE Layer Demo\n" + "-" * 60)
    cfg = MoEConfig(hidden_dim=256, expert_dim=512, num_experts=8, num_experts_per_tok=2)
    moe = MoELayer(cfg)
    x = torch.randn(2, 16, 256)
    if torch.cuda.is_available():
        moe, x = moe.cuda(), x.cuda()
    y = moe(x)
    print(f"Input shape:  {x.shape}\nOutput shape: {y.shape}")
    total = sum(p.numel() for p in moe.parameters())
    per_expert = sum(p.numel() for p in moe.experts[0].parameters())
    print(f"\nTotal params:        {total:,}\nParams per expert:   {per_expert:,}\n"
          f"Active params/token: {per_expert * cfg.num_experts_per_tok:,}")
