"""Transformer block and model -- mirror of ``ch01/transformer.py``.

Same classes, constructor signatures, parameter names and creation order as
the reference (``ch01/transformer.py:9-120``: ``input_layernorm``,
``self_attn``, ``post_attention_layernorm``, ``mlp``; ``embed_tokens``,
``layers``, ``norm``, ``lm_head``), so seeded models and ``state_dict``s are
interchangeable, and the two reference configs.

On a ROCm device every op of the block is a HIP kernel of this build:
``RMSNorm`` is one ``pli_rmsnorm`` launch (fp32 statistics), and the block
folds each residual add into the norm that follows it (``pli_rmsnorm`` with a
residual writes h = x + residual and y = norm(h) in one pass); the attention
is ``GroupedQueryAttention`` (4 ``pli_gemm`` + one causal flash launch, no
``repeat_interleave``), the MLP ``FusedSwiGLUFFN`` (gate/up/silu*mul in one
``pli_gemm_swiglu`` launch + ``pli_gemm``), ``lm_head`` ``pli_gemm``.  CPU
tensors run the reference math unchanged, so ``pytest ch01`` on CPU behaves
exactly like the reference's.
"""
from __future__ import annotations

import torch
import torch.nn as nn

import pli_hip

from .attention import _linear
from .ffn import FusedSwiGLUFFN
from .gqa import GroupedQueryAttention


class RMSNorm(nn.Module):
    def __init__(self, hidden_dim: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_dim))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return pli_hip.rmsnorm(x, self.weight.to(x.dtype), self.eps)
        rms = torch.sqrt(torch.mean(x ** 2, dim=-1, keepdim=True) + self.eps)
        return x / rms * self.weight


class TransformerBlock(nn.Module):
    def __init__(
        self,
        hidden_dim: int,
        num_heads: int,
        num_kv_heads: int,
        intermediate_dim: int,
        norm_eps: float = 1e-6,
    ):
        super().__init__()
        self.input_layernorm = RMSNorm(hidden_dim, eps=norm_eps)
        self.self_attn = GroupedQueryAttention(hidden_dim, num_heads, num_kv_heads)
        self.post_attention_layernorm = RMSNorm(hidden_dim, eps=norm_eps)
        self.mlp = FusedSwiGLUFFN(hidden_dim, intermediate_dim)

    def forward(self, x: torch.Tensor, causal: bool = True) -> torch.Tensor:
        if x.is_cuda:
            # h = x + attn(norm1(x)) and norm2(h) in one pli_rmsnorm launch
            a = self.self_attn(self.input_layernorm(x), causal=causal)
            pn = self.post_attention_layernorm
            h, n2 = pli_hip.rmsnorm(a, pn.weight.to(x.dtype), pn.eps, residual=x)
            return h + self.mlp(n2)
        residual = x
        x = self.input_layernorm(x)
        x = self.self_attn(x, causal=causal)
        x = residual + x
        residual = x
        x = self.post_attention_layernorm(x)
        x = self.mlp(x)
        x = residual + x
        return x


class TransformerModel(nn.Module):
    def __init__(
        self,
        vocab_size: int,
        hidden_dim: int,
        num_layers: int,
        num_heads: int,
        num_kv_heads: int,
        intermediate_dim: int,
        norm_eps: float = 1e-6,
    ):
        super().__init__()
        self.embed_tokens = nn.Embedding(vocab_size, hidden_dim)
        self.layers = nn.ModuleList([
            TransformerBlock(
                hidden_dim=hidden_dim,
                num_heads=num_heads,
                num_kv_heads=num_kv_heads,
                intermediate_dim=intermediate_dim,
                norm_eps=norm_eps,
            )
            for _ in range(num_layers)
        ])
        self.norm = RMSNorm(hidden_dim, eps=norm_eps)
        self.lm_head = nn.Linear(hidden_dim, vocab_size, bias=False)
        self.config = {
            "vocab_size": vocab_size,
            "hidden_dim": hidden_dim,
            "num_layers": num_layers,
            "num_heads": num_heads,
            "num_kv_heads": num_kv_heads,
            "intermediate_dim": intermediate_dim,
        }

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        x = self.embed_tokens(input_ids)
        for layer in self.layers:
            x = layer(x)
        x = self.norm(x)
        if x.is_cuda:
            return _linear(x, self.lm_head.weight)
        return self.lm_head(x)

    def count_parameters(self) -> dict:
        parts = {"embed_tokens": self.embed_tokens, "layers": self.layers, "norm": self.norm,
                 "lm_head": self.lm_head}
        out = {name: sum(p.numel() for p in mod.parameters()) for name, mod in parts.items()}
        out["total"] = sum(out.values())
        return out


# the two model shapes the reference ships (ch01/transformer.py:104-120)
LLAMA_7B_CONFIG = {
    "vocab_size": 32000,
    "hidden_dim": 4096,
    "num_layers": 32,
    "num_heads": 32,
    "num_kv_heads": 32,
    "intermediate_dim": 11008,
}

QWEN3_CONFIG = {
    "vocab_size": 151936,
    "hidden_dim": 4096,
    "num_layers": 32,
    "num_heads": 32,
    "num_kv_heads": 8,
    "intermediate_dim": 11008,
}
