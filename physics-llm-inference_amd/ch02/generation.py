"""Naive (no-cache) generation -- mirror of ``ch02/generation.py``.

``naive_generate`` keeps the reference's signature and sampling
(``ch02/generation.py:10-34``: temperature, optional top-k, multinomial) and
re-runs the whole ``ch01.TransformerModel`` over the growing sequence per
token -- on a ROCm device every layer of that model is a HIP kernel of this
build (``ch01/transformer.py``).  It is the baseline ``cached_generate``
is measured against.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ch01.transformer import TransformerModel


def naive_generate(model: TransformerModel, input_ids: torch.Tensor, max_new_tokens: int,
                   temperature: float = 1.0, top_k: int | None = None) -> torch.Tensor:
    model.eval()
    generated = input_ids.clone()
    with torch.no_grad():
        for _ in range(max_new_tokens):
            next_logits = model(generated)[:, -1, :] / temperature
            if top_k is not None:
                values, indices = torch.topk(next_logits, top_k)
                next_logits = torch.full_like(next_logits, float("-inf")).scatter_(1, indices, values)
            next_token = torch.multinomial(F.softmax(next_logits, dim=-1), num_samples=1)
            generated = torch.cat([generated, next_token], dim=1)
    return generated
