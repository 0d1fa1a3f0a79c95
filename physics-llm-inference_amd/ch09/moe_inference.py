"""MoE inference bookkeeping: an LRU cache of expert weights, a per-batch
execution plan and routing statistics (reference ch09/moe_inference.py:1-126).

Host-side control logic only -- no kernel runs here.  On MI355X the sizing
is different from the reference's premise: 288 GB of HBM holds every expert
of an 8x7B model (~94 GB in bf16) with room to spare, so the cache is mostly
a way to keep a *working set* of device-resident experts when several
models or very large expert counts share a GPU.  The expert GEMMs
themselves run on the grouped HIP kernel behind ``ch09.MoELayer``
(``pli_gemm_grouped``).

Differences from the reference that do not change results:
  * ``update_batch_stats`` counts and sums per expert with two ``bincount``
    passes instead of one masked reduction per expert (weights summed in
    float64; the reference sums each masked float32 slice).
  * ``ExpertCache`` may be given a ``device``; added weights are moved there
    (the default, None, stores the tensor as given, like the reference).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import torch


@dataclass
class ExpertUsageStats:
    """Per-expert counters (reference moe_inference.py:7-13)."""
    expert_id: int
    tokens_routed: int = 0
    total_weight: float = 0.0
    cache_hits: int = 0
    cache_misses: int = 0


class ExpertCache:
    """Least-recently-used set of at most ``max_experts_in_memory`` expert
    weight tensors (reference moe_inference.py:16-54): a lookup refreshes the
    entry and counts a hit, a miss is counted per lookup, adding to a full
    cache evicts the least recently used entry and returns its id."""

    def __init__(self, max_experts_in_memory: int, num_total_experts: int,
                 device: torch.device | str | None = None):
        self.max_experts = max_experts_in_memory
        self.num_total_experts = num_total_experts
        self.device = device
        self.cached_experts: OrderedDict[int, torch.Tensor] = OrderedDict()
        self.stats: dict[int, ExpertUsageStats] = {e: ExpertUsageStats(expert_id=e)
                                                   for e in range(num_total_experts)}

    def get_expert(self, expert_id: int) -> torch.Tensor | None:
        w = self.cached_experts.get(expert_id)
        if w is None:
            self.stats[expert_id].cache_misses += 1
            return None
        self.cached_experts.move_to_end(expert_id)
        self.stats[expert_id].cache_hits += 1
        return w

    def add_expert(self, expert_id: int, weights: torch.Tensor) -> int | None:
        evicted = None
        if len(self.cached_experts) >= self.max_experts:
            evicted, _ = self.cached_experts.popitem(last=False)
        if self.device is not None:
            weights = weights.to(self.device, non_blocking=True)
        self.cached_experts[expert_id] = weights
        return evicted

    def get_cache_hit_rate(self) -> float:
        hits = sum(s.cache_hits for s in self.stats.values())
        total = hits + sum(s.cache_misses for s in self.stats.values())
        return hits / total if total else 0.0

    def get_cached_expert_ids(self) -> list[int]:
        return list(self.cached_experts)


@dataclass
class MoEInferenceConfig:
    """Same fields and defaults as reference moe_inference.py:57-62."""
    num_experts: int = 8
    num_experts_per_tok: int = 2
    max_experts_in_gpu: int = 4
    enable_expert_offload: bool = False


class MoEInferenceEngine:
    """Plans which experts of a routed batch are resident and which must be
    loaded, and accumulates routing statistics (reference
    moe_inference.py:65-126)."""

    def __init__(self, config: MoEInferenceConfig):
        self.config = config
        self.expert_cache = ExpertCache(max_experts_in_memory=config.max_experts_in_gpu,
                                        num_total_experts=config.num_experts)
        self.batch_expert_usage: dict[int, int] = {}

    def plan_expert_execution(self, expert_indices: torch.Tensor) -> dict:
        """Unique experts of ``expert_indices`` in ascending order, split into
        cache hits and loads (every lookup updates the cache's counters)."""
        unique = torch.unique(expert_indices).tolist()
        in_cache, need_load = [], []
        for e in unique:
            (in_cache if self.expert_cache.get_expert(e) is not None else need_load).append(e)
        return {"in_cache": in_cache, "need_load": need_load, "total_unique": len(unique)}

    def update_batch_stats(self, expert_indices: torch.Tensor, expert_weights: torch.Tensor) -> None:
        n = self.config.num_experts
        idx = expert_indices.reshape(-1).to("cpu", torch.int64)
        w = expert_weights.reshape(-1).to("cpu", torch.float64)
        keep = (idx >= 0) & (idx < n)  # the reference only visits ids 0..n-1
        idx, w = idx[keep], w[keep]
        counts = torch.bincount(idx, minlength=n).tolist()
        sums = torch.bincount(idx, weights=w, minlength=n).tolist()
        for e in range(n):
            if counts[e] > 0:
                st = self.expert_cache.stats[e]
                st.tokens_routed += counts[e]
                st.total_weight += sums[e]

    def get_load_balance_metrics(self) -> dict:
        loads = [s.tokens_routed for s in self.expert_cache.stats.values()]
        total = sum(loads)
        if total == 0:
            return {"balance_ratio": 1.0, "max_load": 0, "min_load": 0}
        hi, lo = max(loads), min(loads)
        return {"balance_ratio": lo / hi if hi > 0 else 1.0,
                "max_load": hi,
                "min_load": lo,
                "expected": total / self.config.num_experts,
                "std_dev": torch.tensor(loads, dtype=torch.float32).std().item()}


def explain_moe_inference() -> str:
    return """
MoE inference on MI355X

Memory: 288 GB of HBM3E per GPU.  An 8-expert 7B-class MoE (~47B params,
~94 GB bf16) fits whole on one GPU; a 128-expert 30B model does too.  Expert
offloading to host memory is a fallback for multi-tenant or very large
expert counts, not the default.

Execution:
  - Route, then group tokens by expert and run every expert's GEMM in one
    grouped HIP launch (pli_gemm_grouped), so small experts share the chip.
  - Expert parallelism across GPUs needs an all-to-all over xGMI
    (point-to-point links, ~153 GB/s each): keep dispatch buffers large and
    few.
  - An LRU cache of device-resident experts (ExpertCache) serves skewed
    routing; plan_expert_execution lists hits and loads before the step so
    loads can be issued on a copy stream ahead of the GEMMs.

Balance: unbalanced routing leaves grouped-GEMM tiles idle; track per-expert
token counts (update_batch_stats / get_load_balance_metrics).
"""


if __name__ == "__main__":
    print(explain_moe_inference())
    eng = MoEInferenceEngine(MoEInferenceConfig())
    idx = torch.tensor([[0, 1], [0, 2], [1, 3], [2, 3], [0, 4], [1, 5], [4, 5], [6, 7]])
    wts = torch.rand(idx.shape)
    wts = wts / wts.sum(-1, keepdim=True)
    print(eng.plan_expert_execution(idx))
    eng.update_batch_stats(idx, wts)
    print(eng.get_load_balance_metrics())
