"""Graph-captured decode -- mirror of ``ch08/cuda_graph.py``.

``GraphConfig`` / ``CUDAGraphRunner`` keep the reference's API
(``ch08/cuda_graph.py:7-82``): one captured graph per batch size around a
``model_fn(static_input)``.  On ROCm ``torch.cuda.CUDAGraph`` is a HIP graph,
and every libpli_hip entry point is stream-ordered with no host sync or
allocation, so the HIP kernels capture as they are.

``DecodeStepGraph`` (this build) is what makes that useful for KV-cache
generation: a decode step whose cache length is a host value cannot be
replayed (the length is baked into the captured launches).  With caches from
``CachedTransformerModel.create_caches(..., device_pos=True)`` the append
(``pli_kv_append``) and the attention (``pli_attn_decode_dev``) read the
length from one device int that the step itself advances, so ONE capture
serves every later token: a step is one ``hipGraphLaunch`` instead of
~(10 x layers) kernel launches from Python.
"""
from __future__ import annotations

from collections.abc import Callable
from dataclasses import dataclass

import torch


@dataclass
class GraphConfig:
    batch_sizes: list[int] = None
    max_seq_len: int = 2048
    warmup_iterations: int = 3

    def __post_init__(self):
        if self.batch_sizes is None:
            self.batch_sizes = [1, 2, 4, 8, 16, 32]


class CUDAGraphRunner:
    """Capture ``model_fn`` once per batch size; replay with new inputs copied
    into the static input buffer (``ch08/cuda_graph.py:18-82``)."""

    def __init__(self, config: GraphConfig, model_fn: Callable | None = None):
        self.config = config
        self.model_fn = model_fn
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.static_inputs: dict[int, dict[str, torch.Tensor]] = {}
        self.static_outputs: dict[int, torch.Tensor] = {}

    def capture_graph(self, batch_size: int, input_shape: tuple, dtype: torch.dtype = torch.float16,
                      device: str = "cuda") -> bool:
        if not torch.cuda.is_available() or self.model_fn is None:
            return False
        static_input = torch.zeros(batch_size, *input_shape, dtype=dtype, device=device)
        for _ in range(self.config.warmup_iterations):
            self.model_fn(static_input)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_output = self.model_fn(static_input)
        self.graphs[batch_size] = graph
        self.static_inputs[batch_size] = {"input": static_input}
        self.static_outputs[batch_size] = static_output
        return True

    def run_graph(self, batch_size: int, input_tensor: torch.Tensor) -> torch.Tensor | None:
        if batch_size not in self.graphs:
            return None
        self.static_inputs[batch_size]["input"].copy_(input_tensor)
        self.graphs[batch_size].replay()
        return self.static_outputs[batch_size].clone()

    def has_graph(self, batch_size: int) -> bool:
        return batch_size in self.graphs

    def get_captured_batch_sizes(self) -> list[int]:
        return list(self.graphs.keys())


class DecodeStepGraph:
    """One captured single-token decode step of a ``ch02.CachedTransformerModel``.

        g = DecodeStepGraph(model, batch_size=8, max_seq_len=4096, dtype=torch.bfloat16)
        logits = g.prefill(prompt_ids)           # eager; fills the caches
        for _ in range(n):
            tok = sample(logits[:, -1])
            logits = g.step(tok)                 # one graph launch per token

    ``step`` returns the static logits buffer [B, 1, vocab] (overwritten by the
    next step; clone to keep it).
    """

    def __init__(self, model, batch_size: int, max_seq_len: int, dtype: torch.dtype,
                 device: torch.device | str = "cuda", warmup: int = 2):
        self.model = model
        self.caches = model.create_caches(batch_size, max_seq_len, torch.device(device), dtype,
                                          device_pos=True)
        self.pos = self.caches[0].pos
        self.static_ids = torch.zeros(batch_size, 1, dtype=torch.long, device=device)
        self.graph: torch.cuda.CUDAGraph | None = None
        self.static_logits: torch.Tensor | None = None
        self.warmup = warmup

    @property
    def seq_len(self) -> int:
        return self.caches[0].seq_len

    def _set_len(self, n: int) -> None:
        for c in self.caches:
            c.seq_len = n
        self.pos.fill_(n)

    @torch.no_grad()
    def prefill(self, input_ids: torch.Tensor) -> torch.Tensor:
        logits = self.model(input_ids, self.caches, start_pos=self.seq_len)
        if self.graph is None:
            self._capture()
        return logits

    @torch.no_grad()
    def _capture(self) -> None:
        # warm-up and capture run real steps; they write row `n` of every cache,
        # which the first replayed step overwrites, and the length is restored
        n = self.seq_len
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.model(self.static_ids, self.caches, start_pos=n)
                self._set_len(n)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_logits = self.model(self.static_ids, self.caches, start_pos=n)
        torch.cuda.synchronize()
        self._set_len(n)

    @torch.no_grad()
    def step(self, token_ids: torch.Tensor) -> torch.Tensor:
        if self.graph is None:
            raise RuntimeError("DecodeStepGraph.step before prefill")
        if self.seq_len >= self.caches[0].k.shape[1]:
            raise RuntimeError("KV cache full")
        self.static_ids.copy_(token_ids.view_as(self.static_ids))
        self.graph.replay()
        for c in self.caches:  # host bookkeeping of the device-side append
            c.seq_len += 1
        return self.static_logits


def explain_cuda_graphs() -> str:
    return """
HIP graphs on MI355X (torch.cuda.CUDAGraph on ROCm)

Problem: a decode step is ~10 kernels per layer; from Python each launch
costs several microseconds of host time, more than the kernels themselves at
small batch.

Solution: capture the step once, replay it with one launch.
  - every libpli_hip entry point is stream-ordered, allocation-free and
    sync-free, so it captures as is;
  - the KV-cache length lives in device memory (pli_kv_append,
    pli_attn_decode_dev), so one capture serves every token position;
  - new tokens are copied into the static input buffer before each replay.
"""


def benchmark_graph_vs_eager(model_fn: Callable, input_shape: tuple, batch_size: int = 1,
                             iterations: int = 100, warmup: int = 10, device: str = "cuda") -> dict | None:
    """Per-call time of ``model_fn`` launched eagerly vs captured once and
    replayed as a HIP graph (``ch08/cuda_graph.py:128-182``): wall clock with a
    sync on both sides of the loop, microseconds per call, after ``warmup``
    untimed calls of each form (the graph's are replays).  Returns the
    reference's keys; checking the replayed output is the caller's business
    (a model_fn with random ops legitimately differs call to call)."""
    import time

    if not torch.cuda.is_available():
        return None
    x = torch.randn(batch_size, *input_shape, device=device)

    def per_call(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iterations):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iterations * 1e6

    eager_us = per_call(lambda: model_fn(x))
    static_in = torch.zeros_like(x)
    for _ in range(warmup):  # (allocations made before the capture)
        model_fn(static_in)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_out = model_fn(static_in)

    def replay():
        static_in.copy_(x)
        graph.replay()

    graph_us = per_call(replay)  # (its warm-up calls are graph replays)
    del static_out
    return {"batch_size": batch_size, "input_shape": input_shape, "eager_us": eager_us, "graph_us": graph_us,
            "speedup": eager_us / graph_us}


if __name__ == "__main__":
    # the chapter's demo (ch08/cuda_graph.py:185-214): a three-op elementwise
    # model, eager vs one graph launch
    print(explain_cuda_graphs())
    if torch.cuda.is_available():
        print("\n" + "=" * 60 + "\nHIP Graph Benchmark\n" + "-" * 60)
        for b in (1, 4, 16):
            r = benchmark_graph_vs_eager(lambda t: torch.sigmoid(torch.relu(t) * 2.0), (1024,), batch_size=b,
                                         iterations=1000)
            print(f"Batch {b:3d}: Eager={r['eager_us']:.1f}us, Graph={r['graph_us']:.1f}us, Speedup={r['speedup']:.2f}x")
    else:
        print("\nno ROCm device")
