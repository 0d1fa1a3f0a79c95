"""Chapter 08 on MI355X: graph-captured decode (the hot-path part).

The chunked-prefill / mixed-batch / overlap schedulers of the reference's
ch08 are control plane (SURVEY.md §8 out of scope) and are not mirrored.
"""

from .cuda_graph import CUDAGraphRunner, DecodeStepGraph, GraphConfig, explain_cuda_graphs

__all__ = ["CUDAGraphRunner", "DecodeStepGraph", "GraphConfig", "explain_cuda_graphs"]
