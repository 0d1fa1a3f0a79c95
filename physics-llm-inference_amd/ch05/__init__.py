"""Chapter 05 on MI355X: the HIP tiled GEMM, HBM coalescing probes and the
MFMA probe (Triton is dropped; ``triton_matmul`` aliases the HIP GEMM)."""

from .memory_coalescing import (
    AccessPatternResult,
    coalesced_access,
    measure_access_pattern,
    strided_access,
)
from .tensor_cores import benchmark_tensor_cores, tensor_core_info
from .tiled_matmul import benchmark_tiled_matmul, tiled_matmul, triton_matmul

__all__ = [
    "AccessPatternResult",
    "coalesced_access",
    "strided_access",
    "measure_access_pattern",
    "tiled_matmul",
    "triton_matmul",
    "benchmark_tiled_matmul",
    "tensor_core_info",
    "benchmark_tensor_cores",
]
