"""Chapter 05 on MI355X: the HIP tiled GEMM, HBM coalescing probes, LDS
tiling helpers and the MFMA probe (Triton is dropped; ``triton_matmul`` runs
the HIP GEMM)."""

from .memory_coalescing import (
    AccessPatternResult,
    coalesced_access,
    measure_access_pattern,
    strided_access,
)
from .shared_memory import demonstrate_bank_conflicts, tiled_reduce
from .tensor_cores import benchmark_tensor_cores, tensor_core_info
from .tiled_matmul import benchmark_matmul_demo, benchmark_tiled_matmul, naive_matmul, tiled_matmul
from .triton_matmul import benchmark_triton_matmul, triton_matmul

__all__ = [
    "AccessPatternResult",
    "coalesced_access",
    "strided_access",
    "measure_access_pattern",
    "tiled_reduce",
    "demonstrate_bank_conflicts",
    "tiled_matmul",
    "naive_matmul",
    "benchmark_matmul_demo",
    "triton_matmul",
    "benchmark_triton_matmul",
    "benchmark_tiled_matmul",
    "tensor_core_info",
    "benchmark_tensor_cores",
]
