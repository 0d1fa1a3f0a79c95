"""Chapter 09 on MI355X: tensor-parallel linear layers on the HIP GEMM with a
real RCCL all-reduce, and the collective cost models (MoE is out of scope)."""

from .nccl_primitives import (
    AllGatherConfig,
    AllReduceConfig,
    compute_communication_overlap_potential,
    compute_ring_all_reduce_time,
    simulate_all_gather,
    simulate_all_reduce,
    xgmi_all_reduce_bounds,
)
from .tensor_parallel import (
    ColumnParallelLinear,
    RowParallelLinear,
    TensorParallelConfig,
    TensorParallelMLP,
    compute_tp_memory_savings,
    row_parallel_forward_overlapped,
)

__all__ = [
    "TensorParallelConfig",
    "ColumnParallelLinear",
    "RowParallelLinear",
    "TensorParallelMLP",
    "compute_tp_memory_savings",
    "row_parallel_forward_overlapped",
    "AllReduceConfig",
    "AllGatherConfig",
    "simulate_all_reduce",
    "simulate_all_gather",
    "compute_ring_all_reduce_time",
    "compute_communication_overlap_potential",
    "xgmi_all_reduce_bounds",
]
