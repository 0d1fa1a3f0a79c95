"""Chapter 09 on MI355X: tensor-parallel linear layers on the HIP GEMM with a
real RCCL all-reduce, the collective cost models, and the MoE layer on the
grouped expert GEMM, and the host-side expert cache / execution planner of
moe_inference.py (bookkeeping only, so the reference's test module loads)."""

from .moe_inference import (
    ExpertCache,
    ExpertUsageStats,
    MoEInferenceConfig,
    MoEInferenceEngine,
    explain_moe_inference,
)
from .moe_layer import (
    ExpertLayer,
    MoEConfig,
    MoELayer,
    Router,
    expert_load_balance_loss,
    explain_moe,
)
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
    "MoEConfig",
    "Router",
    "ExpertLayer",
    "MoELayer",
    "expert_load_balance_loss",
    "explain_moe",
    "MoEInferenceEngine",
    "MoEInferenceConfig",
    "ExpertCache",
    "ExpertUsageStats",
    "explain_moe_inference",
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
