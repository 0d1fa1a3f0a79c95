"""Tensor-parallel linear layers -- mirror of ``ch09/tensor_parallel.py``, with
the communication the reference only describes made real.

Reference behaviour kept (``:15-100``): the same constructor arguments, the
same shard shapes (column: W [out/ws, in]; row: W [out, in/ws]), the same
``kaiming_uniform_`` init order, ``RowParallelLinear`` ignores its bias and
returns the partial product when it runs outside a process group, so the
single-process ``world_size=4`` behaviour is unchanged.

MI355X additions:

* on a ROCm device every shard GEMM is the HIP kernel ``pli_gemm``
  (NT layout: W stays [out, in] row-major; bias fused in the epilogue);
* when ``torch.distributed`` is initialised with ``world_size`` ranks,
  ``RowParallelLinear.forward`` completes the row-parallel product with
  ``all_reduce(SUM)`` -- backend "nccl", which is RCCL over xGMI on ROCm
  (one process per GPU, launched by torchrun);
* ``row_parallel_forward_overlapped`` splits the rows of X into chunks and
  all-reduces chunk i (async, on RCCL's stream) while the GEMM of chunk i+1
  runs, hiding compute under the xGMI transfer.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

import pli_hip


@dataclass
class TensorParallelConfig:
    world_size: int = 1
    rank: int = 0
    hidden_dim: int = 4096
    intermediate_dim: int = 14336


def _shard_linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """y = x W^T (+ b) on the local shard; HIP on ROCm tensors."""
    if not x.is_cuda:
        return F.linear(x, w, bias)
    lead = x.shape[:-1]
    y = pli_hip.gemm(x.reshape(-1, x.shape[-1]), w.detach(), trans_b=True,
                     bias=None if bias is None else bias.detach())
    return y.view(*lead, w.shape[0])


def _shard_linear_f32(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x W^T in fp32 (the unrounded partial); HIP pli_gemm_f32out on ROCm."""
    lead = x.shape[:-1]
    if not x.is_cuda:
        return F.linear(x.float(), w.detach().float())
    y = pli_hip.gemm_f32out(x.reshape(-1, x.shape[-1]), w.detach())
    return y.view(*lead, w.shape[0])


def tp_group_active(world_size: int, group=None) -> bool:
    """True when a process group of exactly ``world_size`` ranks exists.  A
    one-rank layer reduces only through a group passed to it explicitly (the
    reference's single-process behaviour stays the default)."""
    return ((world_size > 1 or group is not None) and dist.is_available() and dist.is_initialized()
            and dist.get_world_size(group) == world_size)


class ColumnParallelLinear(nn.Module):
    """Y_r = X W_r^T + b_r with W_r the rank's [out/ws, in] row block.  No
    communication: like the reference, the layer returns its output shard."""

    def __init__(self, in_features: int, out_features: int, world_size: int = 1, rank: int = 0,
                 bias: bool = False):
        super().__init__()
        self.world_size = world_size
        self.rank = rank
        assert out_features % world_size == 0
        self.out_features_per_partition = out_features // world_size
        self.weight = nn.Parameter(torch.empty(self.out_features_per_partition, in_features))
        self.bias = nn.Parameter(torch.zeros(self.out_features_per_partition)) if bias else None
        nn.init.kaiming_uniform_(self.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _shard_linear(x, self.weight, self.bias)


class RowParallelLinear(nn.Module):
    """Y = sum_r X_r W_r^T with W_r the rank's [out, in/ws] column block.

    ``reduce_dtype=torch.float32`` keeps each rank's partial in fp32 (HIP
    ``pli_gemm_f32out`` on ROCm) through the all-reduce and rounds the sum to
    the input dtype once; the default rounds every partial to the input dtype
    first (the reference's F.linear output), so TP ranks stack that many
    roundings (error by TP degree: bench.py ``tp_gemm.partial_rounding``)."""

    def __init__(self, in_features: int, out_features: int, world_size: int = 1, rank: int = 0,
                 bias: bool = False, group=None, reduce_dtype: torch.dtype | None = None):
        super().__init__()
        self.world_size = world_size
        self.rank = rank
        self.group = group
        assert reduce_dtype in (None, torch.float32), "reduce_dtype: None or torch.float32"
        self.reduce_dtype = reduce_dtype
        assert in_features % world_size == 0
        self.in_features_per_partition = in_features // world_size
        self.weight = nn.Parameter(torch.empty(out_features, self.in_features_per_partition))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        nn.init.kaiming_uniform_(self.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.reduce_dtype is not None and x.dtype != self.reduce_dtype:
            y = _shard_linear_f32(x, self.weight)  # reference ignores the bias (:66-68)
            if tp_group_active(self.world_size, self.group):
                dist.all_reduce(y, op=dist.ReduceOp.SUM, group=self.group)
            return y.to(x.dtype)
        y = _shard_linear(x, self.weight, None)  # reference ignores the bias (:66-68)
        if tp_group_active(self.world_size, self.group):
            dist.all_reduce(y, op=dist.ReduceOp.SUM, group=self.group)
        return y


def row_parallel_forward_overlapped(x: torch.Tensor, weight: torch.Tensor, chunks: int = 4,
                                    group=None, world_size: int | None = None,
                                    reduce_dtype: torch.dtype | None = None) -> torch.Tensor:
    """Chunked RowParallel forward: GEMM of rows-chunk i+1 overlaps the async
    all-reduce of chunk i (RCCL runs on its own stream, ordered after the
    chunk's GEMM on the current stream; ``wait`` orders the caller after all
    of them).  ``world_size`` is the layer's TP degree (default: the group's
    size) and gates the all-reduce exactly as ``RowParallelLinear.forward``
    does (``tp_group_active``); ``reduce_dtype=torch.float32`` keeps the
    partials in fp32 (``pli_gemm_f32out``) through the all-reduce and rounds
    the sum once.  Same result as ``RowParallelLinear.forward`` up to the
    per-chunk GEMM's accumulation order."""
    assert reduce_dtype in (None, torch.float32), "reduce_dtype: None or torch.float32"
    if world_size is None:
        world_size = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    reduce = tp_group_active(world_size, group)
    x2 = x.reshape(-1, x.shape[-1])
    m = x2.shape[0]
    f32 = reduce_dtype is not None and x.dtype != reduce_dtype
    out = torch.empty(m, weight.shape[0], dtype=torch.float32 if f32 else x.dtype, device=x.device)
    bounds = [m * i // chunks for i in range(chunks + 1)]
    handles = []
    for i in range(chunks):
        lo, hi = bounds[i], bounds[i + 1]
        if hi == lo:
            continue
        part = out[lo:hi]
        if f32 and x2.is_cuda:
            pli_hip.gemm_f32out(x2[lo:hi], weight.detach(), out=part)
        elif f32:
            part.copy_(F.linear(x2[lo:hi].float(), weight.detach().float()))
        elif x2.is_cuda:
            pli_hip.gemm(x2[lo:hi], weight.detach(), trans_b=True, out=part)
        else:
            part.copy_(F.linear(x2[lo:hi], weight))
        if reduce:
            handles.append(dist.all_reduce(part, op=dist.ReduceOp.SUM, group=group, async_op=True))
    for h in handles:
        h.wait()
    if f32:
        out = out.to(x.dtype)
    return out.view(*x.shape[:-1], weight.shape[0])


class TensorParallelMLP(nn.Module):
    """gate/up column-parallel, down row-parallel: one all-reduce per MLP."""

    def __init__(self, config: TensorParallelConfig):
        super().__init__()
        self.config = config
        self.gate_proj = ColumnParallelLinear(config.hidden_dim, config.intermediate_dim,
                                              config.world_size, config.rank)
        self.up_proj = ColumnParallelLinear(config.hidden_dim, config.intermediate_dim,
                                            config.world_size, config.rank)
        self.down_proj = RowParallelLinear(config.intermediate_dim, config.hidden_dim,
                                           config.world_size, config.rank)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            # gate/up column shards fused with the SwiGLU product in one launch
            # (pli_gemm_swiglu): the rank's [.., I/tp] gate and up activations
            # never reach HBM; down_proj then all-reduces as before
            lead = x.shape[:-1]
            h = pli_hip.gemm_swiglu(x.reshape(-1, x.shape[-1]), self.gate_proj.weight,
                                    self.up_proj.weight)
            return self.down_proj(h.view(*lead, h.shape[-1]))
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


def compute_tp_memory_savings(hidden_dim: int, intermediate_dim: int, world_size: int,
                              dtype_bytes: int = 2) -> dict:
    """MLP weight bytes dense vs per rank (gate + up + down = 3 h i params)."""
    params = 3 * hidden_dim * intermediate_dim
    per_gpu = params / world_size
    return {
        "dense_params": params,
        "dense_memory_mb": params * dtype_bytes / 1024 / 1024,
        "tp_params_per_gpu": per_gpu,
        "tp_memory_per_gpu_mb": per_gpu * dtype_bytes / 1024 / 1024,
        "memory_reduction": world_size,
    }


def explain_tensor_parallelism() -> str:
    """The reference's tensor-parallel primer (ch09/tensor_parallel.py:128-169),
    written for this build's kernels and fabric."""
    return (
        "\nTensor parallelism: one layer's weights split over N GPUs\n\n"
        "Column-parallel  Y = X W, W [in, out] cut along out: rank r holds W[:, r out/N ...]\n"
        "                 and produces its own slice of Y -- no communication.\n"
        "Row-parallel     W cut along in (and X with it): rank r computes a full-size\n"
        "                 partial product X_r W_r, and an all-reduce sums the N partials.\n\n"
        "A transformer pairs them: q/k/v and gate/up column-parallel, the attention\n"
        "output and down projections row-parallel -- one all-reduce per attention\n"
        "block and one per MLP in the forward pass, each of batch x seq x hidden\n"
        "elements.\n\n"
        "On MI355X: each rank's shard runs as an NT GEMM on the matrix cores\n"
        "(pli_gemm, gemm_w5 at large M), the gate/up pair as one fused SwiGLU launch\n"
        "(pli_gemm_swiglu), and the all-reduce goes over RCCL on the xGMI mesh,\n"
        "chunked along M so chunk i's all-reduce overlaps chunk i+1's GEMM\n"
        "(row_parallel_forward_overlapped).  Memory per GPU falls as 1/N; the cost\n"
        "is that communication, which at N = 8 and M = 8192 outweighs the GEMM.\n"
    )


if __name__ == "__main__":
    # the chapter's demo (ch09/tensor_parallel.py:171-203)
    print(explain_tensor_parallelism())
    print("\n" + "=" * 60 + "\nTensor Parallel MLP Demo\n" + "-" * 60)
    for n in (1, 2, 4, 8):
        m = compute_tp_memory_savings(hidden_dim=4096, intermediate_dim=14336, world_size=n)
        print(f"\nWorld size: {n}\n  Dense memory:  {m['dense_memory_mb']:.1f} MB\n"
              f"  Per-GPU memory: {m['tp_memory_per_gpu_mb']:.1f} MB")
    print("\n" + "-" * 60 + "\nSingle GPU simulation:")
    mlp = TensorParallelMLP(TensorParallelConfig(world_size=1, rank=0, hidden_dim=256, intermediate_dim=512))
    x = torch.randn(2, 16, 256)
    if torch.cuda.is_available():
        mlp, x = mlp.cuda(), x.cuda()
    y = mlp(x)
    print(f"Input shape:  {x.shape}\nOutput shape: {y.shape}")
