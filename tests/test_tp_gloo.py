"""Multi-process tensor parallelism on CPU (gloo, world_size 2).

Exercises the distributed code path of ``ch09.RowParallelLinear`` /
``row_parallel_forward_overlapped`` -- the all-reduce that completes the
row-parallel product -- with the same process-per-rank structure the RCCL
run uses on the GPU node (torchrun, one rank per device).
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, out_dir: str):
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ch09 import RowParallelLinear, TensorParallelConfig, TensorParallelMLP
        from ch09 import row_parallel_forward_overlapped
        from oracle.numerics import seeded_normal
        K, N, M = 64, 24, 10
        x = torch.from_numpy(seeded_normal((M, K), 1))
        w = torch.from_numpy(seeded_normal((N, K), 2))
        part = K // world
        sl = slice(rank * part, (rank + 1) * part)
        layer = RowParallelLinear(K, N, world_size=world, rank=rank)
        with torch.no_grad():
            layer.weight.copy_(w[:, sl])
            y = layer(x[:, sl])
            y2 = row_parallel_forward_overlapped(x[:, sl], layer.weight, chunks=3)
            # fp32 partials through the all-reduce (reduce_dtype), bf16 input
            l32 = RowParallelLinear(K, N, world_size=world, rank=rank, reduce_dtype=torch.float32)
            l32.weight.copy_(w[:, sl])
            y3 = l32.to(torch.bfloat16)(x[:, sl].to(torch.bfloat16)).float()
            # the chunked form with fp32 partials, keyed on the layer's world size
            y4 = row_parallel_forward_overlapped(x[:, sl].to(torch.bfloat16), l32.weight, chunks=3,
                                                 world_size=world, reduce_dtype=torch.float32).float()
        # TP MLP: every rank must end with the same full output
        torch.manual_seed(100 + rank)
        mlp = TensorParallelMLP(TensorParallelConfig(world_size=world, rank=rank, hidden_dim=16,
                                                     intermediate_dim=32))
        with torch.no_grad():
            ym = mlp(torch.ones(3, 16))
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), y=y.numpy(), y2=y2.numpy(), ym=ym.numpy(),
                 y3=y3.numpy(), y4=y4.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_row_parallel_allreduce_gloo_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from oracle.linear import linear
    from oracle.numerics import seeded_normal
    x, w = seeded_normal((10, 64), 1), seeded_normal((24, 64), 2)
    full = linear(x, w)
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    for ri in r:
        np.testing.assert_allclose(ri["y"], full, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ri["y2"], full, rtol=1e-5, atol=1e-5)
        # the chunked, overlapped all-reduce is the same sum as the plain one:
        # each row's partial is the same product, all-reduced once
        np.testing.assert_array_equal(ri["y2"], ri["y"])
    np.testing.assert_array_equal(r[0]["ym"], r[1]["ym"])
    # bf16 inputs, fp32 partials summed by the all-reduce, one rounding at the end
    from oracle.numerics import round_to_bf16
    full16 = linear(round_to_bf16(x), round_to_bf16(w))
    for ri in r:
        assert np.abs(ri["y3"] - full16).max() <= 2.0 ** -8 * (np.abs(full16).max() + 1)
        assert np.abs(ri["y4"] - full16).max() <= 2.0 ** -8 * (np.abs(full16).max() + 1)
        np.testing.assert_allclose(ri["y4"], ri["y3"], rtol=2.0 ** -7, atol=1e-6)
