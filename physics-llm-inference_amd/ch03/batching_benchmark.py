"""Batched decode GEMV -- mirror of ``ch03/batching_benchmark.py``.

Y = X W^T over a batch of decode tokens.  On a ROCm device it runs the HIP
kernel ``pli_gemm`` with ``trans_b=1`` (W stays [m, k] row-major, no
transpose copy); ``find_transition_batch_size`` is the reference's doubling
search for the batch whose intensity crosses the ridge point.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

import pli_hip

from .gemv_benchmark import _elem, _sync


@dataclass
class BatchBenchmarkResult:
    batch_size: int
    mean_us: float
    tokens_per_second: float
    tflops: float
    memory_gbps: float


def benchmark_batched_gemv(
    batch_size: int,
    m: int,
    k: int,
    dtype: torch.dtype = torch.float16,
    warmup: int = 10,
    iterations: int = 100,
    device: str = "cuda",
) -> BatchBenchmarkResult:
    weight = torch.randn(m, k, dtype=dtype, device=device)
    x = torch.randn(batch_size, k, dtype=dtype, device=device)
    on_gpu = weight.is_cuda
    y = torch.empty(batch_size, m, dtype=dtype, device=device)

    def call():
        if on_gpu:
            pli_hip.gemm(x, weight, trans_b=True, out=y)
        else:
            x @ weight.T

    for _ in range(warmup):
        call()
    _sync(device)
    times = []
    for _ in range(iterations):
        _sync(device)
        t0 = time.perf_counter()
        call()
        _sync(device)
        times.append((time.perf_counter() - t0) * 1e6)
    mean_us = sum(times) / len(times)
    nbytes = (m * k + batch_size * k + batch_size * m) * _elem(dtype)
    return BatchBenchmarkResult(
        batch_size=batch_size, mean_us=mean_us,
        tokens_per_second=batch_size / (mean_us * 1e-6),
        tflops=2 * batch_size * m * k / (mean_us * 1e-6) / 1e12,
        memory_gbps=nbytes / (mean_us * 1e-6) / 1e9)


def find_transition_batch_size(m: int, k: int, peak_tflops: float,
                               memory_bandwidth_gbps: float) -> int:
    """Smallest power-of-two batch whose intensity reaches the ridge point
    (2-byte elements); returns 2048 if none up to 1024 does."""
    ridge = peak_tflops * 1000 / memory_bandwidth_gbps
    batch = 1
    while True:
        ai = (2 * batch * m * k) / ((m * k + batch * k + batch * m) * 2)
        if ai >= ridge:
            return batch
        batch *= 2
        if batch > 1024:
            return batch


def benchmark_batch_sweep(m: int, k: int, batch_sizes: list[int],
                          dtype: torch.dtype = torch.float16) -> list[BatchBenchmarkResult]:
    return [benchmark_batched_gemv(b, m, k, dtype=dtype) for b in batch_sizes]


if __name__ == "__main__":
    if not torch.cuda.is_available():
        print("ROCm device not available, skipping benchmark")
    else:
        from .roofline import MI355X
        print(f"{'Batch':>6} {'Time (us)':>12} {'Tokens/s':>12} {'TFLOPS':>10} {'GB/s':>10}")
        for b in [1, 2, 4, 8, 16, 32, 64, 128, 256, 512]:
            r = benchmark_batched_gemv(b, 4096, 4096, dtype=torch.bfloat16)
            print(f"{r.batch_size:>6} {r.mean_us:>12.1f} {r.tokens_per_second:>12.0f} "
                  f"{r.tflops:>10.2f} {r.memory_gbps:>10.1f}")
        print("transition batch (MI355X):",
              find_transition_batch_size(4096, 4096, MI355X.peak_tflops, MI355X.memory_bandwidth_gbps))
