"""Prefill GEMM benchmark -- mirror of ``ch03/gemm_benchmark.py``.

Same signature, same wall-clock ``BenchmarkResult`` semantics as the
reference (``:26-70``); on a ROCm device the product is the HIP MFMA kernel
``pli_gemm`` (NN layout, C = A B, torch.mm semantics) instead of
``torch.mm``.  ``kernel_us``/``kernel_gbps`` add the event-timed kernel.
"""
from __future__ import annotations

import time

import torch

import pli_hip

from .gemv_benchmark import BenchmarkResult, _elem, _event_time_us, _sync, summarize


def gemm_flops(m: int, n: int, k: int) -> int:
    return 2 * m * n * k


def gemm_bytes(m: int, n: int, k: int, dtype: torch.dtype = torch.float16) -> int:
    """Compulsory bytes: A (m*k) + B (k*n) + C (m*n)."""
    return (m * k + k * n + m * n) * _elem(dtype)


def benchmark_gemm(
    m: int,
    n: int,
    k: int,
    dtype: torch.dtype = torch.float16,
    warmup: int = 10,
    iterations: int = 100,
    device: str = "cuda",
) -> BenchmarkResult:
    a = torch.randn(m, k, dtype=dtype, device=device)
    b = torch.randn(k, n, dtype=dtype, device=device)
    on_gpu = a.is_cuda
    c = torch.empty(m, n, dtype=dtype, device=device)

    def call():
        if on_gpu:
            pli_hip.gemm(a, b, trans_b=False, out=c)
        else:
            torch.mm(a, b)

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
    kernel_us = _event_time_us(call, iterations) if on_gpu else None
    return summarize(times, gemm_flops(m, n, k), gemm_bytes(m, n, k, dtype), kernel_us)


def benchmark_prefill_gemm(batch_size: int, seq_len: int, hidden_dim: int,
                           dtype: torch.dtype = torch.float16) -> BenchmarkResult:
    return benchmark_gemm(batch_size * seq_len, hidden_dim, hidden_dim, dtype=dtype)


if __name__ == "__main__":
    if not torch.cuda.is_available():
        print("ROCm device not available, skipping benchmark")
    else:
        print("GEMM Benchmark (prefill-like workloads, HIP pli_gemm)")
        for batch, seq, hidden in [(32, 512, 4096), (32, 1024, 4096), (32, 2048, 4096), (1, 4096, 4096)]:
            r = benchmark_gemm(batch * seq, hidden, hidden, dtype=torch.bfloat16, iterations=20)
            print(f"M={batch * seq:6d}, N={hidden}, K={hidden}: wall {r.mean_us:8.1f} us "
                  f"({r.tflops:.1f} TFLOPS), kernel {r.kernel_us:8.1f} us "
                  f"({gemm_flops(batch * seq, hidden, hidden) / r.kernel_us / 1e6:.1f} TFLOPS)")
