"""Decode GEMV benchmark -- mirror of ``ch03/gemv_benchmark.py``.

``benchmark_gemv`` keeps the reference signature and ``BenchmarkResult``
fields, with the reference's per-call wall-clock method (synchronise,
``perf_counter``, call, synchronise: ``:41-48``) so the numbers mean the same
thing.  On a ROCm device the call is the HIP kernel ``pli_gemv``
(csrc/gemv.hip) instead of ``torch.mv``.  Two extra fields report the kernel
itself, timed with HIP events over back-to-back launches: ``kernel_us`` and
``kernel_gbps`` (the roofline-relevant numbers; the wall-clock ones include
launch + sync latency, tens of microseconds against a ~4 us kernel).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

import pli_hip


@dataclass
class BenchmarkResult:
    mean_us: float
    std_us: float
    min_us: float
    max_us: float
    tflops: float
    memory_gbps: float
    kernel_us: float | None = None
    kernel_gbps: float | None = None


def _elem(dtype: torch.dtype) -> int:
    return torch.tensor([], dtype=dtype).element_size()


def gemv_flops(m: int, k: int) -> int:
    return 2 * m * k


def gemv_bytes(m: int, k: int, dtype: torch.dtype = torch.float16) -> int:
    """Compulsory bytes: W (m*k) + x (k) + y (m)."""
    return (m * k + k + m) * _elem(dtype)


def _sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize()


def _event_time_us(fn, iterations: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iterations):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iterations


def summarize(times_us, flops: int, nbytes: int, kernel_us: float | None = None) -> BenchmarkResult:
    t = torch.tensor(times_us, dtype=torch.float64)
    mean = t.mean().item()
    return BenchmarkResult(
        mean_us=mean, std_us=t.std().item() if len(times_us) > 1 else 0.0,
        min_us=t.min().item(), max_us=t.max().item(),
        tflops=flops / (mean * 1e-6) / 1e12, memory_gbps=nbytes / (mean * 1e-6) / 1e9,
        kernel_us=kernel_us,
        kernel_gbps=None if kernel_us is None else nbytes / (kernel_us * 1e-6) / 1e9)


def benchmark_gemv(
    m: int,
    k: int,
    dtype: torch.dtype = torch.float16,
    warmup: int = 10,
    iterations: int = 100,
    device: str = "cuda",
) -> BenchmarkResult:
    weight = torch.randn(m, k, dtype=dtype, device=device)
    x = torch.randn(k, dtype=dtype, device=device)
    on_gpu = weight.is_cuda
    y = torch.empty(m, dtype=dtype, device=device)

    def call():
        if on_gpu:
            pli_hip.gemv(weight, x, out=y)
        else:
            torch.mv(weight, x)

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
    return summarize(times, gemv_flops(m, k), gemv_bytes(m, k, dtype), kernel_us)


def benchmark_decode_gemv(hidden_dim: int, dtype: torch.dtype = torch.float16) -> BenchmarkResult:
    return benchmark_gemv(hidden_dim, hidden_dim, dtype=dtype)


if __name__ == "__main__":
    if not torch.cuda.is_available():
        print("ROCm device not available, skipping benchmark")
    else:
        print("GEMV Benchmark (decode-like workloads, HIP pli_gemv)")
        for hidden in [2048, 4096, 8192, 16384]:
            r = benchmark_gemv(hidden, hidden, dtype=torch.bfloat16)
            print(f"M={hidden:6d}, K={hidden}: wall {r.mean_us:8.1f} us ({r.memory_gbps:.1f} GB/s), "
                  f"kernel {r.kernel_us:7.2f} us ({r.kernel_gbps:.1f} GB/s)")
