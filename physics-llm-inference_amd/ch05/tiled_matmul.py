"""Tiled matmul -- the ch05 GEMM demos re-built as the HIP kernel ``pli_gemm``.

Replaces ``ch05/tiled_matmul.cu:22-61`` (16x16 shared-memory fp32 tiles, a
standalone CUDA ``main``) and the dropped ``ch05/triton_matmul.py``
(``triton_matmul(a, b, block_m, block_n, block_k)``, ``:67-96``): one
signature, one C ABI entry point, two kernels behind it --

* bf16/fp16: 128x128x64 LDS-staged tile on ``v_mfma_f32_32x32x16`` (fp32
  accumulate, output in the input dtype; the Triton kernel stored fp16,
  ``:61``);
* fp32 (and ragged shapes): 64x64 LDS-tiled VALU kernel, fp32 accumulate.

``block_m/block_n/block_k`` are accepted for signature compatibility; the
HIP tile is fixed by the MFMA / LDS mapping.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

import pli_hip


def tiled_matmul(a: torch.Tensor, b: torch.Tensor, block_m: int = 64, block_n: int = 64,
                 block_k: int = 32) -> torch.Tensor:
    """C = A @ B (A [M,K], B [K,N]) on the HIP GEMM; CPU tensors use torch."""
    M, K = a.shape
    K2, N = b.shape
    assert K == K2, f"Dimension mismatch: {K} vs {K2}"
    if not a.is_cuda:
        return torch.matmul(a, b)
    return pli_hip.gemm(a, b, trans_b=False)


# the reference's public name for the same operation (ch05/triton_matmul.py:67)
triton_matmul = tiled_matmul


@dataclass
class MatmulBenchmark:
    m: int
    n: int
    k: int
    hip_us: float
    torch_us: float
    speedup: float


def benchmark_tiled_matmul(m: int = 1024, n: int = 1024, k: int = 1024, warmup: int = 10,
                           iterations: int = 100, device: str = "cuda",
                           dtype: torch.dtype = torch.bfloat16) -> MatmulBenchmark | None:
    """HIP GEMM vs torch.matmul (hipBLASLt on ROCm), event-timed."""
    if not torch.cuda.is_available():
        return None
    a = torch.randn(m, k, device=device, dtype=dtype)
    b = torch.randn(k, n, device=device, dtype=dtype)

    def timed(fn):
        for _ in range(warmup):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iterations):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / iterations

    t_torch = timed(lambda: torch.matmul(a, b))
    t_hip = timed(lambda: tiled_matmul(a, b))
    return MatmulBenchmark(m, n, k, t_hip, t_torch, t_torch / t_hip)


if __name__ == "__main__":
    if torch.cuda.is_available():
        for size in [512, 1024, 2048, 4096]:
            r = benchmark_tiled_matmul(size, size, size)
            print(f"{size}^3 bf16: HIP {r.hip_us:.1f} us ({2 * size**3 / r.hip_us / 1e6:.1f} TFLOP/s), "
                  f"torch {r.torch_us:.1f} us, speedup {r.speedup:.2f}x")
