"""Tiled matmul -- the ch05 GEMM demos re-built as the HIP kernel ``pli_gemm``.

Replaces ``ch05/tiled_matmul.cu:22-61`` (16x16 shared-memory fp32 tiles, a
standalone CUDA ``main``) and the dropped ``ch05/triton_matmul.py``
(``triton_matmul(a, b, block_m, block_n, block_k)``, ``:67-96``): one
signature, one C ABI entry point, two kernels behind it --

* bf16/fp16: ``pli_gemm``'s routes (csrc/gemm.hip) -- large shapes (at least
  128 tiles of 256 x 256, K % 64 == 0) run ``gemm_w5``: a 256 x 256 tile, one
  wave per SIMD owning 128 x 128 of C^T in the accumulator file, K staged 64
  deep by LDS-DMA, ``v_mfma_f32_16x16x32`` (persistent walk for K >= 128);
  smaller shapes the 128 x 128 / 256 x 256 LDS tiles; fp32 accumulate,
  output in the input dtype (the Triton kernel stored fp16, ``:61``);
* fp32: 128x128x32 LDS-staged tile on ``v_mfma_f32_32x32x2_f32`` (exact
  fp32 fma chain); unaligned / K % 4 != 0 shapes take a 64x64 LDS-tiled VALU
  kernel.

``naive_matmul`` is the demo's contrast kernel (``:9-20``, one thread per
output, ``pli_gemm_naive``) and ``benchmark_matmul_demo`` re-runs the demo's
``main`` (``:96-136``: 2048^3 fp32, uniform [0, 0.99] inputs, naive vs
tiled, ms and TFLOP/s).

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


def naive_matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """fp32 C = A @ B, one thread per output element (ch05/tiled_matmul.cu:9-20)."""
    assert a.shape[1] == b.shape[0], f"Dimension mismatch: {a.shape[1]} vs {b.shape[0]}"
    if not a.is_cuda:
        return torch.matmul(a, b)
    return pli_hip.gemm_naive(a, b)


def benchmark_matmul_demo(size: int = 2048, warmup: int = 3, iterations: int = 10,
                          device: str = "cuda") -> dict | None:
    """The ch05/tiled_matmul.cu ``main`` (:96-136): naive vs tiled fp32 GEMM
    at ``size``^3, inputs ``(rand() % 100) / 100`` (here a seeded torch
    draw of the same 100 levels); returns {name: {"ms", "tflops"}} plus the
    max |tiled - naive| difference."""
    if not torch.cuda.is_available():
        return None
    g = torch.Generator(device="cpu").manual_seed(0)
    a = (torch.randint(0, 100, (size, size), generator=g).float() / 100).to(device)
    b = (torch.randint(0, 100, (size, size), generator=g).float() / 100).to(device)
    flops = 2.0 * size ** 3
    res = {}
    outs = {}
    for name, fn in (("naive", naive_matmul), ("tiled", tiled_matmul)):
        for _ in range(warmup):
            outs[name] = fn(a, b)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iterations):
            fn(a, b)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / iterations
        res[name] = {"ms": ms, "tflops": flops / ms / 1e9}
    res["max_abs_diff"] = float((outs["tiled"] - outs["naive"]).abs().max())
    return res


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
        d = benchmark_matmul_demo()
        for name in ("naive", "tiled"):
            print(f"{name}: {d[name]['ms']:.3f} ms, {d[name]['tflops']:.2f} TFLOPS (2048^3 fp32)")
        for size in [512, 1024, 2048, 4096]:
            r = benchmark_tiled_matmul(size, size, size)
            print(f"{size}^3 bf16: HIP {r.hip_us:.1f} us ({2 * size**3 / r.hip_us / 1e6:.1f} TFLOP/s), "
                  f"torch {r.torch_us:.1f} us, speedup {r.speedup:.2f}x")
