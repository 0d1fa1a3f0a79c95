"""``ch05/triton_matmul.py`` on MI355X: the tiled GEMM without Triton.

The north star drops Triton (no multi-backend dispatch): ``triton_matmul``
keeps the reference's signature (``ch05/triton_matmul.py:67-96``) and runs
the HIP GEMM of ``tiled_matmul`` (``pli_gemm``: the 256x256 MFMA tile for
bf16/fp16, fp32 on ``v_mfma_f32_32x32x2_f32`` / the VALU tile), and
``benchmark_triton_matmul`` keeps its signature and ``MatmulBenchmark``
fields (``:14-21``, ``:99-142``) with ``triton_us`` = the HIP kernel's time.
``TRITON_AVAILABLE`` is False: there is no Triton kernel in this build.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from .tiled_matmul import tiled_matmul

TRITON_AVAILABLE = False


@dataclass
class MatmulBenchmark:
    m: int
    n: int
    k: int
    triton_us: float
    torch_us: float
    speedup: float


def triton_matmul(a: torch.Tensor, b: torch.Tensor, block_m: int = 64, block_n: int = 64,
                  block_k: int = 32) -> torch.Tensor:
    """C = A @ B; ``block_*`` are accepted for the reference's signature (the
    HIP tile is fixed by the MFMA / LDS mapping)."""
    return tiled_matmul(a, b, block_m, block_n, block_k)


def benchmark_triton_matmul(m: int = 1024, n: int = 1024, k: int = 1024, warmup: int = 10,
                            iterations: int = 100, device: str = "cuda") -> MatmulBenchmark | None:
    """fp16 [m,k] x [k,n]: torch.matmul (hipBLASLt) vs the HIP tiled GEMM,
    timed as the reference does (sync, perf_counter over the loop)."""
    if not torch.cuda.is_available():
        return None
    a = torch.randn(m, k, device=device, dtype=torch.float16)
    b = torch.randn(k, n, device=device, dtype=torch.float16)

    def timed(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        start = time.perf_counter()
        for _ in range(iterations):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - start) / iterations * 1e6

    torch_us = timed(lambda: torch.matmul(a, b))
    hip_us = timed(lambda: triton_matmul(a, b))
    return MatmulBenchmark(m=m, n=n, k=k, triton_us=hip_us, torch_us=torch_us, speedup=torch_us / hip_us)


def triton_matmul_explained() -> str:
    """The reference's description of its Triton kernel (ch05/triton_matmul.py),
    and what stands in for it here."""
    return (
        "\nThe chapter's Triton matmul: each program instance computes one\n"
        "BLOCK_M x BLOCK_N output tile, walking K in BLOCK_K steps -- load an A and\n"
        "a B tile, tl.dot them into an fp32 accumulator, store the tile once.\n\n"
        "This build has no Triton (TRITON_AVAILABLE is False): triton_matmul runs the\n"
        "hand-written HIP GEMM -- the same tiling idea written for CDNA4: 256 x 256\n"
        "output tiles, one wave per SIMD with a 128 x 128 accumulator block in its\n"
        "AGPRs, A / B staged 64 k deep into LDS by direct-to-LDS DMA two steps ahead,\n"
        "and v_mfma_f32_16x16x32 on the fragments.  benchmark_triton_matmul reports\n"
        "that kernel as `triton_us` next to torch.matmul (hipBLASLt).\n"
    )


if __name__ == "__main__":
    # the chapter's demo (ch05/triton_matmul.py:145-161)
    print(triton_matmul_explained())
    if not torch.cuda.is_available():
        print("no ROCm device")
    else:
        print("\nBenchmark Results:\n" + "=" * 60 + f"\nTriton available: {TRITON_AVAILABLE}")
        for n in (512, 1024, 2048, 4096):
            r = benchmark_triton_matmul(m=n, n=n, k=n)
            print(f"{n}x{n}: HIP GEMM {r.triton_us:.1f} us, Torch {r.torch_us:.1f} us, Speedup {r.speedup:.2f}x")
