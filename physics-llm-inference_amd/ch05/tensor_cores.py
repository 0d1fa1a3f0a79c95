"""Matrix-core probe -- mirror of ``ch05/tensor_cores.py`` for CDNA4 MFMA.

``benchmark_tensor_cores`` times the HIP GEMM at fp16 (MFMA
``v_mfma_f32_32x32x16_f16`` kernel) against fp32 (VALU kernel) on the same
matrices; the reference's heuristic (speedup > 1.5 => matrix cores in use,
``:112-130``) carries over.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

import pli_hip


@dataclass
class TensorCoreResult:
    size: int
    fp16_us: float
    fp32_us: float
    speedup: float
    fp16_tflops: float
    fp32_tflops: float


def tensor_core_info() -> dict:
    return {
        "operation": "D = A * B + C (per-wave MFMA, wave64)",
        "input_types": ["fp16", "bf16", "fp32", "int8", "fp8 (OCP e4m3/e5m2)", "fp6", "fp4"],
        "accumulator_types": ["fp32", "int32"],
        "ampere_shape": "8x8x4 or 16x8x16 (NVIDIA reference)",
        "cdna4_shape": "32x32x16 / 16x16x32 bf16/fp16; 32x32x2 / 16x16x4 fp32",
        "minimum_size": "tiles of 16 or 32 rows/cols",
    }


def benchmark_tensor_cores(size: int = 4096, warmup: int = 10, iterations: int = 100,
                           device: str = "cuda") -> TensorCoreResult | None:
    if not torch.cuda.is_available():
        return None
    a16 = torch.randn(size, size, device=device, dtype=torch.float16)
    b16 = torch.randn(size, size, device=device, dtype=torch.float16)
    a32, b32 = a16.float(), b16.float()

    def timed(a, b):
        for _ in range(warmup):
            pli_hip.gemm(a, b)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iterations):
            pli_hip.gemm(a, b)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / 1e3 / iterations

    t16, t32 = timed(a16, b16), timed(a32, b32)
    flops = 2 * size ** 3
    return TensorCoreResult(size, t16 * 1e6, t32 * 1e6, t32 / t16, flops / t16 / 1e12,
                            flops / t32 / 1e12)
