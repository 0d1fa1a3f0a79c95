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


def explain_tensor_cores() -> str:
    """The reference's matrix-unit primer (ch05/tensor_cores.py), for CDNA4."""
    return (
        "\nMatrix cores on MI355X (CDNA4 MFMA)\n\n"
        "One v_mfma instruction is a whole-wave (64 lanes) D = A B + C on a tile:\n"
        "  v_mfma_f32_16x16x32_bf16 / _f16   16 x 16 outputs over k = 32 (16 cycles)\n"
        "  v_mfma_f32_32x32x16_bf16 / _f16   32 x 32 outputs over k = 16 (32 cycles)\n"
        "  v_mfma_f32_32x32x2_f32            exact fp32 (1/16 of the bf16 rate)\n"
        "Dense bf16 / fp16 peak 2.5 PFLOP/s over 256 CUs; fp32 on the matrix cores\n"
        "157 TFLOP/s.  A, B come from VGPRs / AGPRs (fragments staged through LDS),\n"
        "C / D live in the 256 accumulator registers of the wave.\n\n"
        "Using them well: tiles sized for 64-wide waves (this build's GEMM: 256 x 256\n"
        "per workgroup, 128 x 128 per wave, K staged 64 deep by LDS-DMA), enough\n"
        "independent accumulators to cover the MFMA latency, and the operand reads\n"
        "and next-tile loads issued in the gaps between MFMAs.\n"
    )


def verify_tensor_core_usage(size: int = 4096) -> dict | None:
    """The reference's check (ch05/tensor_cores.py:112-130): a 16-bit GEMM more
    than 1.5x faster than the fp32 one means the matrix cores carry it."""
    r = benchmark_tensor_cores(size=size, warmup=5, iterations=20)
    if r is None:
        return None
    mfma = r.speedup > 1.5
    return {"size": size, "fp16_tflops": r.fp16_tflops, "fp32_tflops": r.fp32_tflops, "speedup": r.speedup,
            "likely_tensor_cores": mfma,
            "note": ("speedup > 1.5x: the 16-bit GEMM runs on the 16-bit MFMA" if mfma else
                     "speedup < 1.5x: both on the same units")}


if __name__ == "__main__":
    # the chapter's demo (ch05/tensor_cores.py:133-158)
    print(explain_tensor_cores())
    print("\nTensor Core Specs:")
    for key, val in tensor_core_info().items():
        print(f"  {key}: {val}")
    if torch.cuda.is_available():
        print("\n" + "=" * 60 + "\nBenchmark Results:\n" + "-" * 60)
        for n in (1024, 2048, 4096):
            r = benchmark_tensor_cores(size=n)
            print(f"Size {n}x{n}:\n  FP16: {r.fp16_us:.1f} us ({r.fp16_tflops:.1f} TFLOPS)\n"
                  f"  FP32: {r.fp32_us:.1f} us ({r.fp32_tflops:.1f} TFLOPS)\n  Speedup: {r.speedup:.2f}x")
        print("\nTensor Core Verification:")
        for key, val in verify_tensor_core_usage().items():
            print(f"  {key}: {val}")
    else:
        print("\nno ROCm device")
