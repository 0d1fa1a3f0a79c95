"""Memory coalescing probes -- mirror of ``ch05/memory_coalescing.py`` with the
bandwidth kernels of ``ch05/coalescing.cu`` re-built in HIP.

``measure_access_pattern`` times the HIP stream kernel (``pli_scale_copy``):
stride 1 is the 16-byte-vector coalesced stream (read + write 2 x 4 B per
element), stride 32 the strided read of ``coalescing.cu:14-20``; efficiency is
against the MI355X HBM3E peak (8000 GB/s) instead of the RTX 3090's 936
(``:66`` of the reference).  ``coalesced_access``/``strided_access`` keep
their torch semantics (clone / gather) for API compatibility.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

import pli_hip

MI355X_HBM_GBPS = 8000.0


@dataclass
class AccessPatternResult:
    pattern_name: str
    time_us: float
    bandwidth_gbps: float
    efficiency: float


def coalesced_access(data: torch.Tensor) -> torch.Tensor:
    return data.clone()


def strided_access(data: torch.Tensor, stride: int = 32) -> torch.Tensor:
    return data[torch.arange(0, data.shape[0], stride, device=data.device)]


def _time_us(fn, warmup: int, iterations: int) -> float:
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iterations):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iterations


def measure_access_pattern(size: int = 1024 * 1024 * 32, warmup: int = 10, iterations: int = 100,
                           device: str = "cuda", stride: int = 32,
                           peak_gbps: float = MI355X_HBM_GBPS):
    """(coalesced, strided) AccessPatternResults from the HIP stream kernels."""
    src = torch.randn(size, device=device)
    dst = torch.empty_like(src)
    t_c = _time_us(lambda: pli_hip.scale_copy(src, dst, 1), warmup, iterations)
    bw_c = 2 * size * 4 / (t_c * 1e-6) / 1e9
    n_s = size // stride
    dst_s = torch.empty(n_s, device=device)
    t_s = _time_us(lambda: pli_hip.scale_copy(src, dst_s, stride), warmup, iterations)
    bw_s = 2 * n_s * 4 / (t_s * 1e-6) / 1e9
    return (AccessPatternResult("coalesced", t_c, bw_c, min(bw_c / peak_gbps, 1.0)),
            AccessPatternResult("strided", t_s, bw_s, min(bw_s / peak_gbps, 1.0)))


def explain_coalescing() -> str:
    """The reference's coalescing primer (ch05/memory_coalescing.py:85-111),
    for a 64-lane CDNA4 wave."""
    return (
        "\nMemory coalescing on MI355X\n\n"
        "A wave is 64 lanes; one vector load instruction hands the texture\n"
        "address unit 64 addresses, and the hardware fetches whole cache lines\n"
        "(128 B) for them.\n\n"
        "Coalesced (good): lane i reads bytes 16 i .. 16 i + 15 (global_load_dwordx4)\n"
        "  -> one instruction moves 1 KiB from 8 lines, every byte used\n\n"
        "Strided (bad): lane i reads 4 bytes at 128 i\n"
        "  -> 64 separate lines for 256 useful bytes: 1/32 of each fetch used,\n"
        "     and the address unit spends a cycle per line\n\n"
        "Rule: give consecutive lanes consecutive 16-byte chunks (this build's\n"
        "GEMV and decode kernels read W / the KV cache that way, and its GEMM and\n"
        "flash kernels stream whole 128-B rows into LDS by LDS-DMA).  The penalty\n"
        "of the strided pattern here is measured by measure_access_pattern.\n"
    )


if __name__ == "__main__":
    print(explain_coalescing())
    if torch.cuda.is_available():
        c, s = measure_access_pattern(size=1 << 28)
        print(f"Coalesced: {c.time_us:.1f} us, {c.bandwidth_gbps:.1f} GB/s ({c.efficiency:.1%})")
        print(f"Strided:   {s.time_us:.1f} us, {s.bandwidth_gbps:.1f} GB/s ({s.efficiency:.1%})")
