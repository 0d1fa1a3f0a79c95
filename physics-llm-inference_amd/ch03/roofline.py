"""Roofline model -- replaces ``ch03/roofline.py`` with an MI355X-first version.

Keeps every symbol of the reference (``HardwareSpec``, the four NVIDIA specs,
``arithmetic_intensity``, ``roofline_throughput``, ``is_compute_bound``,
``ridge_point``, the GEMM/GEMV/batched-GEMV intensities, ``plot_roofline``)
with identical semantics, and adds:

* ``MI355X`` -- datasheet peaks of the target: bf16/fp16 dense MFMA
  2516.6 TFLOP/s (256 CU x 4096 FLOP/clk x 2.4 GHz) and 8000 GB/s HBM3E;
* ``MI355X_FP32_MFMA`` / ``MI355X_FP8`` -- the other dense MFMA peaks;
* ``measure_hbm_bandwidth`` / ``measured_spec`` -- the *achievable* HBM rate
  measured on the device with the HIP stream kernel of ch05/coalescing.cu,
  reported next to the datasheet roofline;
* ``roofline_fraction`` -- achieved / attainable at a given intensity.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class HardwareSpec:
    peak_tflops: float
    memory_bandwidth_gbps: float
    name: str


RTX_3090 = HardwareSpec(peak_tflops=35.6, memory_bandwidth_gbps=936.0, name="RTX 3090")
RTX_4090 = HardwareSpec(peak_tflops=82.6, memory_bandwidth_gbps=1008.0, name="RTX 4090")
A100_80GB = HardwareSpec(peak_tflops=312.0, memory_bandwidth_gbps=2039.0, name="A100 80GB")
H100_SXM = HardwareSpec(peak_tflops=989.0, memory_bandwidth_gbps=3350.0, name="H100 SXM")

# MI355X (gfx950, CDNA4): 256 CUs, 2.4 GHz, 8 TB/s HBM3E (datasheet, dense).
MI355X_CUS = 256
MI355X_CLOCK_GHZ = 2.4
MI355X_BF16_FLOP_PER_CLK_PER_CU = 4096       # v_mfma_f32_32x32x16_bf16: 32768 FLOP / 32 clk / SIMD x 4
MI355X = HardwareSpec(
    peak_tflops=MI355X_CUS * MI355X_BF16_FLOP_PER_CLK_PER_CU * MI355X_CLOCK_GHZ / 1000.0,
    memory_bandwidth_gbps=8000.0,
    name="MI355X",
)
MI355X_FP32_MFMA = HardwareSpec(peak_tflops=157.3, memory_bandwidth_gbps=8000.0,
                                name="MI355X fp32 (MFMA = VALU rate)")
MI355X_FP8 = HardwareSpec(peak_tflops=2 * MI355X.peak_tflops, memory_bandwidth_gbps=8000.0,
                          name="MI355X fp8 (MX-scaled MFMA)")
# xGMI: 7 point-to-point links per GPU, ~153 GB/s each (one direction).
MI355X_XGMI_LINK_GBPS = 153.0
MI355X_XGMI_LINKS = 7


def arithmetic_intensity(flops: int, bytes_moved: int) -> float:
    return flops / bytes_moved


def roofline_throughput(ai: float, hw: HardwareSpec) -> float:
    """Attainable TFLOP/s at intensity ``ai`` (FLOP/B): min(ai*BW, peak)."""
    return min(ai * hw.memory_bandwidth_gbps / 1000, hw.peak_tflops)


def ridge_point(hw: HardwareSpec) -> float:
    """FLOP/B where the bandwidth roof meets the compute roof."""
    return hw.peak_tflops * 1000 / hw.memory_bandwidth_gbps


def is_compute_bound(ai: float, hw: HardwareSpec) -> bool:
    return ai >= ridge_point(hw)


def gemm_arithmetic_intensity(m: int, n: int, k: int) -> float:
    return (2 * m * n * k) / ((m * k + k * n + m * n) * 2)


def gemv_arithmetic_intensity(m: int, k: int) -> float:
    return (2 * m * k) / ((m * k + k + m) * 2)


def batched_gemv_arithmetic_intensity(batch: int, m: int, k: int) -> float:
    return (2 * batch * m * k) / ((m * k + batch * k + batch * m) * 2)


def roofline_fraction(achieved_tflops: float, ai: float, hw: HardwareSpec = MI355X) -> float:
    """Fraction of the attainable roof reached at intensity ``ai``."""
    return achieved_tflops / roofline_throughput(ai, hw)


def measure_hbm_bandwidth(nbytes: int = 1 << 30, iters: int = 20, device: str = "cuda") -> float:
    """Achievable HBM GB/s: the 16-byte-vector stream kernel (read + write,
    ``pli_scale_copy``), buffers 2 x ``nbytes`` >> the 256 MiB Infinity
    Cache, timed with HIP events over back-to-back launches."""
    import torch

    import pli_hip

    n = nbytes // 4
    src = torch.randn(n, device=device)
    dst = torch.empty_like(src)
    for _ in range(3):
        pli_hip.scale_copy(src, dst)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        pli_hip.scale_copy(src, dst)
    e.record()
    e.synchronize()
    sec = s.elapsed_time(e) / 1e3 / iters
    return 2 * n * 4 / sec / 1e9


def measure_hbm_read_bandwidth(nbytes: int = 1 << 30, iters: int = 10, device: str = "cuda") -> float:
    """Achievable HBM READ GB/s: ``pli_hbm_read_probe`` (16-byte non-temporal
    loads) over two alternating ``nbytes`` buffers (2 GiB >> the 256 MiB
    Infinity Cache), best of ``iters`` event-timed launches of each probe
    layout (grid-stride at 8 workgroups per CU; one contiguous slice per
    workgroup at 2, 4 and 8 per CU) -- the ceiling of the read-dominated GEMV
    and decode-attention kernels."""
    import torch

    import pli_hip

    bufs = [torch.empty(nbytes // 4, device=device, dtype=torch.int32).fill_(i + 1) for i in range(2)]
    best = float("inf")
    for mode, per_cu in ((0, 8), (1, 2), (1, 4), (1, 8)):
        blocks = MI355X_CUS * per_cu
        out = torch.empty(blocks * 256, device=device, dtype=torch.int32)
        for b in bufs:
            pli_hip.hbm_read_probe(b, out, blocks, mode)
        for i in range(iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            pli_hip.hbm_read_probe(bufs[i & 1], out, blocks, mode)
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) / 1e3)
    return nbytes / best / 1e9


def measure_mfma_peak(shape: str = "32x32x16", iters: int = 4096, reps: int = 5,
                      device: str = "cuda") -> float:
    """Achievable bf16 MFMA TFLOP/s: ``pli_mfma_probe`` (four independent
    MFMAs per wave from registers, pseudo-random operands, 4 waves per SIMD on
    every CU), best of ``reps`` event-timed launches.  The clock the chip
    holds under that load sets it (MI355X_MICROARCH.md 'DVFS give-back')."""
    import torch

    import pli_hip

    blocks = MI355X_CUS * 4
    out = torch.empty(blocks * 256, device=device, dtype=torch.float32)
    sh = {"32x32x16": 0, "16x16x32": 1}[shape]
    pli_hip.mfma_probe(out, blocks, iters, sh)
    best = float("inf")
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        pli_hip.mfma_probe(out, blocks, iters, sh)
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 1e3)
    return blocks * 4 * iters * 4 * (32768 if sh == 0 else 16384) / best / 1e12


def measured_spec(hbm_gbps: float, mfma_tflops: float | None = None) -> HardwareSpec:
    """An MI355X roof with measured ceilings (datasheet compute peak if None)."""
    return HardwareSpec(peak_tflops=mfma_tflops or MI355X.peak_tflops,
                        memory_bandwidth_gbps=hbm_gbps, name="MI355X (measured)")


def plot_roofline(hw: HardwareSpec, points: list | None = None, save_path: str | None = None):
    """Log-log roofline with optional (name, ai, tflops) points (matplotlib)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import numpy as np

    ai = np.logspace(-2, 4, 1000)
    roof = np.minimum(ai * hw.memory_bandwidth_gbps / 1000, hw.peak_tflops)
    fig, ax = plt.subplots(figsize=(10, 6))
    ax.loglog(ai, roof, "b-", linewidth=2, label="Roofline")
    ridge = ridge_point(hw)
    ax.axvline(x=ridge, color="gray", linestyle="--", alpha=0.5)
    ax.annotate(f"Ridge Point\nAI = {ridge:.1f}", xy=(ridge, hw.peak_tflops * 0.8), fontsize=10)
    for name, p_ai, tflops in points or []:
        ax.scatter([p_ai], [tflops], s=100, c="green" if is_compute_bound(p_ai, hw) else "red",
                   zorder=5)
        ax.annotate(name, xy=(p_ai, tflops), xytext=(5, 5), textcoords="offset points")
    ax.fill_between(ai[ai < ridge], roof[ai < ridge], 0.01, alpha=0.2, color="red",
                    label="Memory Bound")
    ax.fill_between(ai[ai >= ridge], roof[ai >= ridge], 0.01, alpha=0.2, color="green",
                    label="Compute Bound")
    ax.set_xlabel("Arithmetic Intensity (FLOP/Byte)")
    ax.set_ylabel("Throughput (TFLOPS)")
    ax.set_title(f"Roofline Model - {hw.name}")
    ax.legend()
    ax.grid(True, alpha=0.3)
    ax.set_xlim([0.01, 10000])
    ax.set_ylim([0.01, hw.peak_tflops * 1.5])
    if save_path:
        plt.savefig(save_path, dpi=150, bbox_inches="tight")
    return fig, ax


if __name__ == "__main__":
    hw = MI355X
    print(f"{hw.name}: {hw.peak_tflops:.1f} TFLOP/s bf16 dense, {hw.memory_bandwidth_gbps:.0f} GB/s,"
          f" ridge {ridge_point(hw):.1f} FLOP/B")
    for label, ai in (("GEMM 4096^3", gemm_arithmetic_intensity(4096, 4096, 4096)),
                      ("GEMV 4096^2", gemv_arithmetic_intensity(4096, 4096))):
        print(f"{label}: AI {ai:.2f} -> {'compute' if is_compute_bound(ai, hw) else 'memory'} bound,"
              f" roof {roofline_throughput(ai, hw):.1f} TFLOP/s")
