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


def measure_hbm_read_bandwidth_sized(nbytes: int = 33570816, copies: int = 24, reps: int = 8,
                                     device: str = "cuda") -> dict:
    """The size-matched HBM read roof of the ch03 GEMV: ``pli_hbm_read_probe``
    reading ``nbytes`` per launch (default ``gemv_bytes(4096, 4096)``, the
    GEMV's whole footprint) from ``copies`` distinct buffers in turn (24 x 32
    MiB = 768 MiB, three times the 256 MiB Infinity Cache, so every launch
    streams from HBM), the ``copies`` launches captured in ONE HIP graph and
    replayed -- exactly how bench.py times the GEMV, so the per-launch time
    includes the same kernel boundary.  Best per-launch time over the probe
    layouts (grid-stride at 8 workgroups per CU; one contiguous slice per
    workgroup at 2, 4, 8 and 16 per CU).  Returns GB/s, us per launch and
    the layout."""
    import torch

    import pli_hip

    n = (nbytes + 15) // 16 * 4
    bufs = [torch.empty(n, device=device, dtype=torch.int32).fill_(i + 1) for i in range(copies)]
    stream = torch.cuda.current_stream()
    best = None
    for mode, per_cu in ((0, 8), (1, 2), (1, 4), (1, 8), (1, 16)):
        blocks = MI355X_CUS * per_cu
        out = torch.empty(blocks * 256, device=device, dtype=torch.int32)
        for b in bufs:
            pli_hip.hbm_read_probe(b, out, blocks, mode)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for b in bufs:
                pli_hip.hbm_read_probe(b, out, blocks, mode)
        for _ in range(3):
            g.replay()
        times = []
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            g.replay()
            e.record(stream)
            e.synchronize()
            times.append(s.elapsed_time(e) / 1e3 / copies)
        t = sorted(times)[len(times) // 2]
        if best is None or t < best[0]:
            best = (t, mode, per_cu)
        del g
    t, mode, per_cu = best
    return {"GB/s": nbytes / t / 1e9, "us_per_launch": t * 1e6, "bytes_per_launch": nbytes,
            "layout": f"mode {mode} ({'grid-stride' if mode == 0 else 'slice per workgroup'}), {per_cu} WG/CU",
            "how": f"{copies} buffers in turn, one HIP graph of {copies} launches, median of {reps} replays"}


def _graph_probe_us(bufs, blocks: int, mode: int, reps: int) -> float:
    """median us per launch of pli_hbm_read_probe over ``bufs`` in turn, the
    launches captured in one HIP graph (the GEMV leg's timing)"""
    import torch

    import pli_hip

    stream = torch.cuda.current_stream()
    out = torch.empty(blocks * 256, device=bufs[0].device, dtype=torch.int32)
    for b in bufs:
        pli_hip.hbm_read_probe(b, out, blocks, mode)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for b in bufs:
            pli_hip.hbm_read_probe(b, out, blocks, mode)
    for _ in range(3):
        g.replay()
    times = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        g.replay()
        e.record(stream)
        e.synchronize()
        times.append(s.elapsed_time(e) * 1e3 / len(bufs))
    del g
    return sorted(times)[len(times) // 2]


def measure_gemv_floor(gemv_nbytes: int = 33570816, sizes_mib=(8, 32, 128, 512), grid_waves: int = 4096,
                       reps: int = 8, device: str = "cuda") -> dict:
    """The GEMV's measured floor: in graphs timed like the
    ch03 GEMV leg,

    * an (almost) empty launch with the GEMV's wave count (the read probe
      over 16 bytes, ``grid_waves`` waves in 256-thread blocks): the
      per-launch boundary ``empty_us``;
    * the read probe at ``sizes_mib`` per launch (best layout each, buffers
      rotated past the 256 MiB Infinity Cache), fitted as
      ``us = a + bytes / slope``.

    floor_us = a + gemv_nbytes / slope: what a launch that only streams the
    GEMV's bytes costs on this part, boundary included."""
    import numpy as np
    import torch

    tiny = [torch.ones(4, device=device, dtype=torch.int32) for _ in range(24)]
    empty_us = _graph_probe_us(tiny, max(1, grid_waves // 4), 1, reps)
    pts = []
    for mib in sizes_mib:
        nbytes = mib << 20
        copies = max(2, -(-(768 << 20) // nbytes))
        bufs = [torch.empty(nbytes // 4, device=device, dtype=torch.int32).fill_(i + 1) for i in range(copies)]
        best = min(_graph_probe_us(bufs, MI355X_CUS * per_cu, mode, reps)
                   for mode, per_cu in ((0, 8), (1, 4), (1, 8), (1, 16)))
        pts.append((nbytes, best))
        del bufs
    x = np.array([p[0] for p in pts], dtype=np.float64)
    y = np.array([p[1] for p in pts], dtype=np.float64)
    slope_us_per_byte, a = np.polyfit(x, y, 1)
    floor_us = a + gemv_nbytes * slope_us_per_byte
    return {"empty_launch_us": empty_us, "fit_intercept_us": float(a),
            "fit_GB/s": float(1e-3 / slope_us_per_byte),
            "points": [{"bytes": int(b), "us": float(t), "GB/s": b / t * 1e-3} for b, t in pts],
            "floor_us": float(floor_us), "floor_GB/s": gemv_nbytes / floor_us * 1e-3,
            "how": "pli_hbm_read_probe in one HIP graph per size (buffers rotated past 256 MiB), best "
                   "layout per size; least-squares us = a + bytes/slope; floor = a + GEMV bytes/slope; "
                   f"empty launch = the probe over 16 B with {grid_waves} waves"}


def measure_mfma_peak_detail(shape: str = "32x32x16", iters: int = 2048, reps: int = 5,
                             ramp_s: float = 2.0, device: str = "cuda") -> dict:
    """Achievable bf16 MFMA rate of one shape: ``pli_mfma_probe`` (one wave
    per SIMD on every CU, back-to-back MFMAs from registers into independent
    accumulators, pseudo-random operands, the same 64x64 output tile per wave
    for both shapes).  ``ramp_s`` seconds of back-to-back launches first, then
    the best of ``reps`` event-timed launches; the in-kernel clock is the
    median over waves of s_memtime / s_memrealtime ticks x 100 MHz, stamped
    in the last launch (MI355X_MICROARCH.md 'DVFS give-back' item 6)."""
    import time

    import torch

    import pli_hip

    blocks = MI355X_CUS
    out = torch.empty(blocks * 256, device=device, dtype=torch.float32)
    clocks = torch.zeros(blocks * 8, device=device, dtype=torch.int64)
    sh = {"32x32x16": 0, "16x16x32": 1}[shape]
    pli_hip.mfma_probe(out, blocks, iters, sh)
    torch.cuda.synchronize()
    t_end = time.perf_counter() + ramp_s
    while time.perf_counter() < t_end:
        for _ in range(20):
            pli_hip.mfma_probe(out, blocks, iters, sh)
        torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        pli_hip.mfma_probe(out, blocks, iters, sh, clocks=clocks)
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 1e3)
    ck = clocks.view(-1, 2).double().cpu()
    ghz = (ck[:, 0] / ck[:, 1] * 0.1).median().item()
    flops = blocks * 4 * iters * 262144
    return {"TFLOP/s": flops / best / 1e12, "clock_GHz": ghz,
            "TFLOP/s_at_2.4GHz_equiv": flops / best / 1e12 * 2.4 / ghz if ghz > 0 else None}


def measure_mfma_peak(shape: str = "32x32x16", iters: int = 2048, reps: int = 5,
                      device: str = "cuda") -> float:
    """Achievable bf16 MFMA TFLOP/s of one shape (``measure_mfma_peak_detail``
    without the clock ramp)."""
    return measure_mfma_peak_detail(shape, iters, reps, ramp_s=0.0, device=device)["TFLOP/s"]


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
