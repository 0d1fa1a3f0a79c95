#!/usr/bin/env python3
"""Benchmark of the MI355X hot path (the driver's contract).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--quick]

One "step" = one fused flash-attention prefill forward over the BASELINE
config (ch06, B=8 S=4096 H=32 D=128, bf16, non-causal) on every rank.
Flash is "replicas only" (each rank an independent replica, no collective),
so ``value`` = N x per-replica work / max-over-ranks time (weak scaling).

The same JSON line carries, as sub-objects, the other hot-path rows:
  gemv    ch03 decode GEMV 4096x4096 bf16 (W rotated over >256 MiB so every
          launch streams from HBM, not the 256 MiB Infinity Cache)
  decode_attn  ch02 decode attention over a [B, S, Hkv, D] KV cache (B=8,
          Hq=32, Hkv=8, S=32768, D=128 bf16, 1 GiB), split-K flash-decoding
  gemm    ch05/ch03 4096^3 bf16 NN GEMM
  tp_gemm ch09 row-parallel 8192x8192 GEMM, M=8192, + RCCL all-reduce over
          xGMI when N > 1 (compute / all-reduce / total / bus bandwidth)
  cpu_baseline  the reference tile loop restated on torch CPU (oracle, kind
          "port"), rank 0, N=1 only, on a bounded sample of the workload.
  cpu_other     torch.mv / torch.mm / one TP8 shard F.linear on the host cores
  tp_gemm.small_m  the TP shard GEMM at M = 1 and 128
  flash_wallclock_ms  the reference's timing style (sync per call) beside the events
  flash_torch_sdpa    torch SDPA's fused backends on the same tensors (comparison)

All device times are HIP events recorded on the stream the kernels run on.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "physics-llm-inference_amd")
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "flash-attn prefill TFLOP/s + GEMV decode GB/s, as % of MI355X roofline"
PEAK_BF16_TFLOPS = 2516.6   # 256 CU x 4096 FLOP/clk x 2.4 GHz (dense)
PEAK_HBM_GBPS = 8000.0      # HBM3E datasheet
B, H, S, D = 8, 32, 4096, 128
FLASH_KERNEL = ("attn_fwd_v13 persistent (variant 80; v_mfma_f32_16x16x32_bf16, one generated instruction stream, "
                "tools/gen_flash_v13.py)")
JSON_OUT = sys.stdout  # main() points it at the original stdout and sends fd 1 to stderr
GEMM_KERNEL = ("gemm_w5 (256x256 tile, one wave per SIMD, K staged 64 deep; variant 43, its persistent walk, "
               "where M, N are multiples of 256 and K >= 128)")
CAUSAL_KERNEL = "attn_fwd_v13c causal, persistent pair walk (variant 83)"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def event_time_ms(fn, iters: int, stream) -> float:
    """Mean ms per call of ``fn`` over ``iters`` back-to-back calls, HIP events
    recorded on ``stream`` (the stream the kernels are launched on)."""
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(iters):
        fn()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / iters


def ramp(fn, ms: float = 300.0) -> int:
    """Back-to-back calls of ``fn`` for ``ms`` of wall time (a sync every 10),
    untimed: the clock settles on this kernel's own power draw before it is
    timed (a change of kernel moves it; the headline's 1 s ramp)"""
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(10):
            fn()
        n += 10
        torch.cuda.synchronize()
    return n


def paired_time_ms(fns: dict, iters: int, stream, rounds: int = 3, warm: int = 5) -> dict:
    """Median over `rounds` of event_time_ms per callable, the callables
    interleaved round by round after `warm` calls each, so that neither side
    of a comparison pays the clock ramp of the first measurement."""
    for fn in fns.values():
        for _ in range(warm):
            fn()
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            res[k].append(event_time_ms(fn, iters, stream))
    return {k: sorted(v)[len(v) // 2] for k, v in res.items()}


def load_pmc(kernel: str) -> dict:
    """The committed rocprofv3 PMC summary of ``kernel`` (profiles/traffic.json,
    tools/pmc_summary.py), or {}."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel, {})
    except (OSError, ValueError):
        return {}


def load_traffic(kernel: str):
    """Per-launch HBM bytes of ``kernel`` from the PMC summary, or None."""
    return load_pmc(kernel).get("hbm_bytes_per_launch")


def pmc_fields(kernel: str, kernel_ms: float | None = None) -> dict:
    """traffic plus the matrix-core occupancy of ``kernel`` from the PMC
    summary: mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
    GRBM_GUI_ACTIVE / 8), with the clock those passes ran at.  busy is a
    ratio of cycles, so with this run's kernel time it gives the clock the
    unprofiled kernel ran at: (busy cycles per SIMD / busy) / kernel time."""
    r = load_pmc(kernel)
    out = {"traffic": r.get("hbm_bytes_per_launch"), "mfma_busy": r.get("mfma_busy"),
           "pmc_clock_GHz": r.get("clock_GHz"), "lds_bank_conflict_cycles": r.get("SQ_LDS_BANK_CONFLICT")}
    cyc, busy = r.get("mfma_busy_cycles_per_simd"), r.get("mfma_busy")
    if kernel_ms and cyc and busy:
        out["implied_clock_GHz"] = cyc / busy / (kernel_ms * 1e6)
    return out


def calibrate() -> dict:
    """Measured ceilings beside the datasheet roofs: the HBM
    read stream over 2 x 1 GiB and at the GEMV's own 32 MiB footprint
    (graph-replayed over 24 rotated buffers, exactly like the GEMV leg), the
    copy kernel, and the MFMA probe of both bf16 shapes (one wave per SIMD,
    random operands, after a 2 s ramp, in-kernel clock stamped)."""
    from ch03.roofline import (measure_gemv_floor, measure_hbm_bandwidth, measure_hbm_read_bandwidth,
                               measure_hbm_read_bandwidth_sized, measure_mfma_peak_detail)
    m32 = measure_mfma_peak_detail("32x32x16")
    m16 = measure_mfma_peak_detail("16x16x32")
    return {"hbm_GB/s": measure_hbm_read_bandwidth(),
            "hbm_32MiB_per_launch": measure_hbm_read_bandwidth_sized(),
            "gemv_floor": measure_gemv_floor(),
            "hbm_copy_GB/s": measure_hbm_bandwidth(),
            "mfma_32x32x16_TFLOP/s": m32["TFLOP/s"], "mfma_32x32x16_clock_GHz": m32["clock_GHz"],
            "mfma_16x16x32_TFLOP/s": m16["TFLOP/s"], "mfma_16x16x32_clock_GHz": m16["clock_GHz"],
            "how": "hbm: pli_hbm_read_probe over 2 x 1 GiB (read-only, best of 10 per layout); "
                   "hbm_32MiB_per_launch: the same probe reading 33,570,816 B per launch from 24 buffers "
                   "in turn, one HIP graph of 24 launches (the GEMV leg's timing), best layout; "
                   "hbm_copy: pli_scale_copy 2x1 GiB read+write; mfma: pli_mfma_probe, 256 WGs x 4 waves "
                   "(one wave per SIMD), back-to-back MFMAs into independent accumulators, 64x64 output "
                   "tile per wave for both shapes, pseudo-random bf16, 2 s ramp then best of 5; clock = "
                   "median over waves of s_memtime/s_memrealtime x 100 MHz"}


def usable_cores() -> int:
    """Cores this process can actually run on: the affinity mask, capped by
    the cgroup CPU quota (cgroup v2 cpu.max / v1 cfs_quota) -- the GPU box
    shows os.cpu_count() = 256 but grants one GPU's share of them, and
    torch threads beyond the quota oversubscribe and stall."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def cpu_info() -> dict:
    """Host CPU as the CPU baselines ran on it: model name, os.cpu_count(),
    the cores this process may run on (cgroup/affinity) and torch threads."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cores": affinity,
            "usable_cores": usable_cores(), "torch_threads": torch.get_num_threads()}


def bench_torch_sdpa(q, k, v, o, stream) -> dict:
    """The vendor path on the same workload, for comparison only: PyTorch's
    scaled_dot_product_attention restricted to its fused backends (flash, then
    memory-efficient; on ROCm these are AOTriton / CK kernels), non-causal and
    causal, with the max |diff| to this build's output."""
    import pli_hip
    import torch.nn.functional as F
    from torch.nn.attention import SDPBackend, sdpa_kernel
    B_, H_, S_, D_ = q.shape
    out = {}
    for name, be in (("flash", SDPBackend.FLASH_ATTENTION), ("efficient", SDPBackend.EFFICIENT_ATTENTION)):
        try:
            with sdpa_kernel([be]):
                r = {}
                for causal in (False, True):
                    fn = lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal)  # noqa: E731
                    ref = fn()
                    torch.cuda.synchronize()
                    pli_out = pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=o)
                    diff = (ref.float() - pli_out.float()).abs().max().item()
                    ms = event_time_ms(fn, 5, torch.cuda.current_stream())
                    pairs = S_ * (S_ + 1) // 2 if causal else S_ * S_
                    r["causal" if causal else "non_causal"] = {
                        "ms": ms, "TFLOP/s": 4 * B_ * H_ * D_ * pairs / (ms * 1e-3) / 1e12,
                        "max_abs_diff_vs_pli": diff}
                out[name] = r
        except Exception as e:  # backend not built for this arch / dtype
            out[name] = {"unavailable": f"{type(e).__name__}: {str(e)[:160]}"}
    out["note"] = "comparison only (vendor kernels via torch), not part of value"
    return out


def bench_flash_dtypes(stream) -> dict:
    """The default flash route at the bench shape (B8 H32 S4096) for the other
    element types / head dims the reference runs (ch06/test_ch06.py:158-189
    is fp16 head_dim 64; ch01 MHA d=512 h=8 is head_dim 64): fp16 D=128,
    bf16 D=64, fp16 D=64, non-causal and causal; events over 20 launches
    after a 300 ms ramp of the same launch.  Reported only (value is the
    bf16 D=128 headline)."""
    import pli_hip
    out = {}
    for dt, D_ in (("fp16", 128), ("bf16", 64), ("fp16", 64)):
        tdt = torch.float16 if dt == "fp16" else torch.bfloat16
        g = torch.Generator(device="cuda").manual_seed(77)
        q, k, v = (torch.randn(B, H, S, D_, device="cuda", dtype=tdt, generator=g) for _ in range(3))
        o = torch.empty_like(q)
        r = {}
        for causal in (False, True):
            fn = lambda: pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=o)  # noqa: E731
            ramp(fn)
            ms = event_time_ms(fn, 20, stream)
            pairs = S * (S + 1) // 2 if causal else S * S
            r["causal" if causal else "non_causal"] = {"ms": ms,
                                                       "TFLOP/s": 4 * B * H * D_ * pairs / (ms * 1e-3) / 1e12}
        out[f"{dt}_d{D_}"] = r
        del q, k, v, o
    out["kernels"] = ("attn_fwd_v13h (fp16 D128), attn_fwd_pp64 (bf16 D64, since round 6), attn_fwd_v13h_d64 "
                      "(fp16 D64) and the v13 causal forms")
    return out


def headline_summary(r: dict) -> dict:
    """the numbers the round's verdict reads, in one short record (the last
    key of the JSON line, so it survives any tail truncation)"""
    out = {"flash_TFLOP/s": r["roofline"]["achieved"], "flash_frac": r["roofline"]["frac"],
           "flash_kernel_ms": r["roofline"]["kernel_ms"],
           "n_gpus": r.get("n_gpus"), "ranks_seen": r.get("ranks_seen"), "backend": r.get("backend")}
    if "unramped" in r:
        out["flash_unramped_TFLOP/s"] = r["unramped"]["TFLOP/s"]
    if "flash_causal" in r:
        out["causal_TFLOP/s"] = r["flash_causal"]["TFLOP/s"]
        out["causal_ms"] = r["flash_causal"]["ms"]
    if "gemv" in r:
        out["gemv_us"] = r["gemv"]["us_per_launch"]
        out["gemv_GB/s"] = r["gemv"]["GB/s"]
        out["gemv_frac"] = r["gemv"]["roofline"]["frac"]
        if "measured_peak" in r["gemv"]["roofline"]:
            out["gemv_size_matched_probe_GB/s"] = r["gemv"]["roofline"]["measured_peak"]
    if "gemm" in r:
        out["gemm_4096_TFLOP/s"] = r["gemm"]["TFLOP/s"]
        out["gemm_4096_torch_TFLOP/s"] = r["gemm"]["torch_mm_TFLOP/s"]
    if "tp_gemm" in r:
        t = r["tp_gemm"]
        out["tp_gemm_TFLOP/s"] = t["gemm_TFLOP/s"]
        out["tp_gemm_torch_TFLOP/s"] = t["torch_F.linear_TFLOP/s"]
        for tp, sh in t.get("shard_gemm_per_rank", {}).items():
            out[f"{tp}_shard_TFLOP/s"] = [sh["TFLOP/s"], sh["torch_F.linear_TFLOP/s"]]
        # N > 1: the all-reduce leg (ch09 RowParallelLinear over RCCL / xGMI)
        for key in ("allreduce_us", "total_us", "overlapped_total_us", "allreduce_busbw_GB/s",
                    "xgmi_ring_bound_us"):
            if key in t:
                out[f"tp_{key}"] = t[key]
    if "decode_attn" in r:
        out["decode_attn_GB/s"] = r["decode_attn"]["GB/s"]
    if "flash_dtypes" in r:
        for key, val in r["flash_dtypes"].items():
            if isinstance(val, dict):
                out[f"flash_{key}_TFLOP/s"] = [val["non_causal"]["TFLOP/s"], val["causal"]["TFLOP/s"]]
    return out


def bench_gemv(stream, iters: int) -> dict:
    """ch03 decode GEMV 4096x4096 bf16.  W is rotated over 24 copies (768 MiB,
    3x the 256 MiB Infinity Cache) so every launch streams W from HBM.  The
    24 launches are captured once in a HIP graph and replayed, so the time
    per launch is device time (kernel + kernel boundary), not Python launch
    overhead; the eager per-call rate is reported beside it."""
    import pli_hip
    from ch03 import gemv_bytes
    m = k = 4096
    copies = 24
    ws = [torch.randn(m, k, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
    x = torch.randn(k, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(m, device="cuda", dtype=torch.bfloat16)
    for w in ws:
        pli_hip.gemv(w, x, out=y)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for w in ws:
            pli_hip.gemv(w, x, out=y)
    for _ in range(3):
        graph.replay()
    reps = max(1, iters // copies)
    ms = event_time_ms(graph.replay, reps, stream) / copies
    state = {"i": 0}

    def eager():
        pli_hip.gemv(ws[state["i"] % copies], x, out=y)
        state["i"] += 1
    ms_eager = event_time_ms(eager, 4 * copies, stream)
    # the vendor path under the same rotation and graph (comparison only)
    yt = torch.empty(m, device="cuda", dtype=torch.bfloat16)
    for w in ws:
        torch.mv(w, x, out=yt)
    torch.cuda.synchronize()
    tgraph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(tgraph):
        for w in ws:
            torch.mv(w, x, out=yt)
    for _ in range(3):
        tgraph.replay()
    ms_torch = event_time_ms(tgraph.replay, reps, stream) / copies
    nbytes = gemv_bytes(m, k, torch.bfloat16)
    gbps = nbytes / (ms * 1e-3) / 1e9
    # streaming asymptote of the same body: one 16384x16384 launch (512 MiB),
    # through variant 13 (the default's 1 row x 8 chunks per wave in 4-wave
    # blocks) so rocprof keeps the 4096^2 dispatches in a row of their own
    big = torch.randn(16384, 16384, device="cuda", dtype=torch.bfloat16)
    xb = torch.randn(16384, device="cuda", dtype=torch.bfloat16)
    yb = torch.empty(16384, device="cuda", dtype=torch.bfloat16)
    pli_hip.gemv(big, xb, out=yb, variant=13)
    ms_big = event_time_ms(lambda: pli_hip.gemv(big, xb, out=yb, variant=13), 10, stream)
    del big
    return {"workload": "ch03 GEMV 4096x4096 bf16, batch 1, W rotated over 768 MiB (HBM-resident)",
            "us_per_launch": ms * 1e3, "GB/s": gbps, "timing": "HIP graph of 24 launches, events",
            "eager_us_per_call": ms_eager * 1e3,
            "torch_mv_us_per_launch": ms_torch * 1e3,
            "streaming_16384sq_GB/s": gemv_bytes(16384, 16384, torch.bfloat16) / (ms_big * 1e-3) / 1e9,
            "streaming_kernel": "gemv_vec variant 13 (same body, 4-wave blocks)",
            "roofline": {"bound": "hbm", "achieved": gbps, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": gbps / PEAK_HBM_GBPS, "algorithmic_bytes": nbytes,
                         **pmc_fields("gemv_vec")}}


def bench_matmul_demo() -> dict:
    """ch05/tiled_matmul.cu main at its own size (2048^3 fp32, inputs
    (rand() % 100) / 100): the naive contrast kernel vs the fp32 MFMA tile
    (ch05.benchmark_matmul_demo), with the f32 MFMA roofline of the tile."""
    from ch05 import benchmark_matmul_demo
    d = benchmark_matmul_demo(2048, warmup=3, iterations=10)
    peak = PEAK_BF16_TFLOPS / 16  # v_mfma_f32_32x32x2_f32: 1/16 of the bf16 rate
    d["workload"] = "ch05/tiled_matmul.cu 2048^3 fp32, naive vs MFMA tile"
    d["roofline"] = {"bound": "mfma", "achieved": d["tiled"]["tflops"], "peak": peak, "unit": "TFLOP/s",
                     "frac": d["tiled"]["tflops"] / peak, "kernel": "gemm_f32_mfma (v_mfma_f32_32x32x2_f32)"}
    return d


def bench_decode(stream, iters: int) -> dict:
    """ch02 decode step attention: one new token per sequence over the cache
    (GQA 32/8), bf16.  Two caches (2 GiB) alternate so no launch re-reads the
    256 MiB Infinity Cache.  Algorithmic bytes = the valid K + V prefix + q + o.
    The reference formulation (repeat_interleave + matmul + softmax + matmul,
    ch02/kv_cache.py:81-98) is timed on the same device beside it."""
    import math
    import pli_hip
    Bd, Hq, Hkv, n, Dd = 8, 32, 8, 32768, 128
    caches = [(torch.randn(Bd, n, Hkv, Dd, device="cuda", dtype=torch.bfloat16),
               torch.randn(Bd, n, Hkv, Dd, device="cuda", dtype=torch.bfloat16)) for _ in range(2)]
    qd = torch.randn(Bd, 1, Hq, Dd, device="cuda", dtype=torch.bfloat16)
    od = torch.empty_like(qd)
    state = {"i": 0}

    def step():
        kc, vc = caches[state["i"] & 1]
        state["i"] += 1
        pli_hip.attn_decode(qd, kc, vc, n, out=od, causal=False)
    for _ in range(4):
        step()
    ms = event_time_ms(step, iters, stream)
    nbytes = 2 * Bd * n * Hkv * Dd * 2 + 2 * qd.numel() * 2
    gbps = nbytes / (ms * 1e-3) / 1e9

    def ref():
        kc, vc = caches[0]
        qt = qd.transpose(1, 2)
        kt = kc.transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
        vt = vc.transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
        return torch.matmul(torch.softmax(torch.matmul(qt, kt.transpose(-2, -1)) / math.sqrt(Dd),
                                          dim=-1), vt)
    ref()
    ms_ref = event_time_ms(ref, 3, stream)
    del caches
    torch.cuda.empty_cache()
    return {"workload": "ch02 decode attention, B=8 Hq=32 Hkv=8 S=32768 D=128 bf16 (1 GiB cache)",
            "us_per_launch": ms * 1e3, "GB/s": gbps, "timing": "events, 2 caches alternated",
            "reference_formulation_GB/s": nbytes / (ms_ref * 1e-3) / 1e9,
            "roofline": {"bound": "hbm", "achieved": gbps, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": gbps / PEAK_HBM_GBPS, "algorithmic_bytes": nbytes,
                         "traffic": load_traffic("attn_decode_chunk")}}


def bench_gemm(stream, iters: int) -> dict:
    import pli_hip
    n = 4096
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    t = paired_time_ms({"ours": lambda: pli_hip.gemm(a, b, out=c), "torch": lambda: torch.mm(a, b)},
                       iters, stream)
    ms, ms_t = t["ours"], t["torch"]
    tf = 2 * n ** 3 / (ms * 1e-3) / 1e12
    return {"workload": "ch05/ch03 GEMM 4096^3 bf16 NN", "kernel": GEMM_KERNEL, "us_per_launch": ms * 1e3,
            "timing": f"events, median of 3 interleaved rounds of {iters} launches (ours / torch)",
            "TFLOP/s": tf, "torch_mm_TFLOP/s": 2 * n ** 3 / (ms_t * 1e-3) / 1e12,
            "roofline": {"bound": "mfma", "achieved": tf, "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": tf / PEAK_BF16_TFLOPS,
                         "algorithmic_bytes": 3 * n * n * 2, **pmc_fields("gemm_w5 nn", ms)}}


def bench_tp(stream, world: int, rank: int, iters: int) -> dict:
    """RowParallel 8192x8192 (K split over ranks), M = 8192, + RCCL all-reduce."""
    import pli_hip
    from ch09 import row_parallel_forward_overlapped, xgmi_all_reduce_bounds
    M, N, K = 8192, 8192, 8192
    kl = K // world
    x = torch.randn(M, kl, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, kl, device="cuda", dtype=torch.bfloat16) * kl ** -0.5
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gemm = lambda: pli_hip.gemm(x, w, trans_b=True, out=y)  # noqa: E731
    tl = lambda: torch.nn.functional.linear(x, w)  # noqa: E731  (hipBLASLt, same shapes)
    t = paired_time_ms({"ours": gemm, "torch": tl}, iters, stream)
    ms_gemm, ms_torch = t["ours"], t["torch"]
    out = {"workload": f"ch09 RowParallel 8192x8192 TP={world}, M={M}, bf16",
           "timing": f"events, median of 3 interleaved rounds of {iters} launches (ours / torch)",
           "gemm_us": ms_gemm * 1e3, "gemm_TFLOP/s": 2 * M * N * kl / (ms_gemm * 1e-3) / 1e12,
           "torch_F.linear_TFLOP/s": 2 * M * N * kl / (ms_torch * 1e-3) / 1e12}
    # also M in {1, 128} (decode batches; W streamed from HBM)
    small = {}
    for m in (1, 128):
        xs = torch.randn(m, kl, device="cuda", dtype=torch.bfloat16)
        ys = torch.empty(m, N, device="cuda", dtype=torch.bfloat16)
        fs = lambda: pli_hip.gemm(xs, w, trans_b=True, out=ys)  # noqa: E731
        tls = lambda: torch.nn.functional.linear(xs, w)  # noqa: E731
        t = paired_time_ms({"ours": fs, "torch": tls}, 20, stream)
        ms, ms_t = t["ours"], t["torch"]
        small[str(m)] = {"gemm_us": ms * 1e3, "weight_GB/s": N * kl * 2 / (ms * 1e-3) / 1e9,
                         "TFLOP/s": 2 * m * N * kl / (ms * 1e-3) / 1e12, "torch_F.linear_us": ms_t * 1e3}
    out["small_m"] = small
    if world == 1:
        # per-rank compute of the TP = 2 / 4 / 8 row shards (K = 8192 / tp) on
        # this one GPU, so every TP degree's GEMM is measured without a node
        shards = {}
        for tp in (2, 4, 8):
            ks = K // tp
            xs = torch.randn(M, ks, device="cuda", dtype=torch.bfloat16)
            wsh = torch.randn(N, ks, device="cuda", dtype=torch.bfloat16) * ks ** -0.5
            fs = lambda: pli_hip.gemm(xs, wsh, trans_b=True, out=y)  # noqa: E731
            tls = lambda: torch.nn.functional.linear(xs, wsh)  # noqa: E731
            t = paired_time_ms({"ours": fs, "torch": tls}, iters, stream)
            fl = 2 * M * N * ks
            shards[f"tp{tp}"] = {"K": ks, "gemm_us": t["ours"] * 1e3,
                                 "TFLOP/s": fl / (t["ours"] * 1e-3) / 1e12,
                                 "torch_F.linear_TFLOP/s": fl / (t["torch"] * 1e-3) / 1e12}
            del xs, wsh
        out["shard_gemm_per_rank"] = shards
        out["partial_rounding"] = partial_rounding_by_tp()
    if world > 1:
        def ar():
            dist.all_reduce(y)
        for _ in range(2):
            ar()
        torch.cuda.synchronize()
        ms_ar = event_time_ms(ar, iters, stream)

        def full():
            gemm()
            dist.all_reduce(y)
        ms_full = event_time_ms(full, iters, stream)
        ms_ovl = event_time_ms(lambda: row_parallel_forward_overlapped(x, w, chunks=4), iters, stream)
        payload = M * N * 2
        bounds = xgmi_all_reduce_bounds(payload, world)
        out.update({"allreduce_us": ms_ar * 1e3, "total_us": ms_full * 1e3,
                    "overlapped_total_us": ms_ovl * 1e3,
                    "allreduce_busbw_GB/s": payload / (ms_ar * 1e-3) / 1e9 * bounds["bus_factor"],
                    "xgmi_mesh_bound_us": bounds["mesh_us"], "xgmi_ring_bound_us": bounds["ring_us"]})
    return out


def partial_rounding_by_tp(M: int = 1024, N: int = 8192, K: int = 8192) -> dict:
    """Error of the row-parallel sum against the f64 product by TP degree
    (ch09 RowParallelLinear, all-reduce simulated on one GPU by summing the
    tp shard partials in fp32): bf16 partials (each rank's output rounded,
    the default) vs fp32 partials (reduce_dtype=torch.float32,
    pli_gemm_f32out); the sum is rounded to bf16 once at the end.  Also the
    TP-8 shard's fp32-output GEMM time beside the bf16 one at M = 8192."""
    import pli_hip
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    ref = x.double() @ w.double().T
    scale = ref.abs().mean().item()
    res = {"workload": f"M={M} N={N} K={K} bf16, f64 reference", "mean_|ref|": scale}
    for tp in (1, 2, 4, 8):
        ks = K // tp
        s16 = torch.zeros(M, N, device="cuda")
        s32 = torch.zeros(M, N, device="cuda")
        for r in range(tp):
            xs, wsh = x[:, r * ks:(r + 1) * ks], w[:, r * ks:(r + 1) * ks]
            s16 += pli_hip.gemm(xs, wsh, trans_b=True).float()
            s32 += pli_hip.gemm_f32out(xs, wsh)
        e16 = (s16.bfloat16().double() - ref).abs()
        e32 = (s32.bfloat16().double() - ref).abs()
        res[f"tp{tp}"] = {"bf16_partials_mean_err": e16.mean().item(), "bf16_partials_max_err": e16.max().item(),
                          "fp32_partials_mean_err": e32.mean().item(), "fp32_partials_max_err": e32.max().item()}
    xs = torch.randn(8192, K // 8, device="cuda", dtype=torch.bfloat16, generator=g)
    ws = (torch.randn(N, K // 8, device="cuda", generator=g) * (K // 8) ** -0.5).to(torch.bfloat16)
    y16 = torch.empty(8192, N, device="cuda", dtype=torch.bfloat16)
    y32 = torch.empty(8192, N, device="cuda", dtype=torch.float32)
    t = paired_time_ms({"bf16": lambda: pli_hip.gemm(xs, ws, trans_b=True, out=y16),
                        "fp32": lambda: pli_hip.gemm_f32out(xs, ws, out=y32)}, 10, torch.cuda.current_stream())
    res["tp8_shard_M8192_us"] = {"bf16_out": t["bf16"] * 1e3, "fp32_out": t["fp32"] * 1e3}
    return res


def bench_decode_step(batches=(1, 32), prompt: int = 512, steps: int = 32) -> dict:
    """ch02 decode step of a Llama-shaped 0.85B model (vocab 32000, hidden
    2048, 16 layers, 32/8 heads, intermediate 5632, random bf16 weights) as
    one HIP-graph launch per token (ch08.DecodeStepGraph): per-token latency
    over `steps` replays after a `prompt`-token prefill, host loop included."""
    from ch02 import CachedTransformerModel
    from ch08 import DecodeStepGraph
    torch.manual_seed(0)
    model = CachedTransformerModel(32000, 2048, 16, 32, 8, 5632).cuda().bfloat16().eval()
    out = {"workload": "ch02/ch08 decode step, 0.85B Llama shape, bf16, HIP graph per token",
           "prompt": prompt, "timing": f"perf_counter over {steps} replays after 1 warm replay"}
    with torch.no_grad():
        for B in batches:
            ids = torch.randint(0, 32000, (B, prompt), device="cuda")
            tok = torch.randint(0, 32000, (B, 1), device="cuda")
            g = DecodeStepGraph(model, B, prompt + steps + 8, torch.bfloat16)
            g.prefill(ids)
            g.step(tok)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                g.step(tok)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            out[f"batch{B}_ms_per_token"] = ms
            out[f"batch{B}_tok/s"] = B / (ms * 1e-3)
            del g
    del model
    torch.cuda.empty_cache()
    return out


def cpu_baseline(seconds: float = 15.0) -> dict:
    """The reference tile loop (oracle restatement, torch CPU) on a sample of
    the flash workload: B=1 (1/8 of the batch), all 32 heads, S=4096, D=128."""
    from oracle.attention import flash_tile_loop_torch
    b = 1
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(b, H, S, D, generator=g).to(torch.bfloat16) for _ in range(3))
    flops = 4 * b * H * S * S * D
    # torch.set_num_threads(os.cpu_count()) -- capped at the
    # cores the process may actually use (usable_cores: affinity and cgroup
    # quota; 256 threads on a 16-core share stall in OpenMP barriers), and
    # torch's default thread count timed beside it; the faster is the baseline
    default_threads = torch.get_num_threads()
    tried, best = {}, None
    for threads in sorted({usable_cores(), default_threads}, reverse=True):
        torch.set_num_threads(threads)
        flash_tile_loop_torch(q[:, :2], k[:, :2], v[:, :2])  # warm
        times, t_end = [], time.perf_counter() + seconds / 2
        while len(times) < 1 or (time.perf_counter() < t_end and len(times) < 5):
            t0 = time.perf_counter()
            flash_tile_loop_torch(q, k, v)
            times.append(time.perf_counter() - t0)
        sec = min(times)
        tried[str(threads)] = flops / sec / 1e12
        if best is None or sec < best[0]:
            best = (sec, threads, len(times))
    sec, threads, n = best
    torch.set_num_threads(threads)
    info = cpu_info()
    torch.set_num_threads(default_threads)
    return {"value": flops / sec / 1e12, "unit": "TFLOP/s", "cores": threads,
            "kind": "port", **info, "TFLOP/s_by_threads": tried,
            "sample": f"reference tile loop (ch06/flash_attention.py:14-74 restated, oracle/attention.py) "
                      f"on torch CPU bf16, B=1 H=32 S=4096 D=128 = 1/8 of the workload, "
                      f"best of {n} runs ({sec:.2f} s each) at {threads} threads "
                      f"(usable cores {usable_cores()} of os.cpu_count() {os.cpu_count()}, and the default "
                      f"{default_threads}, tried)"}


def cpu_other(cores: int | None = None) -> dict:
    """SURVEY 8(d)'s other CPU baselines, torch CPU on the box's host cores
    (bounded: a few seconds in all): torch.mv 4096^2 (ch03 GEMV, 10 + 100),
    torch.mm 4096^3 NN (ch03 GEMM, 2 + 5), one TP8 row shard F.linear
    ([8192, 1024] x [8192, 1024]^T, 2 + 5)."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(0)
    out = {"cores": torch.get_num_threads(), "dtype": "bf16", "kind": "reference ops (torch CPU)",
           **cpu_info()}
    if cores is not None:
        default_threads = torch.get_num_threads()
        torch.set_num_threads(cores)
        out.update(cores=cores, **cpu_info())

    def tmin(fn, warm, iters):
        for _ in range(warm):
            fn()
        best = float("inf")
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        return best

    w = torch.randn(4096, 4096, generator=g).bfloat16()
    x = torch.randn(4096, generator=g).bfloat16()
    t = tmin(lambda: torch.mv(w, x), 10, 100)
    out["gemv_torch.mv"] = {"us": t * 1e6, "GB/s": 33570816 / t / 1e9}
    a = torch.randn(4096, 4096, generator=g).bfloat16()
    t = tmin(lambda: torch.mm(a, w), 2, 5)
    out["gemm_torch.mm_4096"] = {"ms": t * 1e3, "TFLOP/s": 2 * 4096 ** 3 / t / 1e12}
    xs = torch.randn(8192, 1024, generator=g).bfloat16()
    ws = torch.randn(8192, 1024, generator=g).bfloat16()
    t = tmin(lambda: F.linear(xs, ws), 2, 5)
    out["tp8_shard_F.linear"] = {"ms": t * 1e3, "TFLOP/s": 2 * 8192 * 8192 * 1024 / t / 1e12}
    if cores is not None:
        torch.set_num_threads(default_threads)
    return out


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args) -> int:
    """``bench.py --gpus N`` (N > 1) started as ONE process: start N rank
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    MASTER_ADDR 127.0.0.1) before anything touches the GPU, pass their
    stdout through (rank 0 prints the one JSON line) and exit with the worst
    rank's status.  If a rank fails, the others are stopped (by PID) so none
    waits forever in a collective."""
    import subprocess
    n = args.gpus
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rcs = [None] * n
    deadline = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if deadline is None and any(rc not in (None, 0) for rc in rcs):
            deadline = time.time() + 30  # a rank failed: give the rest 30 s, then stop them
        if deadline is not None and time.time() > deadline:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.kill()
                    rcs[i] = p.wait()
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        log(f"[bench] rank exit codes {rcs}")
    return bad[0] if bad else 0


def selftest_main(args, world: int, rank: int) -> None:
    """CPU rehearsal of the multi-rank contract (tests/test_bench_launcher.py):
    the same launch, rendezvous, barrier + max-over-ranks timing and JSON
    line, with a small torch CPU matmul as the step.  Never a bench result
    (``data`` says so)."""
    if world > 1:
        dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            log(f"[bench] world size {dist.get_world_size()} != --gpus {args.gpus}")
            sys.exit(3)
    a = torch.randn(256, 256)
    step = lambda: a @ a  # noqa: E731
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ranks_seen = torch.ones(1)
    if world > 1:
        dist.all_reduce(ranks_seen)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": world * 2 * 256 ** 3 * args.steps / t.item() / 1e12,
                          "unit": "TFLOP/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": t.item() / args.steps * 1e3, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                          "data": "SELFTEST: launcher rehearsal on CPU, not a measurement",
                          "ranks_seen": int(ranks_seen.item()),
                          "backend": dist.get_backend() if world > 1 else None,
                          "config": {"workload": "selftest"},
                          "summary": {"n_gpus": world, "ranks_seen": int(ranks_seen.item()),
                                      "backend": dist.get_backend() if world > 1 else None}}),
              file=JSON_OUT, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed launches first: the first ~10 flash launches in a process run
    # 2-15 % slower (clock / TLB warm-up; rocprof trace in profiles/r02/final)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quick", action="store_true", help="skip gemm/tp/cpu legs")
    ap.add_argument("--with-decode", action="store_true", help="with --quick: keep the decode leg")
    ap.add_argument("--flash-only", action="store_true",
                    help="only the headline flash step (clean rocprof stats for that kernel)")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU rehearsal of the multi-rank launch (gloo, a CPU matmul step; not a result)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process asked for N GPUs: start the N ranks (nothing has touched the GPU yet)
        sys.exit(launch_ranks(args))
    # stdout carries exactly the one JSON line: anything a library prints there
    # (gloo's connection banner, runtime notices) goes to stderr instead
    global JSON_OUT
    JSON_OUT = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE {world} != --gpus {args.gpus}")
        sys.exit(3)
    if args.selftest:
        selftest_main(args, world, rank)
        return
    backend = None
    if world > 1:
        # PLI_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with
        # fewer GPUs than ranks (ranks share devices round-robin); the driver's
        # runs use the default, RCCL ("nccl") with one rank per GPU
        backend = os.environ.get("PLI_BENCH_BACKEND", "nccl")
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group(backend, device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            log(f"[bench] process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
            sys.exit(3)
    import pli_hip
    assert pli_hip.available(), "libpli_hip.so must be built and a ROCm device visible"

    stream = torch.cuda.current_stream()
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, generator=gen)
               for _ in range(3))
    o = torch.empty_like(q)
    step = lambda: pli_hip.flash_attn_fwd(q, k, v, out=o)  # noqa: E731
    flops_step = 4 * B * H * S * S * D

    # the driver's protocol first, as asked: W warmup steps, then K steps
    # timed (barrier + synchronize both sides) -- reported as `unramped`
    # beside the headline (the headline below follows a 1 s ramp)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    route = pli_hip.last_route()  # the kernel the timed step launches (pli_last_route)
    if world > 1:
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_u = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    unramped = {"wall_ms_per_step": (time.perf_counter() - t_u) / args.steps * 1e3,
                "kernel_ms": ev0.elapsed_time(ev1) / args.steps,
                "note": "the driver's --warmup W then --steps K on a fresh process (no ramp); rank-local"}
    unramped["TFLOP/s"] = 4 * B * H * S * S * D / (unramped["kernel_ms"] * 1e-3) / 1e12
    # device ramp: a fresh process starts from an idle clock state, and a
    # short --warmup (the driver runs W = 5, 8 ms) leaves part of the clock
    # ramp inside the timed steps; run the step back to back for ramp_ms of
    # wall time first (untimed, like the W warmup steps that follow)
    ramp_ms = float(os.environ.get("PLI_BENCH_RAMP_MS", "1000"))
    t_ramp = time.perf_counter()
    n_ramp = 0
    while (time.perf_counter() - t_ramp) * 1e3 < ramp_ms:
        for _ in range(10):
            step()
        n_ramp += 10
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    ev_s, ev_e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_s.record(stream)
    for _ in range(args.steps):
        step()
    ev_e.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev_s.elapsed_time(ev_e) / args.steps  # per launch, on the launch stream
    t = torch.tensor([wall], device="cuda", dtype=torch.float64)
    ranks_seen = torch.ones(1, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(ranks_seen)
    wall_max = t.item()
    value = world * flops_step * args.steps / wall_max / 1e12
    achieved = flops_step / (kernel_ms * 1e-3) / 1e12

    extra = {}
    measured_roof = {}
    log(f"[bench] flash: {achieved:.1f} TF/s per launch ({kernel_ms:.3f} ms)")
    # causal variant of the same workload (ch01 MHA semantics), reported only
    # (a 300 ms ramp of causal launches, then 20 timed: the first launches
    # after a change of kernel or an idle gap run slower -- round 5 used 10
    # warm-up launches and read 1136-1157 where same-process A/B reads
    # 1213-1223)
    if not args.flash_only:
        ramp(lambda: pli_hip.flash_attn_fwd(q, k, v, causal=True, out=o))
        ms_c = event_time_ms(lambda: pli_hip.flash_attn_fwd(q, k, v, causal=True, out=o), 20, stream)
        # the reference's own timing style (sync per call, wall clock), next to the events
        wc = []
        for _ in range(5):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            wc.append(time.perf_counter() - t1)
        extra["flash_wallclock_ms"] = {"mean": sum(wc) / len(wc) * 1e3, "min": min(wc) * 1e3,
                                       "timing": "sync + perf_counter per call, 5 calls"}
        extra["flash_causal"] = {"ms": ms_c, "timing": "events, 20 launches after a 300 ms ramp",
                                 "TFLOP/s": 4 * B * H * D * (S * (S + 1) // 2) / (ms_c * 1e-3) / 1e12,
                                 "kernel": CAUSAL_KERNEL, **pmc_fields("attn_fwd_v13c", ms_c)}
        log(f"[bench] causal: {extra['flash_causal']['TFLOP/s']:.1f} TF/s ({ms_c:.3f} ms)")
    if not args.flash_only:
        log("[bench] calibration")
        cal = calibrate()
        extra["calibration"] = cal
        # the flash kernel's QK^T / PV run on v_mfma_f32_16x16x32_bf16
        measured_roof = {"measured_peak": cal["mfma_16x16x32_TFLOP/s"],
                         "measured_peak_kind": "pli_mfma_probe 16x16x32 (the kernel's shape)",
                         "frac_of_measured": achieved / cal["mfma_16x16x32_TFLOP/s"]}
    if args.flash_only:
        args.quick, args.no_cpu_baseline = True, True
    if not args.flash_only:
        log("[bench] torch sdpa comparison")
        extra["flash_torch_sdpa"] = bench_torch_sdpa(q, k, v, o, stream)
        log("[bench] flash fp16 / head dim 64")
        extra["flash_dtypes"] = bench_flash_dtypes(stream)
        fd = extra["flash_dtypes"]
        log("[bench] flash " + ", ".join(f"{key} {val['non_causal']['TFLOP/s']:.0f}/{val['causal']['TFLOP/s']:.0f}"
                                          for key, val in fd.items() if isinstance(val, dict)) + " TF/s (plain/causal)")
    if args.flash_only:
        pass
    elif not args.quick:
        log("[bench] gemv")
        extra["gemv"] = bench_gemv(stream, 200)
        log(f"[bench] gemv: {extra['gemv']['us_per_launch']:.3f} us = {extra['gemv']['GB/s']:.0f} GB/s")
        log("[bench] decode attention")
        extra["decode_attn"] = bench_decode(stream, 20)
        log("[bench] gemm")
        extra["gemm"] = bench_gemm(stream, 20)
        log(f"[bench] gemm 4096^3: {extra['gemm']['TFLOP/s']:.1f} TF/s (torch.mm "
            f"{extra['gemm']['torch_mm_TFLOP/s']:.1f})")
        log("[bench] tp gemm")
        extra["tp_gemm"] = bench_tp(stream, world, rank, 10)
        log(f"[bench] tp gemm TP={world}: {extra['tp_gemm']['gemm_TFLOP/s']:.1f} TF/s (F.linear "
            f"{extra['tp_gemm']['torch_F.linear_TFLOP/s']:.1f})")
        if world == 1:
            log("[bench] decode step")
            extra["decode_step"] = bench_decode_step()
            log("[bench] ch05 demo")
            extra["ch05_matmul_demo"] = bench_matmul_demo()
    else:
        extra["gemv"] = bench_gemv(stream, 200)
        if args.with_decode:
            extra["decode_attn"] = bench_decode(stream, 20)

    if "calibration" in extra:
        cal = extra["calibration"]
        if "gemv" in extra:
            # the GEMV's own roof: the read probe at its 32 MiB footprint, timed the same way
            r = extra["gemv"]["roofline"]
            sized = cal["hbm_32MiB_per_launch"]["GB/s"]
            r.update({"measured_peak": sized, "measured_peak_kind": "hbm_32MiB_per_launch (size-matched)",
                      "frac_of_measured": r["achieved"] / sized,
                      "frac_of_streaming_read": r["achieved"] / cal["hbm_GB/s"]})
            # the fitted floor: per-launch boundary + the GEMV's bytes at the streaming slope
            fl = cal["gemv_floor"]
            r.update({"floor_us": fl["floor_us"], "empty_launch_us": fl["empty_launch_us"],
                      "frac_of_floor": fl["floor_us"] / extra["gemv"]["us_per_launch"]})
        if "decode_attn" in extra:
            r = extra["decode_attn"]["roofline"]
            r.update({"measured_peak": cal["hbm_GB/s"], "measured_peak_kind": "hbm read stream 2 x 1 GiB",
                      "frac_of_measured": r["achieved"] / cal["hbm_GB/s"]})
        if "gemm" in extra:
            # the 256-tile GEMM runs v_mfma_f32_16x16x32_bf16
            mp = cal["mfma_16x16x32_TFLOP/s"]
            extra["gemm"]["roofline"].update({"measured_peak": mp,
                                              "measured_peak_kind": "pli_mfma_probe 16x16x32 (the kernel's shape)",
                                              "frac_of_measured": extra["gemm"]["TFLOP/s"] / mp})

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ramp": {"ms": ramp_ms, "launches": n_ramp,
                 "note": "untimed back-to-back steps before the warmup (idle clock state of a fresh process)"},
        "unramped": unramped,
        "ms_per_step": wall_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (torch.randn N(0,1), seeded)",
        "ranks_seen": int(ranks_seen.item()),
        "backend": backend,
        "config": {"workload": "ch06 flash-attention prefill fwd, B=8 S=4096 H=32 D=128 bf16, "
                               "non-causal, one fused HIP launch per step",
                   "batch": B, "seq_len": S, "heads": H, "head_dim": D,
                   "parallelism": f"replicas x{world} (flash does not shard; TP GEMM row-parallel)"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / PEAK_BF16_TFLOPS,
                     **pmc_fields("attn_fwd_v13", kernel_ms),
                     "traffic_source": "profiles/traffic.json: rocprofv3 FETCH_SIZE x2 (gfx950) + WRITE_SIZE "
                                       "per launch, separate --pmc passes (tools/pmc_summary.py), not this run",
                     "kernel": FLASH_KERNEL, "route": route, "algorithmic_flops": flops_step,
                     "kernel_ms": kernel_ms, **measured_roof},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.quick:
        log("[bench] cpu baseline")
        result["cpu_baseline"] = cpu_baseline()
        result["cpu_other"] = cpu_other(result["cpu_baseline"]["cores"])
    # the bulky records first, the sub-results a reader checks last: the
    # driver keeps only the tail of stdout (~8 KB), so flash_causal, gemv,
    # gemm, tp_gemm and the one-line summary must sit at the end of the line
    late = ("flash_causal", "flash_dtypes", "decode_attn", "gemv", "gemm", "tp_gemm")
    for key, val in extra.items():
        if key not in late:
            result[key] = val
    for key in late:
        if key in extra:
            result[key] = extra[key]
    result["summary"] = headline_summary(result)
    if rank == 0:
        print(json.dumps(result), file=JSON_OUT, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
