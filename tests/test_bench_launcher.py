"""bench.py's multi-rank contract on CPU (no GPU): ``python bench.py --gpus
N`` started as one process launches N ranks itself, they rendezvous (gloo
here, RCCL on the node), time with a barrier and a max over ranks, and rank 0
prints one JSON line with ``n_gpus`` = N.  ``--selftest`` swaps the flash
step for a CPU matmul so the launch path runs without a device."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {}, PLI_BENCH_BACKEND="gloo")
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


@pytest.mark.timeout(300)
def test_bench_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--selftest", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    # gloo itself prints "[Gloo] Rank i is connected ..." lines to stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["backend"] == "gloo"
    assert d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    assert d["data"].startswith("SELFTEST")
    assert d["summary"] == {"n_gpus": 2, "ranks_seen": 2, "backend": "gloo"}  # the tail the driver keeps


@pytest.mark.timeout(120)
def test_bench_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--selftest"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 3 and "WORLD_SIZE 1 != --gpus 2" in r.stderr


def test_headline_summary_and_tail_order():
    """The JSON line ends with the sub-results and `summary` (the driver
    keeps only ~8 KB of stdout's tail): summary carries the flash, causal,
    dtype-leg, GEMV, GEMM and TP numbers from their records."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r = {"roofline": {"achieved": 1390.0, "frac": 0.552, "kernel_ms": 1.58},
         "unramped": {"TFLOP/s": 1350.0},
         "flash_causal": {"TFLOP/s": 1150.0, "ms": 0.96},
         "gemv": {"us_per_launch": 7.3, "GB/s": 4600.0,
                  "roofline": {"frac": 0.575, "measured_peak": 4510.0}},
         "gemm": {"TFLOP/s": 1258.0, "torch_mm_TFLOP/s": 1223.0},
         "tp_gemm": {"gemm_TFLOP/s": 1488.0, "torch_F.linear_TFLOP/s": 1576.0,
                     "shard_gemm_per_rank": {"tp2": {"TFLOP/s": 1437.0, "torch_F.linear_TFLOP/s": 1511.0}}},
         "flash_dtypes": {"fp16_d128": {"non_causal": {"TFLOP/s": 1300.0}, "causal": {"TFLOP/s": 1108.0}},
                          "kernels": "..."}}
    s = bench.headline_summary(r)
    assert s["flash_TFLOP/s"] == 1390.0 and s["flash_unramped_TFLOP/s"] == 1350.0
    assert s["causal_TFLOP/s"] == 1150.0 and s["gemv_us"] == 7.3 and s["gemv_size_matched_probe_GB/s"] == 4510.0
    assert s["tp2_shard_TFLOP/s"] == [1437.0, 1511.0] and s["flash_fp16_d128_TFLOP/s"] == [1300.0, 1108.0]
    assert len(json.dumps(s)) < 2048  # fits the tail with room to spare
    assert s["n_gpus"] is None and "tp_allreduce_us" not in s  # (a one-GPU record)


def test_headline_summary_multi_rank_keys():
    """N > 1 (verdict r5 item 5): the rank count, backend and the TP
    all-reduce leg (ch09 RowParallelLinear over RCCL) land in `summary`"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r = {"roofline": {"achieved": 1390.0, "frac": 0.552, "kernel_ms": 1.58}, "n_gpus": 2, "ranks_seen": 2,
         "backend": "nccl",
         "tp_gemm": {"gemm_TFLOP/s": 1400.0, "torch_F.linear_TFLOP/s": 1500.0, "allreduce_us": 95.0,
                     "total_us": 480.0, "overlapped_total_us": 420.0, "allreduce_busbw_GB/s": 176.0,
                     "xgmi_ring_bound_us": 90.0}}
    s = bench.headline_summary(r)
    assert (s["n_gpus"], s["ranks_seen"], s["backend"]) == (2, 2, "nccl")
    for key in ("allreduce_us", "total_us", "overlapped_total_us", "allreduce_busbw_GB/s", "xgmi_ring_bound_us"):
        assert s[f"tp_{key}"] == r["tp_gemm"][key]
