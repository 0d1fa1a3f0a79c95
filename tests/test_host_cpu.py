"""Host-side logic on CPU: cost models vs the reference's own values
(golden analytic.json), CPU device paths vs the golden fixtures, and the
reference-visible API surface (names, defaults, parameter order)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle.numerics import array_hash, bf16_from_bits, seeded_normal

with open(os.path.join(GOLDEN, "analytic.json")) as _f:
    AN = json.load(_f)


def test_gemm_gemv_formulas_match_reference():
    from ch03 import gemm_bytes, gemm_flops, gemv_bytes, gemv_flops
    for e in AN["gemm"]:
        dt = getattr(torch, e["dtype"])
        assert gemm_flops(e["m"], e["n"], e["k"]) == e["flops"]
        assert gemm_bytes(e["m"], e["n"], e["k"], dt) == e["bytes"]
    for e in AN["gemv"]:
        dt = getattr(torch, e["dtype"])
        assert gemv_flops(e["m"], e["k"]) == e["flops"]
        assert gemv_bytes(e["m"], e["k"], dt) == e["bytes"]


def test_roofline_matches_reference_specs():
    from ch03 import roofline as rl
    from ch03.batching_benchmark import find_transition_batch_size
    for row in AN["roofline"]:
        spec = getattr(rl, row["hw"])
        assert (spec.peak_tflops, spec.memory_bandwidth_gbps, spec.name) == (row["peak"], row["bw"], row["name"])
        assert rl.ridge_point(spec) == pytest.approx(row["ridge"], rel=1e-12)
        for p in row["points"]:
            assert rl.roofline_throughput(p["ai"], spec) == pytest.approx(p["tput"], rel=1e-12)
            assert rl.is_compute_bound(p["ai"], spec) == p["cb"]
    for row in AN["transition"]:
        spec = getattr(rl, row["hw"])
        assert find_transition_batch_size(4096, 4096, spec.peak_tflops, spec.memory_bandwidth_gbps) == row["batch"]
    ai = AN["ai"]
    assert rl.gemm_arithmetic_intensity(4096, 4096, 4096) == pytest.approx(ai["gemm_4096"], rel=1e-12)
    assert rl.gemv_arithmetic_intensity(4096, 4096) == pytest.approx(ai["gemv_4096"], rel=1e-12)
    for b, v in zip((1, 4, 16, 64, 256, 512), ai["bgemv"]):
        assert rl.batched_gemv_arithmetic_intensity(b, 4096, 4096) == pytest.approx(v, rel=1e-12)
    assert rl.arithmetic_intensity(1000, 100) == ai["basic"]


def test_mi355x_roofline():
    from ch03 import roofline as rl
    assert rl.MI355X.peak_tflops == pytest.approx(2516.5824, rel=1e-9)
    assert rl.MI355X.memory_bandwidth_gbps == 8000.0
    assert rl.ridge_point(rl.MI355X) == pytest.approx(314.57, rel=1e-3)
    # GEMM 4096^3 is compute bound on MI355X, batch-1 GEMV memory bound
    assert rl.is_compute_bound(rl.gemm_arithmetic_intensity(4096, 4096, 4096), rl.MI355X)
    assert not rl.is_compute_bound(rl.gemv_arithmetic_intensity(4096, 4096), rl.MI355X)
    assert rl.roofline_fraction(1258.3, 2048.0) == pytest.approx(0.5, rel=1e-3)


def test_attention_cost_models_match_reference():
    from ch06 import attention_arithmetic_intensity, attention_flops, attention_memory_bytes
    from ch06.flash_attention import flash_attention_memory_bytes
    for e in AN["attn"]:
        B, H, N, D = e["B"], e["H"], e["N"], e["D"]
        st = attention_memory_bytes(B, H, N, D, 2)
        assert (st.qk_bytes, st.softmax_bytes, st.output_bytes, st.total_bytes) == (
            e["mem"]["qk"], e["mem"]["softmax"], e["mem"]["output"], e["mem"]["total"])
        assert st.total_mb == pytest.approx(e["mem"]["total_mb"], rel=1e-12)
        assert attention_flops(B, H, N, D) == e["flops"]
        assert attention_arithmetic_intensity(N, D) == pytest.approx(e["ai"], rel=1e-12)
        fm = flash_attention_memory_bytes(B, H, N, D)
        assert set(fm) == set(e["flash_mem"])
        for k2, v in e["flash_mem"].items():
            assert fm[k2] == (pytest.approx(v, rel=1e-12) if isinstance(v, float) else v)


def test_comm_models_match_reference():
    from ch09 import (AllGatherConfig, AllReduceConfig, compute_communication_overlap_potential,
                      compute_ring_all_reduce_time, simulate_all_gather, simulate_all_reduce)
    from ch09.tensor_parallel import compute_tp_memory_savings
    for e in AN["comm"]:
        ws = e["ws"]
        for got, want in ((simulate_all_reduce(AllReduceConfig(world_size=ws, data_size_mb=10.0)), e["ar"]),
                          (simulate_all_gather(AllGatherConfig(world_size=ws, data_size_per_gpu_mb=10.0)), e["ag"])):
            assert set(got) == set(want)
            for k2 in want:
                assert got[k2] == pytest.approx(want[k2], rel=1e-12)
        assert compute_ring_all_reduce_time(100 * 1024 * 1024, ws) == pytest.approx(e["ring"], rel=1e-12)
    for (c, m), want in zip(((1000, 100), (100, 1000), (500, 200)), AN["overlap"]):
        got = compute_communication_overlap_potential(c, m)
        for k2 in want:
            assert got[k2] == (pytest.approx(want[k2]) if isinstance(want[k2], float) else want[k2])
    for e in AN["tp"]:
        got = compute_tp_memory_savings(4096, 14336, e["ws"])
        for k2 in got:
            assert got[k2] == pytest.approx(e[k2], rel=1e-12)


def test_xgmi_bounds():
    from ch09 import xgmi_all_reduce_bounds
    b = xgmi_all_reduce_bounds(128 * 1024 * 1024, 8)
    assert b["ring_us"] == pytest.approx(2 * 7 / 8 * 128 * 1024 * 1024 / 153e3, rel=1e-9)
    assert b["mesh_us"] == pytest.approx(b["ring_us"] / 7, rel=1e-9)
    assert xgmi_all_reduce_bounds(1e6, 1)["ring_us"] == 0.0


def test_flash_config_defaults():
    from ch06 import FlashAttentionConfig
    c = FlashAttentionConfig()
    assert (c.block_q, c.block_k, c.num_warps, c.num_stages) == (64, 64, 4, 2)


@pytest.mark.parametrize("name", ["flash_b2h4n128d64_fp32.npz", "flash_b1h2n200d64_bf16.npz",
                                  "flash_b1h2n200d128_fp32.npz", "flash_b2h4n128d64_fp16.npz"])
def test_cpu_flash_path_vs_golden(name):
    from ch06 import flash_attention_forward
    g = load_golden(name)
    B, H, N, D = (int(x) for x in g["shape"])
    dt, seed = str(g["dtype"]), int(g["seed"])
    tdt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[dt]
    q, k, v = (torch.from_numpy(seeded_normal((B, H, N, D), seed * 10 + i, dt)).to(tdt) for i in range(3))
    out = flash_attention_forward(q, k, v).float().numpy()
    tol = 1e-5 if dt == "fp32" else 1e-2
    np.testing.assert_allclose(out, g["ref_naive_f64"], atol=tol, rtol=tol)


def test_cpu_mha_is_reference_exact():
    """CPU MultiHeadAttention reproduces the reference module's output."""
    from ch01 import MultiHeadAttention
    g = load_golden("mha.npz")
    torch.manual_seed(0)
    mha = MultiHeadAttention(512, 8)
    x = torch.from_numpy(seeded_normal((1, 128, 512), 31))
    with torch.no_grad():
        np.testing.assert_allclose(mha(x, causal=True).numpy(), g["y_causal"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(mha(x, causal=False).numpy(), g["y_noncausal"], rtol=1e-6, atol=1e-6)


def test_cpu_tp_layers_match_reference():
    from ch09 import ColumnParallelLinear, RowParallelLinear
    g = load_golden("tp.npz")
    torch.manual_seed(1)
    col = ColumnParallelLinear(256, 1024, world_size=4, rank=0, bias=True)
    torch.manual_seed(2)
    row = RowParallelLinear(1024, 256, world_size=4, rank=1, bias=True)
    assert tuple(col.weight.shape) == tuple(g["col_w_shape"])
    assert tuple(row.weight.shape) == tuple(g["row_w_shape"])
    assert array_hash(col.weight.detach().numpy()) == str(g["col_w_hash"])
    assert array_hash(row.weight.detach().numpy()) == str(g["row_w_hash"])
    # Same F.linear as the reference; the last bits depend on the host BLAS
    # kernel (AVX2 vs AVX-512 summation order), so not bit-exact across CPUs.
    with torch.no_grad():
        np.testing.assert_allclose(col(torch.from_numpy(seeded_normal((8, 256), 41))).numpy(), g["col_y"],
                                   rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(row(torch.from_numpy(seeded_normal((8, 256), 42))).numpy(), g["row_y"],
                                   rtol=1e-5, atol=1e-5)


def test_cpu_online_softmax_vs_golden():
    from ch06 import online_softmax, online_softmax_with_output, standard_softmax
    g = load_golden("softmax.npz")
    x3 = torch.from_numpy(seeded_normal((4, 8, 64), 21)).double()
    np.testing.assert_allclose(online_softmax(x3).numpy(), g["x3_online"], rtol=1e-12)
    np.testing.assert_allclose(standard_softmax(x3).numpy(), g["x3_standard"], rtol=1e-12)
    x4 = torch.from_numpy(seeded_normal((2, 4, 32), 22)).double()
    v4 = torch.from_numpy(seeded_normal((2, 4, 32, 16), 23)).double()
    o, d = online_softmax_with_output(x4, v4)
    np.testing.assert_allclose(o.numpy(), g["x4_o"], rtol=1e-10)
    np.testing.assert_allclose(d.numpy(), g["x4_d"], rtol=1e-10)


def test_triton_name_is_the_hip_gemm_on_cpu():
    from ch05 import tiled_matmul, triton_matmul
    a, b = torch.randn(8, 16), torch.randn(16, 4)
    torch.testing.assert_close(triton_matmul(a, b), a @ b)
    torch.testing.assert_close(triton_matmul(a, b, 32, 32, 32), tiled_matmul(a, b))
    from ch05.triton_matmul import TRITON_AVAILABLE, benchmark_triton_matmul
    assert TRITON_AVAILABLE is False  # no Triton kernel in this build
    assert benchmark_triton_matmul() is None  # no device here (the reference returns None too)
    for fn in (tiled_matmul, triton_matmul):
        with pytest.raises(AssertionError):
            fn(a, torch.randn(15, 4))


def test_flash_config_mapping_and_validation():
    """FlashAttentionConfig knobs: the HIP mapping is reported, bad values are
    rejected on the CPU path as on the GPU path."""
    from ch06 import FlashAttentionConfig, flash_attention_forward
    from ch06.flash_attention import HIP_TILING, hip_tiling
    m = hip_tiling(FlashAttentionConfig(block_q=128))
    assert m["block_q"] == {"requested": 128, "hip": 256} and m["num_stages"]["hip"] == HIP_TILING["num_stages"]
    q = torch.randn(1, 2, 32, 16)
    for bad in (FlashAttentionConfig(block_q=0), FlashAttentionConfig(block_k=-64),
                FlashAttentionConfig(num_warps=2.5), FlashAttentionConfig(num_stages=True)):
        with pytest.raises(ValueError):
            flash_attention_forward(q, q, q, config=bad)
    # any valid blocking gives the same result on the CPU recurrence
    a = flash_attention_forward(q, q, q, config=FlashAttentionConfig(block_q=8, block_k=16))
    b = flash_attention_forward(q, q, q)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_moe_inference_bookkeeping():
    """ch09.moe_inference (reference ch09/moe_inference.py:16-126): LRU order
    and eviction, hit/miss counters, the execution plan, and the per-expert
    routing statistics against a per-expert masked restatement."""
    from ch09 import ExpertCache, MoEInferenceConfig, MoEInferenceEngine
    c = ExpertCache(max_experts_in_memory=3, num_total_experts=6)
    for e in (0, 1, 2):
        assert c.add_expert(e, torch.full((2,), float(e))) is None
    assert c.get_expert(0) is not None          # refresh 0: LRU order 1, 2, 0
    assert c.add_expert(3, torch.zeros(2)) == 1
    assert c.add_expert(4, torch.zeros(2)) == 2
    assert c.get_cached_expert_ids() == [0, 3, 4]
    assert c.get_expert(1) is None and c.get_expert(5) is None
    assert c.get_cache_hit_rate() == pytest.approx(1 / 3)

    eng = MoEInferenceEngine(MoEInferenceConfig(num_experts=8, max_experts_in_gpu=2))
    eng.expert_cache.add_expert(5, torch.zeros(1))
    g = torch.Generator().manual_seed(3)
    idx = torch.randint(0, 8, (64, 2), generator=g)
    idx[0] = torch.tensor([5, 1])
    w = torch.rand(64, 2, generator=g)
    plan = eng.plan_expert_execution(idx)
    uniq = sorted(set(idx.flatten().tolist()))
    assert plan["total_unique"] == len(uniq)
    assert plan["in_cache"] == [5] and plan["need_load"] == [e for e in uniq if e != 5]
    eng.update_batch_stats(idx, w)
    eng.update_batch_stats(idx[:10], w[:10])
    for e in range(8):
        m1, m2 = idx == e, idx[:10] == e
        st = eng.expert_cache.stats[e]
        assert st.tokens_routed == int(m1.sum() + m2.sum())
        assert st.total_weight == pytest.approx(float(w[m1].double().sum() + w[:10][m2].double().sum()), rel=1e-6)
    met = eng.get_load_balance_metrics()
    loads = [eng.expert_cache.stats[e].tokens_routed for e in range(8)]
    assert met["max_load"] == max(loads) and met["min_load"] == min(loads)
    assert met["expected"] == pytest.approx(sum(loads) / 8)
    assert met["std_dev"] == pytest.approx(float(np.std(loads, ddof=1)), rel=1e-5)
    assert MoEInferenceEngine(MoEInferenceConfig()).get_load_balance_metrics() == \
        {"balance_ratio": 1.0, "max_load": 0, "min_load": 0}
