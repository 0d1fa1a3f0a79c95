"""GPU tests of the ch01 / ch02 / ch05 mirrors that sit on the hot-path
kernels: the 3-D single-head attention wrappers, the
transformer block / model (ch01/transformer.py, which the reference's own
ch01 and ch02 tests import), naive generation, and the ch05 benchmark
harnesses (a15)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import attention as oatt
from oracle.numerics import seeded_normal

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B,S,d,dt", [(2, 16, 64, torch.float32), (3, 200, 128, torch.bfloat16),
                                      (1, 77, 64, torch.float16), (2, 130, 80, torch.float32)])
def test_3d_attention_wrappers_vs_oracle(B, S, d, dt):
    """ch01 naive_attention / causal_attention / SingleHeadAttention (3-D,
    ch01/attention.py:8-42) on the flash kernel with H = 1, against the f64
    single-head oracle."""
    from ch01 import SingleHeadAttention, causal_attention, naive_attention
    q, k, v = (seeded_normal((B, S, d), 60 + i) for i in range(3))
    tol = 1e-3 if dt == torch.float32 else 1e-2
    t = [torch.from_numpy(x).to(DEV).to(dt) for x in (q, k, v)]
    qr, kr, vr = (x.float().cpu().numpy() for x in t)  # the rounded inputs
    for fn, causal in ((naive_attention, False), (causal_attention, True)):
        out = fn(*t)
        assert out.dtype == dt and tuple(out.shape) == (B, S, d)
        ref = oatt.naive_attention_3d(qr, kr, vr, causal=causal)
        assert np.abs(out.float().cpu().numpy() - ref).max() <= tol, fn.__name__
    torch.manual_seed(0)
    sha = SingleHeadAttention(d, d).to(DEV)
    x = torch.from_numpy(seeded_normal((B, S, d), 70)).to(DEV)
    with torch.no_grad():
        y = sha(x).cpu()
        y_cpu = sha.cpu()(x.cpu())
    torch.testing.assert_close(y, y_cpu, rtol=2e-3, atol=2e-3)


def _seeded_model(dtype):
    from ch01 import TransformerModel
    torch.manual_seed(0)
    return TransformerModel(vocab_size=500, hidden_dim=256, num_layers=2, num_heads=8, num_kv_heads=2,
                            intermediate_dim=512).to(dtype).eval()


def test_transformer_model_gpu_matches_cpu_reference_math():
    """ch01.TransformerModel on the HIP kernels (pli_rmsnorm with the residual
    fused, GQA = 4 pli_gemm + causal flash, fused SwiGLU, lm_head pli_gemm) vs
    the same seeded model on the CPU path (the reference's exact math), fp32."""
    model = _seeded_model(torch.float32)
    ids = torch.randint(0, 500, (2, 40), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = model(ids)
        out = model.to(DEV)(ids.to(DEV)).cpu()
    assert out.shape == ref.shape == (2, 40, 500)
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3)
    block = model.layers[0]
    x = torch.randn(2, 40, 256, generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        yg = block(x.to(DEV), causal=False).cpu()
        yc = block.cpu()(x, causal=False)
    torch.testing.assert_close(yg, yc, rtol=2e-3, atol=2e-3)


def test_transformer_model_bf16_tracks_fp32():
    """bf16 model on the GPU stays within bf16 error of the fp32 CPU model
    (greedy next tokens agree on most positions)."""
    m32 = _seeded_model(torch.float32)
    m16 = _seeded_model(torch.float32).to(torch.bfloat16).to(DEV)
    ids = torch.randint(0, 500, (2, 64), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = m32(ids)
        out = m16(ids.to(DEV)).float().cpu()
    err = (out - ref).abs().max().item()
    assert err < 0.1 * ref.abs().max().item(), err
    agree = (out.argmax(-1) == ref.argmax(-1)).float().mean().item()
    assert agree > 0.9, agree


def test_naive_generate_on_gpu():
    """ch02.naive_generate over the HIP transformer: prompt kept, length
    right, and greedy-equivalent (top_k=1) tokens equal the CPU model's."""
    from ch02 import naive_generate
    model = _seeded_model(torch.float32)
    ids = torch.randint(0, 500, (1, 8), generator=torch.Generator().manual_seed(4))
    torch.manual_seed(5)
    cpu = naive_generate(model, ids, max_new_tokens=6, top_k=1)
    model = model.to(DEV)
    torch.manual_seed(5)
    gpu = naive_generate(model, ids.to(DEV), max_new_tokens=6, top_k=1).cpu()
    assert gpu.shape == (1, 14) and torch.equal(gpu[:, :8], ids)
    assert torch.equal(gpu, cpu)


def test_ch05_benchmarks_run_on_gpu():
    """ch05 benchmark_tensor_cores (MFMA bf16/fp16 vs fp32) and
    benchmark_triton_matmul (HIP tiled GEMM vs torch.matmul) return sane
    results; the 16-bit MFMA GEMM beats the fp32 one by a wide margin."""
    from ch05 import benchmark_tensor_cores, benchmark_triton_matmul, triton_matmul
    r = benchmark_tensor_cores(size=1024, warmup=3, iterations=10)
    assert r is not None and r.fp16_us > 0 and r.fp32_us > 0
    assert r.speedup > 1.5, r
    m = benchmark_triton_matmul(512, 512, 512, warmup=3, iterations=10)
    assert m.triton_us > 0 and m.torch_us > 0 and m.speedup > 0
    a = torch.randn(128, 256, device=DEV, dtype=torch.float16)
    b = torch.randn(256, 64, device=DEV, dtype=torch.float16)
    torch.testing.assert_close(triton_matmul(a, b), torch.matmul(a, b), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("m,n,k,blocks", [(64, 64, 64, (32, 32, 32)), (256, 256, 128, None),
                                           (128, 64, 256, None)])
def test_ch05_triton_matmul_reference_cases(m, n, k, blocks):
    """The reference's TestTritonMatmul cases (/root/reference/ch05/test_ch05.py:117-136),
    which skip forever there without Triton: 64^2 with 32-blocks, 256x128 @
    128x256 and the non-square 128x256 @ 256x64, fp16, against torch.matmul
    at the reference's rtol = atol = 1e-2 (the mirror runs the HIP GEMM)."""
    from ch05 import triton_matmul
    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    a = torch.randn(m, k, device=DEV, dtype=torch.float16, generator=g)
    b = torch.randn(k, n, device=DEV, dtype=torch.float16, generator=g)
    kw = {} if blocks is None else dict(block_m=blocks[0], block_n=blocks[1], block_k=blocks[2])
    out = triton_matmul(a, b, **kw)
    assert out.shape == (m, n) and out.dtype == torch.float16
    torch.testing.assert_close(out, torch.matmul(a, b), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("m,n,k,trans_b,bias", [(128, 128, 32, False, False), (200, 136, 68, False, True),
                                                (1, 300, 1024, True, True), (257, 129, 4, True, False),
                                                (512, 384, 1000, True, True), (96, 4, 12, False, False)])
def test_fp32_gemm_mfma_vs_f64(m, n, k, trans_b, bias):
    """pli_gemm at fp32 (v_mfma_f32_32x32x2_f32 tile, ragged M/N edges, both
    layouts, bias) against the f64 product of the same fp32 inputs."""
    import pli_hip
    a = seeded_normal((m, k), 81)
    b = seeded_normal((n, k) if trans_b else (k, n), 82)
    bi = seeded_normal((n,), 83) if bias else None
    ref = a.astype(np.float64) @ (b.T if trans_b else b).astype(np.float64)
    if bias:
        ref = ref + bi
    out = pli_hip.gemm(torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV), trans_b=trans_b,
                       bias=None if bi is None else torch.from_numpy(bi).to(DEV)).cpu().numpy()
    # fp32 accumulation of k products of N(0,1): error ~ k * 2^-24 * sqrt(k)
    assert np.abs(out - ref).max() <= 4e-6 * k + 1e-5


def test_fp32_gemm_unaligned_takes_valu_path():
    """K % 4 != 0 / odd leading dimension: the VALU fallback, same contract."""
    import pli_hip
    a = seeded_normal((70, 33), 84)
    b = seeded_normal((33, 45), 85)
    out = pli_hip.gemm(torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(out, a.astype(np.float64) @ b, rtol=0, atol=1e-4)


def test_naive_matmul_and_demo_2048():
    """ch05/tiled_matmul.cu main at its own size (2048^3 fp32): the naive
    contrast kernel and the MFMA tile kernel agree, both match f64 on sampled
    rows, and the tile kernel is many times faster."""
    from ch05 import benchmark_matmul_demo, naive_matmul, tiled_matmul
    a = torch.from_numpy(seeded_normal((100, 36), 86)).to(DEV)
    b = torch.from_numpy(seeded_normal((36, 70), 87)).to(DEV)
    ref = a.double().cpu() @ b.double().cpu()
    torch.testing.assert_close(naive_matmul(a, b).cpu().double(), ref, rtol=0, atol=1e-4)
    d = benchmark_matmul_demo(2048, warmup=2, iterations=5)
    # inputs in [0, 0.99]: sums ~500, fp32 ulp there 2^-15; different orders
    assert d["max_abs_diff"] < 0.05, d
    assert d["tiled"]["ms"] * 4 < d["naive"]["ms"], d
    g = torch.Generator(device="cpu").manual_seed(0)
    a2 = torch.randint(0, 100, (2048, 2048), generator=g).float() / 100
    b2 = torch.randint(0, 100, (2048, 2048), generator=g).float() / 100
    c = tiled_matmul(a2.to(DEV), b2.to(DEV)).cpu()
    rows = torch.tensor([0, 1, 777, 2047])
    ref2 = a2[rows].double() @ b2.double()
    assert (c[rows].double() - ref2).abs().max().item() < 0.02
