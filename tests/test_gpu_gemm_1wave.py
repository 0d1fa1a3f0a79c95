"""gemm_w5 (csrc/gemm_w5.hip; GEMM variant 41, the default route for large
bf16 / fp16 shapes since round 3: K staged 64 deep) and gemm_w4v
(csrc/gemm_w4v.hip; variant 40, K 32 deep) against the f64 product of the same rounded
inputs (reference ch03/gemm_benchmark.py:35-49 times torch.mm on these shapes;
ch09/tensor_parallel.py:66-68 is the NT F.linear form) and bitwise against
the 256-tile kernel (variant 2), which runs the same MFMA chains in the same
k order.  Ragged M / N (rows past the edge re-read the last row and are never
stored), K a multiple of 32 but not of 64, bias, fp16 and strided leading
dimensions are covered."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(m, n, k, tb, dt, seed, lda=None, ldb=None):
    g = torch.Generator(device=DEV).manual_seed(seed)
    a = torch.randn(m, lda or k, device=DEV, dtype=dt, generator=g)[:, :k]
    if tb:
        b = torch.randn(n, ldb or k, device=DEV, dtype=dt, generator=g)[:, :k]
    else:
        b = torch.randn(k, ldb or n, device=DEV, dtype=dt, generator=g)[:, :n]
    return a, b


def _ref(a, b, tb, bias=None):
    r = a.double() @ (b.double().t() if tb else b.double())
    return r + bias.double() if bias is not None else r


@pytest.mark.parametrize("variant", [41, 43, 40])
@pytest.mark.parametrize("tb", [True, False], ids=["nt", "nn"])
@pytest.mark.parametrize("m,n,k", [(512, 512, 64), (256, 256, 32), (300, 520, 96), (1000, 776, 4096),
                                   (777, 1032, 160), (2048, 8192, 1024), (4096, 4096, 4096), (264, 392, 128)])
def test_w4v_vs_f64_and_v2(m, n, k, tb, variant):
    import pli_hip
    if variant in (41, 43) and k % 64:
        pytest.skip("gemm_w5 takes K % 64 == 0")
    if variant == 43 and (m % 256 or n % 256):
        pytest.skip("the persistent gemm_w5 takes M, N multiples of 256")
    a, b = _inputs(m, n, k, tb, torch.bfloat16, m * 7 + n * 3 + k)
    o = pli_hip.gemm(a, b, trans_b=tb, variant=variant)
    ref = _ref(a, b, tb)
    err = ((o.double() - ref).abs() / (ref.abs() + 1)).max().item()
    assert err <= 1e-2, f"v{variant} {m}x{n}x{k} tb={tb}: max rel err {err:.3e}"
    if k % 64 == 0 and m >= 512 and n >= 512:
        assert torch.equal(o, pli_hip.gemm(a, b, trans_b=tb, variant=2)), f"v{variant} != gemm_256 (same chain order)"


@pytest.mark.parametrize("variant", [41, 43, 40])
@pytest.mark.parametrize("tb", [True, False], ids=["nt", "nn"])
def test_w4v_bias_fp16_and_default_route(tb, variant):
    import pli_hip
    a, b = _inputs(1024, 1024, 512, tb, torch.float16, 5)
    bias = torch.randn(1024, device=DEV, dtype=torch.float16)
    o = pli_hip.gemm(a, b, trans_b=tb, bias=bias, variant=variant)
    ref = _ref(a, b, tb, bias)
    err = ((o.double() - ref).abs() / (ref.abs() + 1)).max().item()
    assert err <= 4e-3, f"fp16 + bias tb={tb}: max rel err {err:.3e}"
    # the default route takes gemm_w5 (persistent: M, N multiples of 256,
    # K >= 128) at this size (128+ tiles of 256^2); every variant here runs
    # the same MFMA chains, so all agree bitwise
    a, b = _inputs(4096, 2048, 1024, tb, torch.bfloat16, 6)
    assert torch.equal(pli_hip.gemm(a, b, trans_b=tb), pli_hip.gemm(a, b, trans_b=tb, variant=variant))


@pytest.mark.parametrize("variant", [41, 40])
@pytest.mark.parametrize("tb", [True, False], ids=["nt", "nn"])
def test_w4v_strided_leading_dims(tb, variant):
    import pli_hip
    a, b = _inputs(600, 520, 256, tb, torch.bfloat16, 9, lda=384, ldb=392 if tb else 528)
    assert a.stride(0) == 384
    o = torch.empty(600, 536, device=DEV, dtype=torch.bfloat16)[:, :520]
    pli_hip.gemm(a, b, trans_b=tb, out=o, variant=variant)
    ref = _ref(a, b, tb)
    err = ((o.double() - ref).abs() / (ref.abs() + 1)).max().item()
    assert err <= 1e-2, f"strided tb={tb}: max rel err {err:.3e}"


@pytest.mark.parametrize("tb", [True, False], ids=["nt", "nn"])
@pytest.mark.parametrize("m,n,k", [(8192, 8192, 1024), (16384, 4096, 64), (16384, 4096, 128), (4608, 4096, 192),
                                   (8192, 4096, 8192)])
def test_w5_persistent_walks_vs_f64(m, n, k, tb):
    """Variant 43 with more tiles than CUs (every workgroup walks several
    tiles, the K stream crossing tile seams; K = 128 is the two-step
    minimum, K = 64 takes the one-tile form): sampled rows vs f64, and
    bitwise against the one-tile form (41)."""
    import pli_hip
    a, b = _inputs(m, n, k, tb, torch.bfloat16, m + n + k)
    o = pli_hip.gemm(a, b, trans_b=tb, variant=43)
    assert torch.equal(o, pli_hip.gemm(a, b, trans_b=tb, variant=41))
    rows = torch.randperm(m, generator=torch.Generator().manual_seed(1))[:48].to(DEV)
    ref = a[rows].double() @ (b.double().t() if tb else b.double())
    err = ((o[rows].double() - ref).abs() / (ref.abs() + 1)).max().item()
    assert err <= 1e-2, f"{m}x{n}x{k} tb={tb}: max rel err {err:.3e}"


def test_w5_f32out_persistent_deep_k():
    """The fp32-output form (RowParallelLinear(reduce_dtype=torch.float32))
    on its persistent walk at K = 8192 (two tiles per workgroup): sampled
    rows against f64 -- unrounded partials: fp32 accumulation error only,
    well under the 2^-9 of a bf16 output."""
    import pli_hip
    a, b = _inputs(8192, 4096, 8192, True, torch.bfloat16, 11)
    o = pli_hip.gemm_f32out(a, b)
    assert o.dtype == torch.float32
    rows = torch.randperm(8192, generator=torch.Generator().manual_seed(2))[:48].to(DEV)
    ref = a[rows].double() @ b.double().t()
    err = ((o[rows].double() - ref).abs() / (ref.abs() + 1)).max().item()
    assert err <= 5e-4, f"f32out K=8192: max rel err {err:.3e}"  # fp32 sums of 8192 products; bf16 output alone is 2^-9
    # bitwise: the bf16-output default route rounds the same accumulators
    assert torch.equal(o.to(torch.bfloat16), pli_hip.gemm(a, b, trans_b=True))
