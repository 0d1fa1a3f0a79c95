"""GPU parity of the fused SwiGLU projection (pli_gemm_swiglu) on every
route -- skinny (m <= 16), small-M MFMA (m <= 128), 128x128 MFMA tile,
phased 256x128 tile (m, n >= 256, k % 64 == 0), generic (fp32 / ragged) --
against the f64 oracle, and of the FFN / TP-MLP
modules that use it.  Bound: |err| <= tol * (|ref| + 1) (the outputs grow
like sqrt(K)); bf16 1e-2, fp16 4e-3, fp32 1e-4 as for pli_gemm."""
from __future__ import annotations


import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.linear import swiglu
from oracle.numerics import seeded_normal

pytestmark = pytest.mark.gpu
TDT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
TOL = {"fp32": 1e-4, "fp16": 4e-3, "bf16": 1e-2}

CASES = [  # m, n, k, dtype -> route
    (1, 4096, 4096, "bf16"),     # skinny, decode batch 1
    (5, 1376, 4096, "bf16"),     # skinny, n % 16 != 0
    (16, 4096, 1024, "fp16"),    # small-M MFMA
    (48, 2048, 512, "bf16"),     # small-M MFMA, NBG = 4
    (128, 1024, 4096, "bf16"),   # small-M MFMA, NBG = 8
    (200, 1000, 768, "bf16"),    # 128x128 tile, ragged m and n
    (1024, 2048, 1024, "fp16"),  # 128x128 tile (64 tiles of 256x128: too few for the phased tile)
    (2304, 1376, 256, "bf16"),   # phased 256x128 tile (>= 96 tiles), ragged n (10.75 column tiles)
    (2100, 1536, 640, "fp16"),   # phased tile, ragged m, 10 K-tiles
    (2048, 5632, 2048, "bf16"),  # phased tile, Llama-shaped MLP
    (3072, 1024, 64, "bf16"),    # phased tile, one K-tile
    (33, 100, 72, "bf16"),       # generic: n % 8 != 0
    (64, 96, 40, "fp32"),        # generic fp32
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "m{}n{}k{}_{}".format(*c))
def test_gemm_swiglu_vs_oracle(case):
    import pli_hip
    m, n, k, dt = case
    x = seeded_normal((m, k), 1, dt) * 0.5
    wg = seeded_normal((n, k), 2, dt) * k ** -0.5
    wu = seeded_normal((n, k), 3, dt) * k ** -0.5
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(TDT[dt])
    h = pli_hip.gemm_swiglu(d(x), d(wg), d(wu))
    ref = swiglu(x, wg, wu)
    got = h.float().cpu().numpy().astype(np.float64)
    bad = np.abs(got - ref) > TOL[dt] * (np.abs(ref) + 1)
    assert not bad.any(), f"{bad.sum()} beyond tol, max err {np.abs(got - ref).max():.3e}"


@pytest.mark.parametrize("split_k", [True, False])
@pytest.mark.parametrize("case", [(32, 1024, 4096, "bf16"), (100, 416, 8192, "bf16"),
                                  (200, 384, 4096, "fp16"), (256, 512, 2048, "bf16"),
                                  (64, 4096, 1024, "bf16")],
                         ids=lambda c: "m{}n{}k{}_{}".format(*c))
def test_gemm_swiglu_decode_batch_split_k(case, split_k):
    """Decode batches 16 < m <= 256: gate and up split-K planes through the
    wrapper's workspace + the silu(g) * u reduce, and the no-workspace routes."""
    import pli_hip
    m, n, k, dt = case
    x = seeded_normal((m, k), 4, dt) * 0.5
    wg = seeded_normal((n, k), 5, dt) * k ** -0.5
    wu = seeded_normal((n, k), 6, dt) * k ** -0.5
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(TDT[dt])
    h = pli_hip.gemm_swiglu(d(x), d(wg), d(wu), split_k=split_k)
    ref = swiglu(x, wg, wu)
    got = h.float().cpu().numpy().astype(np.float64)
    bad = np.abs(got - ref) > TOL[dt] * (np.abs(ref) + 1)
    assert not bad.any(), f"{bad.sum()} beyond tol, max err {np.abs(got - ref).max():.3e}"


@pytest.mark.parametrize("m", [64, 3072])
def test_gemm_swiglu_strided_halves_of_fused_weight(m):
    """FusedSwiGLUFFN passes the two row halves of one [2n, k] weight (m = 3072:
    the phased tile, 96 tiles)."""
    import pli_hip
    n, k = 1024, 256
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(2 * n, k, device="cuda", dtype=torch.bfloat16) * k ** -0.5
    h = pli_hip.gemm_swiglu(x, w[:n], w[n:])
    ref = swiglu(x.float().cpu().numpy(), w[:n].float().cpu().numpy(), w[n:].float().cpu().numpy())
    assert np.abs(h.float().cpu().numpy() - ref).max() <= 1e-2 * (np.abs(ref).max() + 1)


@pytest.mark.parametrize("name,seed", [("NaiveFFN", 5), ("SwiGLUFFN", 6), ("FusedSwiGLUFFN", 7)])
def test_ffn_modules_on_gpu_match_reference(name, seed):
    import ch01
    g = load_golden("ffn.npz")
    torch.manual_seed(seed)
    m = getattr(ch01, name)(256, 512).cuda()
    x = torch.from_numpy(seeded_normal((2, 16, 256), 51)).cuda()
    with torch.no_grad():
        np.testing.assert_allclose(m(x).cpu().numpy(), g[name], rtol=1e-3, atol=1e-3)


def test_tp_mlp_on_gpu_matches_reference_and_bf16_tracks():
    from ch09 import TensorParallelConfig, TensorParallelMLP
    g = load_golden("ffn.npz")
    torch.manual_seed(8)
    m = TensorParallelMLP(TensorParallelConfig(world_size=1, rank=0, hidden_dim=256,
                                               intermediate_dim=512))
    x = torch.from_numpy(seeded_normal((2, 16, 256), 51))
    with torch.no_grad():
        np.testing.assert_allclose(m.cuda()(x.cuda()).cpu().numpy(), g["TensorParallelMLP"],
                                   rtol=1e-3, atol=1e-3)
        yb = m.bfloat16()(x.cuda().bfloat16()).float().cpu().numpy()
    rel = np.linalg.norm(yb - g["TensorParallelMLP"]) / np.linalg.norm(g["TensorParallelMLP"])
    assert rel < 2e-2, rel


@pytest.mark.parametrize("m,n,k", [(2048, 5632, 2048), (4096, 1792, 4096), (2100, 1376, 640)])
def test_gemm_swiglu_w5_route_matches_phased(m, n, k):
    """gemm_w5's SwiGLU form (variant 3, the prefill default since round 4)
    against the phased 256 x 128 tile (variant 4): the same MFMA
    chains in k order and the same silu(g) * u in fp32, so bitwise equal;
    and sampled rows against the f64 oracle."""
    import pli_hip
    g = torch.Generator(device="cuda").manual_seed(m + n + k)
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16, generator=g)
    wg = torch.randn(n, k, device="cuda", dtype=torch.bfloat16, generator=g) * k ** -0.5
    wu = torch.randn(n, k, device="cuda", dtype=torch.bfloat16, generator=g) * k ** -0.5
    h3 = pli_hip.gemm_swiglu(x, wg, wu, variant=3)
    h4 = pli_hip.gemm_swiglu(x, wg, wu, variant=4)
    assert torch.equal(h3, h4), f"max diff {(h3.float() - h4.float()).abs().max().item():.3e}"
    rows = torch.randperm(m, generator=torch.Generator().manual_seed(5))[:24]
    ref = swiglu(x[rows].float().cpu().numpy(), wg.float().cpu().numpy(), wu.float().cpu().numpy())
    err = np.abs(h3[rows].float().cpu().numpy() - ref) / (np.abs(ref) + 1)
    assert err.max() <= TOL["bf16"], f"max rel err {err.max():.3e}"
