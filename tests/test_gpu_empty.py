"""Empty and zero-length operands through the HIP entry points (include/pli.h:
"an operand with zero elements may be NULL"): torch gives empty tensors a NULL
data_ptr, and the reference's ops -- torch.mm / F.linear / torch.mv / softmax /
naive_attention (ch06/attention_memory.py:19-33) -- return empty results for
empty outputs and zeros (or the bias) for empty reductions.  Each case is
checked against the same torch op on the same (empty) inputs."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def naive(q, k, v, causal=False):
    s = (q.float() @ k.float().transpose(-1, -2)) * q.shape[-1] ** -0.5
    if causal and s.numel():
        nq, nk = s.shape[-2:]
        s = s.masked_fill(torch.ones(nq, nk, dtype=torch.bool, device=s.device).triu(nk - nq + 1), float("-inf"))
    return (torch.softmax(s, -1) @ v.float()).to(q.dtype)


@pytest.mark.parametrize("dtype", (torch.bfloat16, torch.float16, torch.float32))
@pytest.mark.parametrize("shape", [(0, 4, 16, 16, 64), (2, 4, 0, 16, 64), (2, 4, 16, 0, 64), (1, 2, 5, 0, 128),
                                   (0, 4, 0, 0, 128)], ids=lambda s: "b{}h{}q{}k{}d{}".format(*s))
def test_flash_empty(shape, dtype):
    import pli_hip
    B, H, Nq, Nk, D = shape
    q = torch.randn(B, H, Nq, D, device=DEV, dtype=dtype)
    k = torch.randn(B, H, Nk, D, device=DEV, dtype=dtype)
    v = torch.randn(B, H, Nk, D, device=DEV, dtype=dtype)
    for causal in (False, True):
        out = pli_hip.flash_attn_fwd(q, k, v, causal=causal and Nq <= Nk)
        ref = naive(q, k, v)
        assert out.shape == ref.shape
        assert torch.equal(out, torch.zeros_like(ref)) if Nk == 0 else out.numel() == 0


def test_decode_empty_cache_and_batch():
    import pli_hip
    q = torch.randn(2, 1, 8, 128, device=DEV, dtype=torch.bfloat16)
    kc = torch.randn(2, 64, 2, 128, device=DEV, dtype=torch.bfloat16)
    out = pli_hip.attn_decode(q, kc, kc.clone(), 0, causal=False)
    assert torch.equal(out, torch.zeros_like(q))
    out = pli_hip.attn_decode(q[:0], kc[:0], kc[:0].clone(), 0)
    assert out.shape == (0, 1, 8, 128)
    pos = torch.zeros(1, device=DEV, dtype=torch.int32)
    before = kc.clone()
    pli_hip.kv_append(kc[:, :0], kc[:, :0].clone(), kc, kc.clone(), pos)  # nothing to append
    assert torch.equal(kc, before)


@pytest.mark.parametrize("dtype", (torch.bfloat16, torch.float16, torch.float32))
@pytest.mark.parametrize("mnk", [(0, 64, 64), (64, 0, 64), (64, 64, 0), (0, 0, 0), (3, 40, 0)])
def test_gemm_empty(mnk, dtype):
    import pli_hip
    m, n, k = mnk
    a = torch.randn(m, k, device=DEV, dtype=dtype)
    b_nn = torch.randn(k, n, device=DEV, dtype=dtype)
    b_nt = torch.randn(n, k, device=DEV, dtype=dtype)
    bias = torch.randn(n, device=DEV, dtype=dtype)
    assert torch.equal(pli_hip.gemm(a, b_nn), torch.mm(a, b_nn))
    assert torch.equal(pli_hip.gemm(a, b_nt, trans_b=True), F.linear(a, b_nt))
    assert torch.equal(pli_hip.gemm(a, b_nt, trans_b=True, bias=bias), F.linear(a, b_nt, bias))
    if dtype != torch.float32:
        assert torch.equal(pli_hip.gemm_f32out(a, b_nt), F.linear(a.float(), b_nt.float()))
        h = pli_hip.gemm_swiglu(a, b_nt, b_nt.clone())
        assert torch.equal(h, (F.silu(F.linear(a.float(), b_nt.float())) * F.linear(a.float(), b_nt.float())).to(dtype))
    else:
        assert torch.equal(pli_hip.gemm_naive(a, b_nn), torch.mm(a, b_nn))


@pytest.mark.parametrize("dtype", (torch.bfloat16, torch.float32))
@pytest.mark.parametrize("mk", [(0, 4096), (4096, 0), (0, 0)])
def test_gemv_empty(mk, dtype):
    import pli_hip
    m, k = mk
    w = torch.randn(m, k, device=DEV, dtype=dtype)
    x = torch.randn(k, device=DEV, dtype=dtype)
    out = torch.full((m,), 7.0, device=DEV, dtype=dtype)  # K == 0 must overwrite it with zeros
    assert torch.equal(pli_hip.gemv(w, x, out=out), torch.mv(w, x))


def test_rows_empty():
    import pli_hip
    x = torch.randn(0, 512, device=DEV, dtype=torch.bfloat16)
    wt = torch.randn(512, device=DEV, dtype=torch.bfloat16)
    assert pli_hip.rmsnorm(x, wt).shape == (0, 512)
    h, y = pli_hip.rmsnorm(x, wt, residual=x.clone())
    assert h.shape == y.shape == (0, 512)
    for shape in ((0, 300), (6, 0)):
        z = torch.randn(*shape, device=DEV)
        assert torch.equal(pli_hip.softmax_rows(z), torch.softmax(z, -1))


def test_moe_no_tokens():
    import pli_hip
    logits = torch.randn(0, 8, device=DEV, dtype=torch.bfloat16)
    weights, idx, pos, gather, offsets = pli_hip.moe_route(logits, 2)
    assert weights.shape == (0, 2) and torch.equal(offsets.cpu(), torch.zeros(9, dtype=torch.int32))
    y = torch.randn(4, 64, device=DEV, dtype=torch.bfloat16)
    assert pli_hip.moe_combine(y, pos, weights, 0).shape == (0, 64)
