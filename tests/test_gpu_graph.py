"""GPU checks of graph-replayable decode: pli_kv_append, pli_attn_decode_dev,
ch08.DecodeStepGraph over ch02.CachedTransformerModel, and the reference's
CUDAGraphRunner API (ch08/cuda_graph.py:18-82)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_kv_append_matches_slice_assignment():
    import pli_hip
    B, S, Hkv, D, T = 3, 64, 4, 128, 5
    kc = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    ref_k, ref_v = kc.clone(), vc.clone()
    kn = torch.randn(B, T, Hkv, D, device="cuda", dtype=torch.bfloat16)
    vn = torch.randn_like(kn)
    pos = torch.tensor([17], device="cuda", dtype=torch.int32)
    pli_hip.kv_append(kn, vn, kc, vc, pos)
    ref_k[:, 17:22], ref_v[:, 17:22] = kn, vn
    assert torch.equal(kc, ref_k) and torch.equal(vc, ref_v)
    pos.fill_(S - 2)  # rows past the capacity are dropped, not written out of bounds
    pli_hip.kv_append(kn, vn, kc, vc, pos)
    ref_k[:, S - 2:], ref_v[:, S - 2:] = kn[:, :2], vn[:, :2]
    assert torch.equal(kc, ref_k) and torch.equal(vc, ref_v)


@pytest.mark.parametrize("n,add", [(1, 0), (300, 1), (4095, 1), (2000, 3)])
def test_attn_decode_dev_equals_host_length(n, add):
    import pli_hip
    B, H, Hkv, D, S = 2, 32, 8, 128, 4096
    Sq = add if add else 1
    q = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16)
    kc = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    n_dev = torch.tensor([n], device="cuda", dtype=torch.int32)
    got = pli_hip.attn_decode_dev(q, kc, vc, n_dev, n_kv_add=add, causal=Sq > 1)
    ref = pli_hip.attn_decode(q, kc, vc, min(n + add, S), causal=Sq > 1)
    assert (got.float() - ref.float()).abs().max().item() <= 2 ** -7


@pytest.mark.parametrize("B,S", [(1, 1), (2, 1), (4, 4), (16, 1), (3, 5),
                                 (17, 1), (32, 1), (8, 4), (5, 5), (64, 1), (3, 40), (128, 1)])
def test_qkv_into_cache_matches_separate_projections(B, S):
    """pli_gemm_multi_nt: q plus k/v rows written into the caches at pos ==
    three pli_gemm calls + pli_kv_append; rows past the capacity dropped.
    Up to 16 rows the skinny kernel, 17-128 the small-M MFMA kernel."""
    import pli_hip
    torch.manual_seed(B * 10 + S)
    hidden, H, Hkv, D, S_max = 1024, 16, 4, 64, 40
    x = torch.randn(B, S, hidden, device="cuda", dtype=torch.bfloat16)
    wq = torch.randn(H * D, hidden, device="cuda", dtype=torch.bfloat16) * 0.03
    wk = torch.randn(Hkv * D, hidden, device="cuda", dtype=torch.bfloat16) * 0.03
    wv = torch.randn(Hkv * D, hidden, device="cuda", dtype=torch.bfloat16) * 0.03
    for p0 in (7, S_max - 2):
        kc = torch.randn(B, S_max, Hkv, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        rk, rv = kc.clone(), vc.clone()
        pos = torch.tensor([p0], device="cuda", dtype=torch.int32)
        q = torch.empty(B, S, H * D, device="cuda", dtype=torch.bfloat16)
        pli_hip.qkv_into_cache(x, wq, wk, wv, q, kc, vc, pos)
        x2 = x.reshape(B * S, hidden)
        ref_q = pli_hip.gemm(x2, wq, trans_b=True).view(B, S, -1)
        kn = pli_hip.gemm(x2, wk, trans_b=True).view(B, S, Hkv, D)
        vn = pli_hip.gemm(x2, wv, trans_b=True).view(B, S, Hkv, D)
        pli_hip.kv_append(kn, vn, rk, rv, pos)
        tol = 2 ** -7
        assert (q.float() - ref_q.float()).abs().max().item() <= tol * ref_q.float().abs().max().item()
        assert (kc.float() - rk.float()).abs().max().item() <= tol * rk.float().abs().max().item()
        assert (vc.float() - rv.float()).abs().max().item() <= tol * rv.float().abs().max().item()
        n_in = min(S, S_max - p0)  # untouched rows stay bitwise
        assert torch.equal(kc[:, :p0], rk[:, :p0]) and torch.equal(vc[:, p0 + n_in:], rv[:, p0 + n_in:])
        fp = (x2.float() @ wk.float().t()).view(B, S, Hkv, D)[:, :n_in]
        assert (kc[:, p0:p0 + n_in].float() - fp).abs().max().item() <= 2 ** -6 * fp.abs().max().item()


def _model():
    from ch02 import CachedTransformerModel
    torch.manual_seed(0)
    return CachedTransformerModel(1000, 512, 2, 8, 2, 1024).cuda().bfloat16().eval()


@pytest.mark.parametrize("B", [2, 24])
def test_decode_step_graph_replays_eager_steps(B):
    """Greedy decode: graph replay == eager steps over the same device-length
    kernels (bitwise), and tracks the host-length eager path (batch 24: q/k/v
    and the cache append in one small-M launch)."""
    from ch08 import DecodeStepGraph
    model = _model()
    P, N = 24, 12
    ids = torch.randint(0, 1000, (B, P), device="cuda")
    with torch.no_grad():
        # eager, device-length caches
        caches = model.create_caches(B, 64, torch.device("cuda"), torch.bfloat16, device_pos=True)
        lg = model(ids, caches)
        eager, tok = [], lg[:, -1:].argmax(-1)
        for _ in range(N):
            lg = model(tok, caches, start_pos=caches[0].seq_len)
            eager.append(lg.float().clone())
            tok = lg[:, -1:].argmax(-1)
        # host-length caches (pli_attn_decode with a host n_kv)
        hc = model.create_caches(B, 64, torch.device("cuda"), torch.bfloat16)
        lg = model(ids, hc)
        host, tok = [], lg[:, -1:].argmax(-1)
        for _ in range(N):
            lg = model(tok, hc, start_pos=hc[0].seq_len)
            host.append(lg.float().clone())
            tok = lg[:, -1:].argmax(-1)
        # graph
        g = DecodeStepGraph(model, B, 64, torch.bfloat16)
        lg = g.prefill(ids)
        tok = lg[:, -1:].argmax(-1)
        for i in range(N):
            lg = g.step(tok)
            assert torch.equal(lg.float(), eager[i]), f"step {i}"
            rel = (lg.float() - host[i]).norm() / host[i].norm()
            assert rel < 1e-2, (i, float(rel))
            tok = lg[:, -1:].argmax(-1)
    assert g.seq_len == P + N and int(g.pos.item()) == P + N
    assert all(c.seq_len == P + N for c in g.caches)


def test_cuda_graph_runner_api():
    from ch08 import CUDAGraphRunner, GraphConfig
    w = torch.randn(64, 64, device="cuda", dtype=torch.float16)
    runner = CUDAGraphRunner(GraphConfig(batch_sizes=[1, 4]), model_fn=lambda x: torch.relu(x @ w))
    for b in (1, 4):
        assert runner.capture_graph(b, (64,))
    x = torch.randn(4, 64, device="cuda", dtype=torch.float16)
    out = runner.run_graph(4, x)
    torch.testing.assert_close(out, torch.relu(x @ w))
    assert runner.run_graph(2, x[:2]) is None
    assert runner.has_graph(1) and sorted(runner.get_captured_batch_sizes()) == [1, 4]


@pytest.mark.parametrize("M", [1, 3])
def test_rms_gemm_matches_norm_then_gemm(M):
    """pli_rms_gemm_nt == pli_rmsnorm (+ residual) followed by the unfused
    projection: bitwise at one row (same reduction and dot orders), within
    bf16 rounding at more rows (the unfused GEMM is then the MFMA small-M
    kernel)."""
    import pli_hip
    torch.manual_seed(M)
    hd, N, I = 2048, 1536, 2816
    a = torch.randn(M, hd, device="cuda", dtype=torch.bfloat16)
    res = torch.randn(M, hd, device="cuda", dtype=torch.bfloat16)
    g = (1 + 0.1 * torch.randn(hd, device="cuda")).bfloat16()
    w = torch.randn(N, hd, device="cuda", dtype=torch.bfloat16) * hd ** -0.5
    wg = torch.randn(I, hd, device="cuda", dtype=torch.bfloat16) * hd ** -0.5
    wu = torch.randn(I, hd, device="cuda", dtype=torch.bfloat16) * hd ** -0.5
    h_ref, y = pli_hip.rmsnorm(a, g, 1e-6, residual=res)
    h = torch.empty_like(a)

    def same(x, ref):
        if M == 1:
            assert torch.equal(x, ref)
        else:
            assert (x.float() - ref.float()).abs().max().item() <= 2 ** -7 * (ref.float().abs().max().item() + 1)

    out = pli_hip.rms_linear(a, g, 1e-6, w, residual=res, h_out=h)
    assert torch.equal(h, h_ref)
    same(out, pli_hip.gemm(y, w, trans_b=True))
    same(pli_hip.rms_swiglu(a, g, 1e-6, wg, wu, residual=res), pli_hip.gemm_swiglu(y, wg, wu))
    # no residual: h_out untouched, y = rmsnorm(a)
    y0 = pli_hip.rmsnorm(a, g, 1e-6)
    same(pli_hip.rms_linear(a, g, 1e-6, w), pli_hip.gemm(y0, w, trans_b=True))
    # q/k/v into the caches at the device position
    B, S = (M, 1)
    H, Hkv, D, S_max = 16, 4, 64, 24
    wq = torch.randn(H * D, hd, device="cuda", dtype=torch.bfloat16) * hd ** -0.5
    wk = torch.randn(Hkv * D, hd, device="cuda", dtype=torch.bfloat16) * hd ** -0.5
    wv = torch.randn(Hkv * D, hd, device="cuda", dtype=torch.bfloat16) * hd ** -0.5
    kc = torch.zeros(B, S_max, Hkv, D, device="cuda", dtype=torch.bfloat16)
    vc, kr, vr = torch.zeros_like(kc), torch.zeros_like(kc), torch.zeros_like(kc)
    pos = torch.tensor([5], device="cuda", dtype=torch.int32)
    q = torch.empty(B, S, H * D, device="cuda", dtype=torch.bfloat16)
    qr = torch.empty_like(q)
    pli_hip.rms_qkv_into_cache(a.view(B, S, hd), g, 1e-6, wq, wk, wv, q, kc, vc, pos,
                               residual=res.view(B, S, hd))
    pli_hip.qkv_into_cache(y.view(B, S, hd), wq, wk, wv, qr, kr, vr, pos)
    assert torch.equal(q, qr) and torch.equal(kc, kr) and torch.equal(vc, vr)


@pytest.mark.parametrize("B", [1, 2])
def test_fused_decode_step_matches_unfused(B):
    """The model's fused decode path (5 launches per layer) against the
    unfused launches over the same caches: bitwise at batch 1, close at 2."""
    import ch02.cached_generation as cg
    model = _model()
    ids = torch.randint(0, 1000, (B, 20), device="cuda")
    outs = {}
    try:
        for fused in (True, False):
            cg.FUSED_DECODE = fused
            with torch.no_grad():
                caches = model.create_caches(B, 48, torch.device("cuda"), torch.bfloat16, device_pos=True)
                lg = model(ids, caches)
                tok = lg[:, -1:].argmax(-1)
                steps = []
                for _ in range(6):
                    lg = model(tok, caches, start_pos=caches[0].seq_len)
                    steps.append(lg.float().clone())
                    tok = lg[:, -1:].argmax(-1)
            outs[fused] = (steps, caches[0].k.clone(), int(caches[0].pos.item()))
    finally:
        cg.FUSED_DECODE = True
    (sf, kf, pf), (su, ku, pu) = outs[True], outs[False]
    assert pf == pu == 26
    for a, b in zip(sf, su):
        if B == 1:
            assert torch.equal(a, b)
        else:
            assert ((a - b).norm() / b.norm()).item() < 1e-2
    if B == 1:
        assert torch.equal(kf, ku)


@pytest.mark.parametrize("B", [1, 8])
@pytest.mark.parametrize("fused", [True, False])
def test_device_pos_cache_overflow_raises(B, fused):
    """A device-length cache that would overrun max_seq_len raises (the
    kernels clamp to the capacity and would otherwise return wrong logits
    silently; the reference raises on its slice-assignment mismatch)."""
    import ch02.cached_generation as cg
    from ch02 import CachedTransformerModel
    torch.manual_seed(0)
    model = CachedTransformerModel(1000, 256, 2, 4, 2, 512).cuda().bfloat16().eval()
    cg.FUSED_DECODE = fused
    try:
        with torch.no_grad():
            caches = model.create_caches(B, 12, torch.device("cuda"), torch.bfloat16, device_pos=True)
            ids = torch.randint(0, 1000, (B, 10), device="cuda")
            model(ids, caches)
            tok = torch.randint(0, 1000, (B, 1), device="cuda")
            model(tok, caches, start_pos=10)
            model(tok, caches, start_pos=11)           # fills the cache exactly
            with pytest.raises(RuntimeError, match="overflow"):
                model(tok, caches, start_pos=12)
            with pytest.raises(RuntimeError, match="overflow"):
                model(torch.randint(0, 1000, (B, 13), device="cuda"),
                      model.create_caches(B, 12, torch.device("cuda"), torch.bfloat16, device_pos=True))
    finally:
        cg.FUSED_DECODE = True
