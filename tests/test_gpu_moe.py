"""GPU parity of the MoE path: pli_moe_route, pli_gemm_grouped (plain and
fused SwiGLU), pli_moe_combine and ch09.MoELayer, against the f64 oracle and
the reference's own layer output (moe.npz)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.linear import moe_route, swiglu
from oracle.numerics import seeded_normal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (37, 8, 2), (256, 16, 4), (5, 64, 8)])
def test_moe_route_vs_oracle(T, E, k):
    import pli_hip
    logits = torch.from_numpy(seeded_normal((T, E), T * E)).cuda()
    w, idx, pos, gather, offsets = pli_hip.moe_route(logits, k)
    rw, ridx = moe_route(logits.double().cpu().numpy(), k)
    np.testing.assert_array_equal(idx.cpu().numpy(), ridx)
    np.testing.assert_allclose(w.cpu().numpy(), rw, rtol=1e-5, atol=1e-6)
    off = offsets.cpu().numpy()
    counts = np.bincount(ridx.ravel(), minlength=E)
    np.testing.assert_array_equal(np.diff(off), counts)
    p, gth = pos.cpu().numpy(), gather.cpu().numpy()[:T * k]
    assert sorted(p.ravel().tolist()) == list(range(T * k))          # a permutation
    for t in range(T):
        for j in range(k):
            e = ridx[t, j]
            assert off[e] <= p[t, j] < off[e + 1] and gth[p[t, j]] == t


@pytest.mark.parametrize("variant", [None, 1, 2])
@pytest.mark.parametrize("T,E,k,H,I,dead", [
    (4, 8, 2, 256, 512, ()),         # decode sizes: weight-streaming grouped kernel
    (24, 8, 2, 256, 512, ()),        # 48 rows: the LDS-staged grouped kernel (default)
    (64, 8, 2, 512, 1024, ()),       # 16 rows / expert: LDS kernel (default) / phased 256-row tile (1)
    (300, 8, 2, 256, 256, ()),       # 600 rows: experts span several 128-row slabs
    (1200, 4, 2, 384, 640, ()),      # ~600 rows / expert = 3 slots each; ragged n on both GEMMs
    (600, 16, 1, 256, 512, (3, 7, 11)),  # experts with no rows: their slots / slabs are skipped
])
def test_grouped_gemm_and_combine_vs_oracle(T, E, k, H, I, dead, variant):
    import pli_hip
    x = torch.from_numpy(seeded_normal((T, H), 1, "bf16")).cuda().bfloat16()
    logits = torch.from_numpy(seeded_normal((T, E), 2)).cuda()
    for e in dead:
        logits[:, e] -= 100.0
    ws = [[torch.from_numpy(seeded_normal(s, 10 * e + i, "bf16") * s[1] ** -0.5).cuda().bfloat16()
           for i, s in enumerate(((I, H), (H, I), (I, H)))] for e in range(E)]
    w, idx, pos, gather, offsets = pli_hip.moe_route(logits, k)
    t1 = pli_hip.weight_table([e[0] for e in ws])
    t2 = pli_hip.weight_table([e[1] for e in ws])
    t3 = pli_hip.weight_table([e[2] for e in ws])
    h = pli_hip.gemm_grouped(x, gather, t1, offsets, T * k, I, H, H, wu_table=t3, variant=variant)
    y = pli_hip.gemm_grouped(h, None, t2, offsets, T * k, H, I, I, variant=variant)
    out = pli_hip.moe_combine(y, pos, w, T)
    # per-row check of the grouped SwiGLU against the oracle
    xn, gth = x.double().cpu().numpy(), gather.cpu().numpy()
    off = offsets.cpu().numpy()
    hn = h.double().cpu().numpy()
    for e in range(E):
        rows = range(off[e], off[e + 1])
        if not len(rows):
            continue
        ref = swiglu(xn[gth[list(rows)]], ws[e][0].double().cpu().numpy(), ws[e][2].double().cpu().numpy())
        assert np.abs(hn[list(rows)] - ref).max() <= 1e-2 * (np.abs(ref).max() + 1)
    # end to end vs the f64 layer with the same routing
    if dead:
        assert all(off[e] == off[e + 1] for e in dead)
    rw, ridx = moe_route(logits.double().cpu().numpy(), k)
    exp = np.zeros((T, H))
    for t in range(T):
        for j in range(k):
            e = ridx[t, j]
            hh = swiglu(xn[t:t + 1], ws[e][0].double().cpu().numpy(), ws[e][2].double().cpu().numpy())
            exp[t] += rw[t, j] * (hh @ ws[e][1].double().cpu().numpy().T)[0]
    got = out.double().cpu().numpy()
    assert np.abs(got - exp).max() <= 2e-2 * (np.abs(exp).max() + 1)


def test_moe_layer_gpu_matches_reference():
    from ch09 import MoEConfig, MoELayer
    g = load_golden("moe.npz")
    cfg = MoEConfig(hidden_dim=256, expert_dim=512, num_experts=8, num_experts_per_tok=2)
    torch.manual_seed(9)
    moe = MoELayer(cfg).cuda()
    x = torch.from_numpy(seeded_normal((2, 8, 256), 61)).cuda()
    with torch.no_grad():
        y32 = moe(x).cpu().numpy()                      # fp32: dense HIP path
        yb = moe.bfloat16()(x.bfloat16()).float().cpu().numpy()  # bf16: grouped path
    np.testing.assert_allclose(y32, g["y"], rtol=1e-3, atol=1e-4)
    rel = np.linalg.norm(yb - g["y"]) / np.linalg.norm(g["y"])
    assert rel < 2e-2, rel
