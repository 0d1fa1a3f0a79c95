"""CPU checks of the MoE mirror and oracle against the reference MoELayer
(tests/golden/moe.npz), plus the reference's own ch09 MoE contracts
(ch09/test_ch09.py:33-96) restated."""
from __future__ import annotations

import numpy as np
import torch

from conftest import load_golden
from oracle.linear import moe_layer, moe_route
from oracle.numerics import array_hash, seeded_normal


def _moe():
    from ch09 import MoEConfig, MoELayer
    cfg = MoEConfig(hidden_dim=256, expert_dim=512, num_experts=8, num_experts_per_tok=2)
    torch.manual_seed(9)
    return MoELayer(cfg)


def _experts(moe):
    return [(e.w1.weight.detach().numpy(), e.w2.weight.detach().numpy(), e.w3.weight.detach().numpy())
            for e in moe.experts]


def test_moe_mirror_matches_reference():
    g = load_golden("moe.npz")
    moe = _moe()
    for n, p in moe.named_parameters():
        assert array_hash(p.detach().numpy()) == str(g[f"hash_{n}"]), n
    x = torch.from_numpy(seeded_normal((2, 8, 256), 61))
    with torch.no_grad():
        np.testing.assert_allclose(moe(x).numpy(), g["y"], rtol=1e-5, atol=1e-6)
        w, idx, logits = moe.router(x.view(-1, 256))
    np.testing.assert_array_equal(idx.numpy(), g["router_idx"])
    np.testing.assert_allclose(w.numpy(), g["router_w"], rtol=1e-6)


def test_moe_oracle_pinned_to_reference():
    g = load_golden("moe.npz")
    moe = _moe()
    x = seeded_normal((2, 8, 256), 61).reshape(-1, 256)
    ref = moe_layer(x, moe.router.gate.weight.detach().numpy(), _experts(moe), 2)
    np.testing.assert_allclose(ref.reshape(2, 8, 256), g["y"], rtol=1e-4, atol=1e-6)
    w, idx = moe_route(g["router_logits"], 2)
    np.testing.assert_array_equal(idx, g["router_idx"])


def test_reference_ch09_moe_contracts():
    from ch09 import ExpertLayer, MoEConfig, MoELayer, Router, expert_load_balance_loss
    c = MoEConfig()
    assert (c.hidden_dim, c.expert_dim, c.num_experts, c.num_experts_per_tok) == (4096, 14336, 8, 2)
    cfg = MoEConfig(hidden_dim=64, num_experts=8, num_experts_per_tok=2)
    r = Router(cfg)
    w, idx, logits = r(torch.randn(10, 64))
    assert w.shape == (10, 2) and idx.shape == (10, 2) and logits.shape == (10, 8)
    torch.testing.assert_close(w.sum(-1), torch.ones(10))
    assert ExpertLayer(64, 256)(torch.randn(5, 64)).shape == (5, 64)
    moe = MoELayer(MoEConfig(hidden_dim=64, expert_dim=256, num_experts=4))
    assert moe(torch.randn(2, 10, 64)).shape == (2, 10, 64)
    loss = expert_load_balance_loss(torch.randn(32, 8), 8, 2)
    assert loss.ndim == 0 and loss.item() > 0
