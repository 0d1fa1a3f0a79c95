"""CPU checks of the FFN / TP-MLP mirrors and the SwiGLU oracle against the
reference's own outputs (tests/golden/ffn.npz, made by make_golden.py)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.linear import swiglu_ffn
from oracle.numerics import array_hash, seeded_normal

HIDDEN, INTER = 256, 512


@pytest.fixture(scope="module")
def g():
    return load_golden("ffn.npz")


def _check_hashes(mod, name, g):
    for n, p in mod.named_parameters():
        assert array_hash(p.detach().numpy()) == str(g[f"{name}_hash_{n}"]), n


@pytest.mark.parametrize("name,seed", [("NaiveFFN", 5), ("SwiGLUFFN", 6), ("FusedSwiGLUFFN", 7)])
def test_ffn_mirrors_match_reference(g, name, seed):
    import ch01
    torch.manual_seed(seed)
    m = getattr(ch01, name)(HIDDEN, INTER)
    _check_hashes(m, name, g)
    x = torch.from_numpy(seeded_normal((2, 16, HIDDEN), 51))
    with torch.no_grad():
        np.testing.assert_allclose(m(x).numpy(), g[name], rtol=1e-5, atol=1e-5)


def test_tp_mlp_mirror_matches_reference(g):
    from ch09 import TensorParallelConfig, TensorParallelMLP
    torch.manual_seed(8)
    m = TensorParallelMLP(TensorParallelConfig(world_size=1, rank=0, hidden_dim=HIDDEN,
                                               intermediate_dim=INTER))
    _check_hashes(m, "TensorParallelMLP", g)
    x = torch.from_numpy(seeded_normal((2, 16, HIDDEN), 51))
    with torch.no_grad():
        np.testing.assert_allclose(m(x).numpy(), g["TensorParallelMLP"], rtol=1e-5, atol=1e-5)


def test_swiglu_oracle_pinned_to_reference(g):
    """The f64 SwiGLU oracle reproduces the reference SwiGLUFFN / TP MLP."""
    import ch01
    from ch09 import TensorParallelConfig, TensorParallelMLP
    x = seeded_normal((2, 16, HIDDEN), 51)
    torch.manual_seed(6)
    m = ch01.SwiGLUFFN(HIDDEN, INTER)
    ref = swiglu_ffn(x, m.gate_proj.weight.detach().numpy(), m.up_proj.weight.detach().numpy(),
                     m.down_proj.weight.detach().numpy())
    np.testing.assert_allclose(ref, g["SwiGLUFFN"], rtol=1e-4, atol=1e-5)
    torch.manual_seed(8)
    t = TensorParallelMLP(TensorParallelConfig(world_size=1, rank=0, hidden_dim=HIDDEN,
                                               intermediate_dim=INTER))
    ref = swiglu_ffn(x, t.gate_proj.weight.detach().numpy(), t.up_proj.weight.detach().numpy(),
                     t.down_proj.weight.detach().numpy())
    np.testing.assert_allclose(ref, g["TensorParallelMLP"], rtol=1e-4, atol=1e-5)


def test_fused_unfused_equivalence_contract():
    """ch01/test_ch01.py:110-128 restated: FusedSwiGLUFFN with the two
    weights concatenated equals SwiGLUFFN."""
    import ch01
    torch.manual_seed(0)
    u = ch01.SwiGLUFFN(64, 128)
    f = ch01.FusedSwiGLUFFN(64, 128)
    with torch.no_grad():
        f.gate_up_proj.weight.copy_(torch.cat([u.gate_proj.weight, u.up_proj.weight], 0))
        f.down_proj.weight.copy_(u.down_proj.weight)
        x = torch.randn(2, 8, 64)
        torch.testing.assert_close(f(x), u(x), rtol=1e-5, atol=1e-5)
