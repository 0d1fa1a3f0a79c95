"""GPU parity of pli_rmsnorm (RMSNorm, optionally with the residual add
fused) against the f64 oracle.  Output tolerance: relative 2^-7 for 16-bit
storage (two roundings: the stored residual sum and the output), 1e-5 fp32;
the fused h output must equal the torch add bit for bit."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle.linear import rms_norm

pytestmark = pytest.mark.gpu
TDT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
TOL = {"fp32": 1e-5, "fp16": 2 ** -7, "bf16": 2 ** -7}


@pytest.mark.parametrize("rows,n,dt,res", [
    (8, 2048, "bf16", False),     # vector path, 1 chunk/thread
    (3, 4096, "fp16", True),      # residual fused, 2 chunks/thread
    (5, 5000, "bf16", True),      # 4 chunks/thread, ragged last chunk
    (4, 100, "bf16", False),      # n % 8 != 0: generic
    (2, 16384, "bf16", True),     # past the register-resident size: generic
    (6, 768, "fp32", True),       # fp32 generic
    (1, 2048, "bf16", True),      # decode batch 1
])
def test_rmsnorm_vs_oracle(rows, n, dt, res):
    import pli_hip
    g = torch.Generator(device="cuda").manual_seed(rows * n)
    x = torch.randn(rows, n, device="cuda", generator=g).to(TDT[dt])
    w = (1 + 0.1 * torch.randn(n, device="cuda", generator=g)).to(TDT[dt])
    r = torch.randn(rows, n, device="cuda", generator=g).to(TDT[dt]) if res else None
    out = pli_hip.rmsnorm(x, w, 1e-6, residual=r)
    if res:
        h, y = out
        assert torch.equal(h, x + r)
    else:
        y = out
    ref = rms_norm(x.double().cpu().numpy(), w.double().cpu().numpy(), 1e-6,
                   None if r is None else r.double().cpu().numpy())
    got = y.double().cpu().numpy()
    assert np.abs(got - ref).max() <= TOL[dt] * (np.abs(ref).max() + 1)


def test_rmsnorm_module_on_gpu_matches_reference_formula():
    from ch02 import RMSNorm
    m = RMSNorm(1024).cuda()
    with torch.no_grad():
        m.weight.copy_(torch.linspace(0.5, 1.5, 1024))
    x = torch.randn(4, 7, 1024, device="cuda")
    ref = x / torch.sqrt(torch.mean(x ** 2, dim=-1, keepdim=True) + 1e-6) * m.weight
    torch.testing.assert_close(m(x), ref, rtol=1e-5, atol=1e-5)
