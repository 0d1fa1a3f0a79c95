"""The synchronous debug mode on the device (include/pli.h
pli_debug_sync): with it on, every launch is synchronised and checked, the
results and routes are the same as without it."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_debug_sync_same_results_and_routes():
    import pli_hip
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(1, 4, 512, 128, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    a = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(512, 384, device="cuda", dtype=torch.bfloat16, generator=g)
    ref_o = pli_hip.flash_attn_fwd(q, k, v)
    route_o = pli_hip.last_route()
    ref_c = pli_hip.gemm(a, b)
    route_c = pli_hip.last_route()
    torch.cuda.synchronize()
    prev = pli_hip.debug_sync(1)
    try:
        o = pli_hip.flash_attn_fwd(q, k, v)
        assert pli_hip.last_route() == route_o == "attn_fwd_v13"
        c = pli_hip.gemm(a, b)
        assert pli_hip.last_route() == route_c
    finally:
        pli_hip.debug_sync(int(prev))
    assert torch.equal(o, ref_o) and torch.equal(c, ref_c)
