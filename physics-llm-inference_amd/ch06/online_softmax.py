"""Online softmax -- mirror of ``ch06/online_softmax.py``.

ROCm tensors run the HIP row kernels (``pli_softmax_rows``,
``pli_online_softmax_with_output``): one wave per row, single pass with the
(m, d) recurrence merged across lanes, fp32 statistics.  CPU tensors use the
closed forms in torch (the recurrence's fixed point), which equal the
reference's element-by-element Python loops up to rounding.
"""
from __future__ import annotations

import torch

import pli_hip


def standard_softmax(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    """max-subtracted softmax along ``dim`` (``:5-10``)."""
    if x.is_cuda and dim in (-1, x.dim() - 1):
        return pli_hip.softmax_rows(x)
    e = torch.exp(x - x.max(dim=dim, keepdim=True).values)
    return e / e.sum(dim=dim, keepdim=True)


def online_softmax(x: torch.Tensor) -> torch.Tensor:
    """Softmax over the last dim via the online (m, d) recurrence (``:13-25``)."""
    if x.is_cuda:
        return pli_hip.softmax_rows(x)
    m = x.max(dim=-1, keepdim=True).values
    e = torch.exp(x - m)
    return e / e.sum(dim=-1, keepdim=True)


def online_softmax_with_output(x: torch.Tensor, v: torch.Tensor):
    """(o, d) with o = softmax(x) . v and d = sum exp(x - max) (``:28-53``)."""
    if x.is_cuda:
        return pli_hip.online_softmax_with_output(x, v)
    m = x.max(dim=-1, keepdim=True).values
    e = torch.exp(x - m)
    d = e.sum(dim=-1)
    o = torch.einsum("...n,...nd->...d", e, v) / d.unsqueeze(-1)
    return o, d


def explain_online_softmax() -> str:
    return ("Online softmax keeps a running max m and denominator d; a new element x\n"
            "updates m' = max(m, x), d' = d e^{m-m'} + e^{x-m'}.  Partial states merge the\n"
            "same way, which is what lets one wave reduce a row in a single pass.")


def demonstrate_online_softmax():
    x = torch.tensor([1.0, 2.0, 3.0, 4.0, 5.0])
    return standard_softmax(x), online_softmax(x)


if __name__ == "__main__":
    # the chapter's demo (ch06/online_softmax.py:101-115)
    print(explain_online_softmax())
    print("\n" + "=" * 60 + "\nVerification\n" + "-" * 60)
    demonstrate_online_softmax()
    xs = torch.randn(4, 8, 64)
    print(f"\nBatch verification:\nMax difference: {(standard_softmax(xs) - online_softmax(xs)).abs().max().item():.2e}")
