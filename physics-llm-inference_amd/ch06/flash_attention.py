"""FlashAttention forward -- MI355X mirror of ``ch06/flash_attention.py``.

``flash_attention_forward(q, k, v, scale=None, config=None)`` keeps the
reference signature and return contract (a NEW tensor shaped like ``q`` in
``q.dtype``; inputs are never written).  Device dispatch:

* ROCm tensors -> ONE launch of the fused HIP kernel ``pli_flash_attn_fwd``
  (csrc/flash_attn.hip) instead of the reference's Python double loop
  (``ch06/flash_attention.py:38-68``, ~12 torch launches per tile pair).
  There is no fallback: a missing library raises ``pli_hip.PliError``.
* CPU tensors -> the same online-softmax tile recurrence in torch CPU ops
  (fp32 statistics), so CPU callers keep working.

``FlashAttentionConfig`` keeps its four fields (``:6-11``).  They are Triton
launch knobs in the reference's design notes; on MI355X each one maps to a
fixed property of the default HIP kernel, attn_fwd_v13 (``hip_tiling``
returns the mapping): ``block_q`` -> 256 query rows per workgroup (4 waves x
64 rows, one wave per SIMD, four 16-row q-blocks per wave on the 16x16x32
MFMA), ``block_k`` -> 64-key K/V tiles, ``num_warps`` -> 4 wave64s per
workgroup, ``num_stages`` -> a 5-slot LDS ring with K/V DMA'd two tiles
ahead (causal runs the same program with the mask, attn_fwd_v13c, at any
diagonal offset; fp16 on
the f16 MFMA; D = 64 on half-width images; key counts that are not a multiple
of 64 on the ragged form, attn_fwd_v13r; Nk <= 64 and other head dims take
attn_fwd_v12 / v10 / v7; since round 6 non-causal D = 64 shapes that fill
the chip run attn_fwd_pp64 -- 512 rows per workgroup, 8 waves of 64, two
per SIMD in ping-pong).  The GPU path ignores the requested values (results do not
depend on the blocking; the kernel's tiles are set by the MFMA / LDS
mapping); the CPU recurrence uses ``block_q``/``block_k`` as the reference
does.  Non-positive or non-integer fields are rejected on both paths.  Softmax statistics are fp32 on both paths (the reference keeps
them in ``q.dtype``, ``:32-33``; that only adds rounding).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

import pli_hip


@dataclass
class FlashAttentionConfig:
    block_q: int = 64
    block_k: int = 64
    num_warps: int = 4
    num_stages: int = 2


# what each FlashAttentionConfig knob means on the HIP path: bf16 and fp16,
# D = 128 and 64, causal or not, any Nk > 64 (ragged Nk included) run the
# generated attn_fwd_v13 family (v13 / v13c / v13h / v13hc / v13r / v13rc /
# the _d64 bodies) -- 256-row blocks of 4 waves x 64 rows, 64-key tiles, a
# 5-slot LDS ring two tiles ahead; only other head dims and Nk <= 64 fall
# back to attn_fwd_v12 / v10 / v7 (csrc/flash_v13.hip attn_v13_ok).  Non-causal
# D = 64 where B H ceil(Nq / 512) fills the CUs: attn_fwd_pp64 (512-row blocks
# of 8 waves, a 6-slot ring four tiles ahead; tools/v14/pp64.py)
HIP_TILING = {"block_q": 256, "block_k": 64, "num_warps": 4, "num_stages": 5}


def hip_tiling(config: "FlashAttentionConfig | None" = None) -> dict:
    """The HIP kernel's fixed tiling next to the requested config:
    {field: {"requested": value, "hip": value}} (the GPU path runs "hip")."""
    config = config or FlashAttentionConfig()
    _check_config(config)
    return {f: {"requested": getattr(config, f), "hip": v} for f, v in HIP_TILING.items()}


def _check_config(config) -> None:
    for f in ("block_q", "block_k", "num_warps", "num_stages"):
        v = getattr(config, f)
        if isinstance(v, bool) or not isinstance(v, int) or v <= 0:
            raise ValueError(f"FlashAttentionConfig.{f} must be a positive int, got {v!r}")


def _flash_cpu(q, k, v, scale, block_q, block_k, causal=False):
    B, H, N, D = q.shape
    Nk = k.shape[2]
    qf, kf, vf = q.float(), k.float(), v.float()
    out = torch.empty_like(qf)
    for qs in range(0, N, block_q):
        qe = min(qs + block_q, N)
        qb = qf[:, :, qs:qe]
        m = torch.full((B, H, qe - qs, 1), float("-inf"))
        den = torch.zeros((B, H, qe - qs, 1))
        acc = torch.zeros((B, H, qe - qs, D))
        for ks in range(0, Nk, block_k):
            ke = min(ks + block_k, Nk)
            s = torch.matmul(qb, kf[:, :, ks:ke].transpose(-2, -1)) * scale
            if causal:
                qi = torch.arange(qs, qe).view(-1, 1)
                kj = torch.arange(ks, ke).view(1, -1)
                s = s.masked_fill(kj > qi + (Nk - N), float("-inf"))
            m_new = torch.maximum(m, s.amax(dim=-1, keepdim=True))
            safe = torch.where(torch.isinf(m_new), torch.zeros_like(m_new), m_new)
            alpha = torch.exp(m - safe)
            p = torch.exp(s - safe)
            den = den * alpha + p.sum(dim=-1, keepdim=True)
            acc = acc * alpha + torch.matmul(p, vf[:, :, ks:ke])
            m = m_new
        out[:, :, qs:qe] = acc / den
    return out.to(q.dtype)


def flash_attention_forward(
    q: torch.Tensor,
    k: torch.Tensor,
    v: torch.Tensor,
    scale: float | None = None,
    config: FlashAttentionConfig | None = None,
) -> torch.Tensor:
    if config is None:
        config = FlashAttentionConfig()
    _check_config(config)
    B, H, N, D = q.shape
    if scale is None:
        scale = D ** -0.5
    if q.is_cuda:
        return pli_hip.flash_attn_fwd(q, k, v, scale=scale, causal=False)
    return _flash_cpu(q, k, v, scale, config.block_q, config.block_k)


def flash_attention_memory_bytes(
    batch_size: int,
    num_heads: int,
    seq_len: int,
    head_dim: int,
    block_size: int = 64,
    dtype_bytes: int = 2,
) -> dict:
    """HBM / on-chip byte model of ``ch06/flash_attention.py:77-104``.

    HBM = read Q, K, V + write O; the naive path additionally materialises
    the [B, H, N, N] score matrix.  On-chip bytes per tile are Q/K/V/O tiles
    of ``block_size x head_dim``, one score tile and two statistics rows.
    """
    tensor = batch_size * num_heads * seq_len * head_dim * dtype_bytes
    hbm = 4 * tensor
    tile = block_size * head_dim * dtype_bytes
    sram = 4 * tile + block_size * block_size * dtype_bytes + 2 * block_size * dtype_bytes
    scores = batch_size * num_heads * seq_len * seq_len * dtype_bytes
    return {
        "hbm_bytes": hbm,
        "hbm_mb": hbm / 1024 / 1024,
        "sram_bytes_per_block": sram,
        "sram_kb_per_block": sram / 1024,
        "naive_hbm_bytes": hbm + scores,
        "memory_savings": f"{seq_len // block_size}x",
    }


def explain_flash_attention() -> str:
    return (
        "FlashAttention on MI355X (attn_fwd_v13): one wave per SIMD keeps 64 query rows\n"
        "(Q^T and O^T in the accumulator file), K/V arrive by LDS-DMA in 64-key tiles two\n"
        "tiles ahead, S^T = K Q^T and O^T += V^T P^T run on v_mfma_f32_16x16x32 (bf16 or\n"
        "f16; head dim 128 or 64), P = exp2(s c - mu) goes from the scores straight into\n"
        "the PV operand, the row sums l run on the matrix core and a tile takes the\n"
        "rescale path only when some row's l reaches 1 (defer-max).  HBM traffic is\n"
        "O(N d): Q, K, V read once per head, O written once."
    )


def _demo() -> None:
    """`python -m ch06.flash_attention`: the chapter's demo on this build --
    the explanation, a check of the fused kernel against the materialised
    attention on the chapter's fp16 head-dim-64 shape, and the HBM byte model
    over sequence lengths (the reference module's __main__, ch06/
    flash_attention.py:143-177)"""
    from .attention_memory import naive_attention

    print(explain_flash_attention())
    if not torch.cuda.is_available():
        print("\nno ROCm device: the kernel check is skipped")
    else:
        print("\n" + "=" * 60 + "\nCorrectness Verification\n" + "-" * 60)
        shape = (2, 8, 256, 64)
        q, k, v = (torch.randn(*shape, device="cuda", dtype=torch.float16) for _ in range(3))
        diff = (naive_attention(q, k, v) - flash_attention_forward(q, k, v)).abs().max().item()
        print(f"Max difference: {diff:.6f} (kernel {pli_hip.last_route()})")
        print(f"Correctness: {'PASS' if diff < 0.01 else 'FAIL'}")
    print("\n" + "=" * 60 + "\nMemory Analysis\n" + "-" * 60)
    for n in (512, 1024, 2048, 4096, 8192):
        m = flash_attention_memory_bytes(batch_size=1, num_heads=32, seq_len=n, head_dim=64)
        print(f"Seq {n:5d}: Flash HBM={m['hbm_mb']:.1f} MB, Naive HBM={m['naive_hbm_bytes'] / 2**20:.1f} MB, "
              f"Savings={m['memory_savings']}")


if __name__ == "__main__":
    _demo()
