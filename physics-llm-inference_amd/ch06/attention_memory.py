"""Attention memory/FLOP models and the materialised oracle (mirror of
``ch06/attention_memory.py``).

``naive_attention`` is the reference's own checker: softmax(QK^T*scale)V with
the [B,H,N,N] score matrix materialised.  It stays a plain torch computation
on every device on purpose -- it is the independent baseline the HIP flash
kernel is compared with (``ch06/test_ch06.py:169-189``), so routing it through
the same kernel would make that test vacuous.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class AttentionMemoryStats:
    batch_size: int
    num_heads: int
    seq_len: int
    head_dim: int
    qk_bytes: int
    softmax_bytes: int
    output_bytes: int
    total_bytes: int
    total_mb: float


def naive_attention(q, k, v, scale: float | None = None) -> torch.Tensor:
    """``ch06/attention_memory.py:19-33``: materialised scores, softmax over keys."""
    D = q.shape[-1]
    if scale is None:
        scale = D ** -0.5
    scores = torch.matmul(q, k.transpose(-2, -1)) * scale
    return torch.matmul(torch.softmax(scores, dim=-1), v)


def attention_memory_bytes(batch_size, num_heads, seq_len, head_dim, dtype_bytes=2):
    """Bytes of the naive path: the N x N scores written, the softmax output
    written, and the [B,H,N,D] output (``:36-59`` of the reference)."""
    square = batch_size * num_heads * seq_len * seq_len * dtype_bytes
    out = batch_size * num_heads * seq_len * head_dim * dtype_bytes
    total = 2 * square + out
    return AttentionMemoryStats(batch_size, num_heads, seq_len, head_dim,
                                qk_bytes=square, softmax_bytes=square, output_bytes=out,
                                total_bytes=total, total_mb=total / 1024 / 1024)


def attention_flops(batch_size, num_heads, seq_len, head_dim) -> int:
    """QK^T and PV (2*B*H*N^2*D each) plus 5 FLOPs per score for the softmax."""
    n2 = batch_size * num_heads * seq_len * seq_len
    return 4 * n2 * head_dim + 5 * n2


def attention_arithmetic_intensity(seq_len, head_dim) -> float:
    """FLOP per byte of the naive path per head (2-byte elements)."""
    n2 = seq_len * seq_len
    return (4 * n2 * head_dim + 5 * n2) / (4 * n2 + 6 * seq_len * head_dim)


def explain_attention_bottleneck() -> str:
    return ("Naive attention writes and re-reads the N x N score matrix: O(N^2) HBM traffic.\n"
            "FlashAttention keeps score tiles on chip (registers/LDS): O(N d) traffic.")


@torch.no_grad()
def benchmark_attention_memory(seq_lens=None, head_dim=64, num_heads=32, batch_size=1,
                               device="cuda") -> dict:
    """Peak device memory of the naive path vs the byte model (``:90-133``)."""
    if seq_lens is None:
        seq_lens = [512, 1024, 2048, 4096, 8192]
    results = {}
    for n in seq_lens:
        try:
            torch.cuda.reset_peak_memory_stats()
            q, k, v = (torch.randn(batch_size, num_heads, n, head_dim, device=device,
                                   dtype=torch.float16) for _ in range(3))
            naive_attention(q, k, v)
            torch.cuda.synchronize()
            model = attention_memory_bytes(batch_size, num_heads, n, head_dim, 2)
            results[n] = {"theoretical_mb": model.total_mb,
                          "actual_mb": torch.cuda.max_memory_allocated() / 1024 / 1024,
                          "qk_matrix_mb": model.qk_bytes / 1024 / 1024}
            del q, k, v
            torch.cuda.empty_cache()
        except torch.cuda.OutOfMemoryError:
            results[n] = {"oom": True}
            torch.cuda.empty_cache()
    return results


if __name__ == "__main__":
    # the chapter's demo (ch06/attention_memory.py:127-156): the score matrix's
    # bytes and arithmetic intensity by sequence length, then (on a device)
    # measured allocations of the materialised attention
    print(explain_attention_bottleneck())
    print("\n" + "=" * 60 + "\nMemory Scaling by Sequence Length\n" + "-" * 60)
    for n in (512, 1024, 2048, 4096, 8192, 16384, 32768):
        st = attention_memory_bytes(batch_size=1, num_heads=32, seq_len=n, head_dim=64, dtype_bytes=2)
        print(f"Seq {n:6d}: {st.total_mb:8.1f} MB, AI={attention_arithmetic_intensity(n, 64):.2f} FLOP/byte")
    if torch.cuda.is_available():
        print("\n" + "=" * 60 + "\nActual Memory Usage (GPU)\n" + "-" * 60)
        for n, d in benchmark_attention_memory().items():
            print(f"Seq {n}: OOM" if "oom" in d else
                  f"Seq {n}: theoretical={d['theoretical_mb']:.1f} MB, actual={d['actual_mb']:.1f} MB")
