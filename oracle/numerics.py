"""Seeded inputs and low-precision rounding, in numpy (test infrastructure only).

Inputs for every parity test are ``np.random.RandomState(seed).standard_normal``
(the numpy legacy stream is stable across numpy versions) cast to float32 and
then rounded to the compute dtype.  The reference draws its inputs with
``torch.randn`` (e.g. ``ch06/test_ch06.py:161-164``); a fixed, portable stream is
used instead so the golden fixtures are reproducible without the reference.
"""
from __future__ import annotations

import hashlib

import numpy as np


def round_to_bf16(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest-even bfloat16, returned as float32 values.

    Same rounding as ``torch.Tensor.to(torch.bfloat16)`` (RNE on the f32 bits);
    NaN stays NaN.
    """
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    rounded = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = rounded.astype(np.uint32).view(np.float32)
    return np.where(np.isnan(x), x, out).astype(np.float32)


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """bfloat16-representable float32 values -> their uint16 bit patterns."""
    x = np.ascontiguousarray(round_to_bf16(x), dtype=np.float32)
    return (x.view(np.uint32) >> 16).astype(np.uint16)


def bf16_from_bits(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def round_to_dtype(x: np.ndarray, dtype: str) -> np.ndarray:
    """Round float32 values to ``dtype`` in {"fp32","fp16","bf16"}; float32 out."""
    x = np.asarray(x, dtype=np.float32)
    if dtype == "fp32":
        return x.copy()
    if dtype == "fp16":
        return x.astype(np.float16).astype(np.float32)
    if dtype == "bf16":
        return round_to_bf16(x)
    raise ValueError(f"unknown dtype {dtype!r}")


def seeded_normal(shape, seed: int, dtype: str = "fp32") -> np.ndarray:
    """N(0,1) float32 draws from RandomState(seed), rounded to ``dtype``."""
    rs = np.random.RandomState(seed)
    x = rs.standard_normal(size=shape).astype(np.float32)
    return round_to_dtype(x, dtype)


def array_hash(x: np.ndarray) -> str:
    """Short sha256 of the float32 bytes (pins fixture inputs)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    return hashlib.sha256(x.tobytes()).hexdigest()[:16]
