"""Adversarial flash-attention inputs shared by the GPU tests and
tests/golden/make_stress.py (which records the reference's own bf16 output on
them).  Inputs come from np.random.RandomState and are bf16-rounded, so both
sides rebuild them bit for bit.

* ``spike``  -- one key row aligned with query row 3, so row 3's max jumps past
  the defer threshold in a late tile (the rescale branch) and a few other rows
  put a large share of their weight on that key;
* ``first``  -- every score negative and ~ -166 (log2 units) in the first
  tile, lower after it: exp2 of a score against a zero max underflows, so the
  first tile must set the running max;
* ``late``   -- two late keys raise the max of rows 10 and 300 by 39-65 log2
  units in tiles 3 and 9;
* ``all``    -- Q scaled by 6: |scores| ~ 9 log2 units, the rescale branch in
  many tiles.
* ``seam2`` / ``seam5`` -- GQA 40/8 (72/8) heads, Q scaled by 4 (peaky rows,
  the rescale branch in several tiles), shaped so that the persistent flash
  kernel (variant 71) walks more than one block per workgroup with blocks
  of 2 (5) key tiles: its K/V stream crosses block seams, and N = 320 gives
  a ragged last query block.  The reference flash has no GQA: its fixture
  entry is computed on K/V repeated to the query heads (the same math).
"""
from __future__ import annotations

import numpy as np

from oracle.numerics import round_to_bf16, seeded_normal

STRESS = ("spike", "first", "late", "all", "seam2", "seam5")


def stress_inputs(name: str):
    if name in ("seam2", "seam5"):
        B, H, Hkv, N = (4, 72, 8, 128) if name == "seam2" else (4, 40, 8, 320)
        seed = 21 if name == "seam2" else 25
        q = seeded_normal((B, H, N, 128), seed, "bf16") * np.float32(4.0)  # exact in bf16
        k = seeded_normal((B, Hkv, N, 128), seed + 1, "bf16")
        v = seeded_normal((B, Hkv, N, 128), seed + 2, "bf16")
        return q, k, v
    if name == "spike":
        B, H, N, D = 1, 2, 512, 128
        q = seeded_normal((B, H, N, D), 7, "bf16")
        k = seeded_normal((B, H, N, D), 8, "bf16")
        v = seeded_normal((B, H, N, D), 9, "bf16")
        k[:, :, 450] = np.float32(4.0) * np.sign(q[:, :, 3])  # row 3 jumps at tile 7
        return q, round_to_bf16(k), v
    B, H, N, D = 1, 4, 640, 128
    rng = np.random.RandomState({"first": 11, "late": 12, "all": 13}[name])
    q = rng.standard_normal((B, H, N, D)).astype(np.float32)
    k = rng.standard_normal((B, H, N, D)).astype(np.float32)
    v = rng.standard_normal((B, H, N, D)).astype(np.float32)
    if name == "first":
        sgn = np.sign(q[:, :, :1])
        q = np.abs(q) * sgn
        k[:, :, :64] = -16.0 * sgn * np.abs(k[:, :, :64])
        k[:, :, 64:] = -20.0 * sgn * np.abs(k[:, :, 64:])
    elif name == "late":
        k[:, :, 600] = 5.0 * np.sign(q[:, :, 10])
        k[:, :, 200] = 3.0 * np.sign(q[:, :, 300])
    elif name == "all":
        q *= 6.0
    return tuple(round_to_bf16(t) for t in (q, k, v))


def prescaled_q(q: np.ndarray, scale: float) -> np.ndarray:
    """The Q the prescaled kernel (variant 50) effectively uses, as float64:
    q*c rounded to bf16 (c = scale*log2(e) in f32, as on the device), divided
    back by c, so that softmax(q_eff k^T scale) = softmax over exp2(round(q c) k)."""
    c = np.float32(scale) * np.float32(1.4426950408889634)
    return round_to_bf16((q.astype(np.float32) * c).astype(np.float32)).astype(np.float64) / float(c)
