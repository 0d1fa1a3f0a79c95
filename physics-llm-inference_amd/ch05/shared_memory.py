"""Shared memory (LDS) and tiling -- mirror of ``ch05/shared_memory.py``.

Same functions, dataclass and return shapes as the reference
(``ch05/shared_memory.py:6-104``).  The MI355X facts differ from the CUDA
numbers the reference prints: a CU has 160 KiB of LDS (the default of
``max_blocks_by_shared_memory``), and LDS banking is per instruction --
32 four-byte banks per 32-lane half-wave for ``ds_read_b32`` (the pattern
the reference's bank formula describes), 64 banks for the 8- and 16-byte
reads (MI355X_MICROARCH.md "LDS").  ``tiled_reduce`` keeps the reference's
torch formulation (it is a host-side illustration, no kernel of its own).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

MI355X_LDS_PER_CU = 160 * 1024


@dataclass
class TileConfig:
    tile_size: int
    num_tiles: int
    shared_memory_bytes: int


def compute_tile_config(n: int, tile_size: int = 32) -> TileConfig:
    """Tiles of ``tile_size`` fp32 elements covering ``n`` (ceil), and the LDS
    bytes one tile takes."""
    return TileConfig(tile_size=tile_size, num_tiles=(n + tile_size - 1) // tile_size,
                      shared_memory_bytes=tile_size * 4)


def tiled_reduce(data: torch.Tensor, tile_size: int = 256) -> torch.Tensor:
    """Sum of a 1-D tensor as per-tile partial sums, then the sum of those
    (the two-level order a tiled reduction kernel uses)."""
    n = data.shape[0]
    parts = [data[s:min(s + tile_size, n)].sum() for s in range(0, n, tile_size)]
    return torch.stack(parts).sum()


def demonstrate_bank_conflicts() -> dict:
    return {
        "shared_memory_banks": 32,
        "bank_width_bytes": 4,
        "conflict_free_pattern": "consecutive lanes access consecutive 4-byte words",
        "conflict_pattern": "lanes of one 32-lane group access different addresses in the same bank",
        "bank_formula": "bank = (address / 4) % 32",
        "mi355x_wide_reads": "ds_read_b64 / ds_read_b128 / ds_read_b64_tr_b16: 64 banks, "
                             "bank = (address / 4) % 64, lane groups of 32 / 16",
        "lds_per_cu_bytes": MI355X_LDS_PER_CU,
    }


def explain_shared_memory() -> str:
    return """
LDS (shared memory) on MI355X

LDS is on-chip memory shared by the waves of one workgroup: 160 KiB per CU,
up to 256 bytes per clock.  Banking is per instruction: ds_read_b32 serves
each 32-lane half-wave through 32 four-byte banks, the 8- and 16-byte reads
through 64 banks; lanes of one group that hit the same bank at different
addresses serialise.

Tiled matrix multiplication (the ch05 HIP GEMM):
- stage tiles of A and B in LDS (here by LDS-DMA, swizzled on the source address)
- s_barrier, then every wave reads its MFMA fragments from LDS
- each HBM byte is re-used tile_size times from LDS instead of HBM
"""


def shared_memory_requirements(threads_per_block: int, elements_per_thread: int,
                               dtype_bytes: int = 4) -> int:
    return threads_per_block * elements_per_thread * dtype_bytes


def max_blocks_by_shared_memory(shared_per_block: int, shared_per_sm: int = MI355X_LDS_PER_CU):
    """Workgroups per CU that the LDS alone admits (inf when none is used)."""
    if shared_per_block == 0:
        return float("inf")
    return shared_per_sm // shared_per_block


if __name__ == "__main__":
    # the chapter's demo (ch05/shared_memory.py)
    print(explain_shared_memory())
    print("\nBank Conflict Info:")
    for key, val in demonstrate_bank_conflicts().items():
        print(f"  {key}: {val}")
    cfg = compute_tile_config(n=1024, tile_size=32)
    print(f"\nTile Configuration Example:\n  Tiles: {cfg.num_tiles}\n  Shared memory: {cfg.shared_memory_bytes} bytes")
    print("\nShared Memory Occupancy Impact:")
    for kib in (0, 16, 32, 48):
        blocks = max_blocks_by_shared_memory(kib * 1024)
        print(f"  {kib:3d} KB -> " + ("unlimited blocks" if blocks == float("inf") else f"{blocks} blocks/CU"))
