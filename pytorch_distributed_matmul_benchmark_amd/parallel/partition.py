"""Work partitioning for the scaling modes (pure functions, CPU-testable).

Reference behaviour and the fixes made here:
  * batch_parallel splits a fixed global batch of 4 as ``4 // ws``
    (matmul_scaling_benchmark.py:111,283), so ws=8 gets an EMPTY batch and
    ws=3 silently does 3 batches while reporting 4 (Q3). ``global_batch``
    keeps 4 as the default but rounds it up to a multiple of ws, so every
    rank gets ``global_batch // ws ≥ 1`` GEMMs and the reported FLOPs are the
    FLOPs actually done.
  * matrix_parallel gives the remainder columns to the last rank
    (matmul_scaling_benchmark.py:179-183), which breaks the equal-size
    all_gather (Q4). ``column_shard`` pads every shard to the same width
    ``ceil(N / ws)`` (rounded up to ``align``) and reports the valid width,
    so the all-gather is always uniform and the padding is trimmed after.
"""
from __future__ import annotations

from dataclasses import dataclass


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


def round_up(a: int, b: int) -> int:
    return ceil_div(a, b) * b


def global_batch(ws: int, requested: int = 4) -> int:
    """Smallest multiple of ``ws`` that is ≥ ``requested`` (and ≥ ws)."""
    if ws < 1:
        raise ValueError("world size must be ≥ 1")
    return max(round_up(max(requested, 1), ws), ws)


def local_batch(ws: int, requested: int = 4) -> int:
    return global_batch(ws, requested) // ws


@dataclass(frozen=True)
class Shard:
    start: int   # first global column owned by this rank
    width: int   # number of VALID columns (may be < padded for the last rank(s))
    padded: int  # uniform shard width used for allocation and the all-gather

    @property
    def stop(self) -> int:
        return self.start + self.width


def column_shard(n: int, ws: int, rank: int, align: int = 1) -> Shard:
    """Column block of an N-wide matrix owned by ``rank`` in a ws-way 1-D split."""
    if not 0 <= rank < ws:
        raise ValueError(f"rank {rank} outside world of {ws}")
    padded = round_up(ceil_div(n, ws), align)
    start = min(rank * padded, n)
    width = max(0, min(n, start + padded) - start)
    return Shard(start=start, width=width, padded=padded)


def row_chunks(m: int, chunks: int, align: int = 256) -> list:
    """Split ``m`` rows into ≤ ``chunks`` contiguous [start, stop) ranges whose
    boundaries sit on multiples of ``align`` (so every chunk but the last is
    a whole number of 256-row GEMM tiles)."""
    chunks = max(1, int(chunks))
    step = round_up(ceil_div(m, chunks), align)
    out = []
    s = 0
    while s < m:
        e = min(m, s + step)
        out.append((s, e))
        s = e
    return out or [(0, 0)]
