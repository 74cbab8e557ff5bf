"""Record sharding across the GPUs of one node.

Every record's CRC is independent, so a batch is split into contiguous record
ranges, one per rank, balanced by BYTES (not record count: Zipf lengths), and
each rank hashes its own range where it already lives (generated in place or
H2D'd over its own PCIe link).  No data moves between GPUs.  Results are
reduced to a per-rank digest -- crc32c(0, LE bytes of the rank's CRC vector)
-- and the global digest is recovered from the per-rank digests with the
CRC combine identity crc(A||B) = Z_|B|(crc(A)) ^ crc(B), so verifying a
sharded run moves 4 bytes per rank.  An RCCL all-gather of the full CRC
vectors (mi_comm_allgather_u32) is available for callers that need them.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def balanced_ranges(lengths: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) record ranges, one per rank, with ~equal byte sums.

    Rank r's range ends at the first record whose inclusive prefix sum reaches
    (r + 1) / world of the total; empty ranges are allowed when there are
    fewer records than ranks.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    n = int(len(lengths))
    if n == 0:
        return [(0, 0)] * world
    pref = np.cumsum(np.asarray(lengths, dtype=np.uint64), dtype=np.uint64)
    total = int(pref[-1])
    bounds = [0]
    for r in range(1, world):
        target = (total * r + world - 1) // world
        cut = int(np.searchsorted(pref, target, side="left")) + 1
        bounds.append(min(max(cut, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def equal_ranges(count: int, world: int) -> list[tuple[int, int]]:
    """Fixed-length records: equal record counts per rank."""
    return [(count * r // world, count * (r + 1) // world) for r in range(world)]


def combine_digests(digests: Sequence[int], counts: Sequence[int]) -> int:
    """Digest of the concatenated CRC vectors from per-shard digests.

    digest(A || B) = combine(digest(A), digest(B), 4 * |B|).  An empty shard
    contributes nothing.  Pure operator algebra (mi_crc32c_combine).
    """
    from . import combine
    acc = None
    for d, c in zip(digests, counts):
        if c == 0:
            continue
        acc = d if acc is None else combine(acc, d, 4 * int(c))
    return 0 if acc is None else acc
