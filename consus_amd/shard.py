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

One record too large for one GPU (or simply large enough to amortise a
launch per GPU) is split the other way: record_slices cuts its bytes into
one slice per rank, each rank computes crc32c(0, slice) where the slice
lives, and fold_slice_crcs chains the (crc, length) pairs -- 8 bytes per
rank -- into crc32c(init, record) with the same combine operator
("gather 8 x (crc, len) pairs and fold them").
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


def record_slices(nbytes: int, world: int, align: int = 4096) -> list[tuple[int, int]]:
    """(start, length) of each rank's slice of one nbytes-long record.

    Equal shares rounded down to a multiple of `align` (so every interior
    cut is chunk-aligned relative to the record start); the last rank takes
    the remainder.  Slices may be empty when nbytes < world * align.
    """
    if world < 1 or align < 1:
        raise ValueError("world and align must be >= 1")
    share = (nbytes // world) // align * align
    out, start = [], 0
    for r in range(world):
        length = share if r < world - 1 else nbytes - start
        out.append((start, length))
        start += length
    return out


def fold_slice_crcs(crcs: Sequence[int], lengths: Sequence[int], init: int = 0) -> int:
    """crc32c(init, S_0 || S_1 || ...) from crcs[i] = crc32c(0, S_i).

    init behaves as the CRC of a virtual prefix, so the fold starts from it:
    acc = combine(acc, crc_i, |S_i|) left to right; empty slices are skipped
    (crc32c(0, "") = 0 and combine by 0 bytes is the identity anyway).
    """
    from . import combine
    acc = init & 0xFFFFFFFF
    for c, n in zip(crcs, lengths):
        if n:
            acc = combine(acc, int(c), int(n))
    return acc


def gather_fold(local_crc: int, local_len: int, init: int = 0, group=None) -> int | None:
    """All-gather every rank's (crc32c(0, slice), slice length) over the
    torch.distributed control plane and fold them on rank 0 (None elsewhere).
    Ranks must hold their slices in rank order."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    got = [None] * world
    dist.all_gather_object(got, (int(local_crc), int(local_len)), group=group)
    if dist.get_rank(group) != 0:
        return None
    return fold_slice_crcs([g[0] for g in got], [g[1] for g in got], init)
