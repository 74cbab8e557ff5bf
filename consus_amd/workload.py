"""Synthetic record batches of BASELINE.json configs 3 and 5.

Config 3: 1M records, lengths mi_workload_zipf_lengths(0x5EED) (64 B - 64 KiB,
Zipf 1.2), packed back to back from offset 0 of the splitmix64 stream
0xDA7A5EED.

Config 5: 64 MiB durable-log segments.  Frame i (i = 0, 1, ...) is
[recno = i + 1 as u64 BE][len as u64 BE][entry][4-byte CRC slot], the entry
being the next `len` bytes of the stream 0xDA7A5EED and `len` the i-th
config-3 length; frames fill a segment greedily until the next one does not
fit (txman/durable_log.cc:54-61, 195-224 framing).  The CRC of a frame covers
header || entry (= crc32c(crc32c(0, header, 16), entry), :215-218).
"""
from __future__ import annotations

from typing import Callable, Iterator

import numpy as np

ZIPF_SEED = 0x5EED
DATA_SEED = 0xDA7A5EED
SEGMENT_BYTES = 64 << 20


def zipf_records(count: int, first: int = 0):
    """(offsets u64, lengths u32, total bytes) of config-3 records [first, first+count)."""
    from . import zipf_lengths
    lengths = zipf_lengths(ZIPF_SEED, count, first=first)
    offsets = np.zeros(count, dtype=np.uint64)
    if count:
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    return offsets, lengths, int(lengths.sum(dtype=np.uint64))


def log_segments(nseg: int, fill: Callable[[int, int], np.ndarray],
                 seg_bytes: int = SEGMENT_BYTES) -> Iterator[tuple]:
    """Yield nseg config-5 segments as (buf u8, frame offsets u64, covered lengths u32).

    fill(nbytes, byte_offset) returns bytes [byte_offset, +nbytes) of the
    stream DATA_SEED (device fill + download in bench.py, the oracle in the
    golden generator).
    """
    from . import zipf_lengths
    rec = 0          # next frame index
    data_pos = 0     # next entry byte in the stream
    batch = np.zeros(0, dtype=np.uint32)
    batch_first = 0
    for _ in range(nseg):
        sizes = []
        used = 0
        while True:
            if rec - batch_first >= batch.size:
                batch_first = rec
                batch = zipf_lengths(ZIPF_SEED, 65536, first=rec)
            n = int(batch[rec - batch_first])
            if used + 20 + n > seg_bytes:
                break
            sizes.append(n)
            used += 20 + n
            rec += 1
        lens = np.array(sizes, dtype=np.uint64)
        frame_off = np.zeros(lens.size, dtype=np.uint64)
        if lens.size:
            frame_off[1:] = np.cumsum(lens[:-1] + 20, dtype=np.uint64)
        payload = fill(int(lens.sum()), data_pos)
        buf = np.zeros(used, dtype=np.uint8)
        first_recno = rec - lens.size + 1
        hdr = np.zeros((lens.size, 2), dtype=">u8")
        hdr[:, 0] = np.arange(first_recno, first_recno + lens.size, dtype=np.uint64)
        hdr[:, 1] = lens
        hdr_b = hdr.view(np.uint8).reshape(-1, 16)
        src = 0
        for i in range(lens.size):
            o = int(frame_off[i])
            n = int(lens[i])
            buf[o:o + 16] = hdr_b[i]
            buf[o + 16:o + 16 + n] = payload[src:src + n]
            src += n
        data_pos += src
        yield buf, frame_off, (lens + 16).astype(np.uint32)
