"""Seeded random batches against the oracle (bit-exact), through every
variable-length entry point: host batches on the direct kernel and on the
planned path, device batches with and without the size hint, fixed-stride
batches (also split over 2-5 ranges through the multi-device entry
points), the sorted path at random grids, the window path at random
workgroups and windows, the direct kernel's two forms
and its zero-copy read from pinned memory, and single buffers (host and
device).  Shapes mix empty, tiny,
row- and chunk-edge, and multi-chunk records; offsets packed, random,
overlapping and unordered; inits random or absent.

FUZZ_ROUNDS (environment) raises the number of rounds for longer soaks.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROUNDS = int(os.environ.get("FUZZ_ROUNDS", "24"))


def random_lengths(rng, count):
    kind = rng.integers(0, 5)
    if kind == 0:
        return rng.integers(0, 40, count)
    if kind == 1:
        return rng.integers(0, 5000, count)
    if kind == 2:  # around row / group / chunk edges
        edges = np.array([127, 128, 129, 1023, 1024, 1025, 4095, 4096, 4097, 8192])
        return edges[rng.integers(0, edges.size, count)] + rng.integers(-2, 3, count)
    if kind == 3:
        return rng.integers(0, 70000, count)
    return np.minimum(rng.zipf(1.3, count) * 64, 300000)


@pytest.mark.parametrize("round_", range(ROUNDS))
def test_fuzz_round(engine, oracle, round_):
    rng = np.random.default_rng(9000 + round_)
    count = int(rng.integers(1, 3000))
    lengths = np.clip(random_lengths(rng, count), 0, None).astype(np.uint32)
    layout = rng.integers(0, 3)
    if layout == 0:  # packed back to back from a random start
        offsets = np.zeros(count, dtype=np.uint64)
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
        offsets += np.uint64(rng.integers(0, 4096))
        size = int(offsets[-1] + lengths[-1]) + 64
    else:  # random, possibly overlapping, unordered
        size = int(lengths.max()) + int(rng.integers(1, 1 << 20))
        offsets = np.array([rng.integers(0, size - int(L) + 1) for L in lengths], dtype=np.uint64)
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32) if rng.integers(0, 2) else None
    want = oracle.batch(buf, offsets, lengths, inits)

    # host batches: direct kernel when every record is short, and the planned path
    for planned in (False, True):
        got = engine.crc32c_batch(buf, offsets, lengths, inits, planned=planned)
        assert np.array_equal(got, want), ("host", planned)
    # the direct kernel's LDS image and LDS-free forms, and the same bytes read
    # in place from mapped pinned memory (the durable log's flush path)
    if int(lengths.max()) <= 16384:
        try:
            for lite in ("0", "1"):
                os.environ["MI_CRC32C_DIRECT_LITE"] = lite
                got = engine.crc32c_batch(buf, offsets, lengths, inits)
                assert np.array_equal(got, want), ("direct", lite)
        finally:
            os.environ.pop("MI_CRC32C_DIRECT_LITE", None)
        pinned = engine.PinnedBuffer(size)
        try:
            pinned.array[:] = buf
            got = engine.crc32c_batch(pinned.array, offsets, lengths, inits)
            assert np.array_equal(got, want), "zero-copy"
        finally:
            pinned.free()
    # the multi-device entry point, split into 2-5 byte-balanced ranges on the one GPU
    ndev = int(rng.integers(2, 6))
    got = engine.crc32c_batch_multi(buf, offsets, lengths, inits, devices=[0] * ndev, shard_min=1)
    assert np.array_equal(got, want), ("multi", ndev)

    # device batch, with the size hint and without it (plan read-back)
    data = engine.DeviceBuffer(size)
    data.upload(buf)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    d_ini = None
    if inits is not None:
        d_ini = engine.DeviceBuffer(count * 4)
        d_ini.upload(inits)
    for hint in (int(lengths.sum(dtype=np.uint64)), 0):
        engine.device_batch(data, d_off, d_len, count, d_out, inits=d_ini, total_bytes=hint)
        assert np.array_equal(d_out.download(np.uint32, count), want), ("device", hint)

    # the sorted path again (the hinted call above took it with its batch-sized
    # piece), one workgroup per CU or a few workgroups (shares cut inside
    # records), at a random piece size (512 B - 64 KiB)
    grid = [None, "1", "2", "5", "64"][int(rng.integers(0, 5))]
    plog = [None, "9", "10", "12", "13", "14", "15", "16"][int(rng.integers(0, 8))]
    ring = [None, "2", "4"][int(rng.integers(0, 3))]
    lanes = [None, "0", "1", "3"][int(rng.integers(0, 4))]  # rows of a lane item (default 2)
    os.environ["MI_CRC32C_VARPATH"] = "sorted"
    if lanes:
        os.environ["MI_CRC32C_SORT_LANE_ROWS"] = lanes
    if ring:
        os.environ["MI_CRC32C_SORT_RING"] = ring
    if grid:
        os.environ["MI_CRC32C_SORTED_GRID"] = grid
    if plog:
        os.environ["MI_CRC32C_SORT_PIECE_LOG2"] = plog
    try:
        before = engine.stats()["sorted_batches"]
        engine.device_batch(data, d_off, d_len, count, d_out, inits=d_ini,
                            total_bytes=max(int(lengths.sum(dtype=np.uint64)), 1))
        assert np.array_equal(d_out.download(np.uint32, count), want), ("sorted", grid, plog, ring, lanes)
        assert engine.stats()["sorted_batches"] == before + 1
    finally:
        os.environ.pop("MI_CRC32C_VARPATH", None)
        os.environ.pop("MI_CRC32C_SORTED_GRID", None)
        os.environ.pop("MI_CRC32C_SORT_PIECE_LOG2", None)
        os.environ.pop("MI_CRC32C_SORT_RING", None)
        os.environ.pop("MI_CRC32C_SORT_LANE_ROWS", None)

    # the window path forced (count < 3000 is inside its record bound), at a
    # random workgroup (one wave, four, one twelve-wave workgroup per CU) and
    # window (4 / 8 / 16 rows), with the hint or an understated one (looping)
    block = [None, "64", "256", "768"][int(rng.integers(0, 4))]
    rows = [None, "4", "8", "16"][int(rng.integers(0, 4))]
    os.environ["MI_CRC32C_VARPATH"] = "window"
    if block:
        os.environ["MI_CRC32C_WIN_BLOCK"] = block
    if rows:
        os.environ["MI_CRC32C_WIN_ROWS"] = rows
    try:
        before = engine.stats()["window_batches"]
        hint = max(int(lengths.sum(dtype=np.uint64)), 1) if rng.integers(0, 4) else 1
        d_out.upload(np.full(count, 0xABABABAB, dtype=np.uint32))
        engine.device_batch(data, d_off, d_len, count, d_out, inits=d_ini, total_bytes=hint)
        assert np.array_equal(d_out.download(np.uint32, count), want), ("window", block, rows, hint)
        assert engine.stats()["window_batches"] == before + 1
    finally:
        os.environ.pop("MI_CRC32C_VARPATH", None)
        os.environ.pop("MI_CRC32C_WIN_BLOCK", None)
        os.environ.pop("MI_CRC32C_WIN_ROWS", None)

    # single buffers: one record on the host and on the device
    i = int(rng.integers(0, count))
    o, L = int(offsets[i]), int(lengths[i])
    init = int(inits[i]) if inits is not None else 0
    assert engine.crc32c(init, buf[o:o + L]) == int(want[i])
    assert engine.crc32c_device(data, L, init_crc=init, offset=o) == int(want[i])

    # a fixed-stride batch over the same bytes
    stride = int(rng.integers(1, 5000))
    flen = min(int(rng.integers(0, stride + 1)), size)  # the buffer may be shorter
    fcount = max(1, min(500, (size - flen) // stride))
    fini = rng.integers(0, 2**32, fcount, dtype=np.uint32) if rng.integers(0, 2) else None
    fwant = oracle.fixed(buf, stride, flen, fcount, inits=fini)
    assert np.array_equal(engine.crc32c_fixed(buf, stride, flen, fcount, inits=fini), fwant), (stride, flen)
    assert np.array_equal(engine.crc32c_fixed_multi(buf, stride, flen, fcount, inits=fini,
                                                    devices=[0] * ndev, shard_min=1), fwant), ("fixed multi", ndev)
    for b in (data, d_off, d_len, d_out) + ((d_ini,) if d_ini is not None else ()):
        b.free()
